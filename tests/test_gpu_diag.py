"""GPU parity of the anti-diagonal score-only fill (fill_diag_kernel) at every
columns-per-lane width it is built for, forced through GA_FILL_MODE=diag and
GA_DIAG_COLS_PER_LANE on a fresh context: the cost against the CPU oracle on shapes with a
partial last stripe (n not a multiple of 64*TD, n < 64*TD), chains of several workgroups,
rows shorter than the stripe skew, an int16 profile and host-supplied boundary triples."""
import numpy as np
import pytest

from tests.conftest import splitmix_seq, set_knob, del_knob

pytestmark = pytest.mark.gpu

SCORING = dict(match_score=2, mismatch_score=-3, gap_open_score=-5, gap_extension_score=-1)


def _engine(monkeypatch, td):
    from globalign_amd import _native
    set_knob(monkeypatch, "GA_FILL_MODE", "diag")
    set_knob(monkeypatch, "GA_DIAG_COLS_PER_LANE", str(td))
    return _native.Engine(0)


def _oracle_cost(s1, s2, cmat, goc, row0=None, col0=None):
    from oracle import core
    tab = core.Tables(cmat)
    a, b = tab.codes(s1), tab.codes(s2)
    if row0 is None:
        big = (tab.max_cost + 1) * max(len(s1), len(s2))
        row0, col0 = core.boundary(tab, a, b, goc, big)
    return int(min(core.fill_score(tab, a, b, goc, row0, col0)))


def _fill(monkeypatch, td, s1, s2, kw, **load_kw):
    from globalign_amd._native import CostTables
    from globalign_amd.scoring import validate_and_transform_args
    _, _, _, cmat, _, goc, _ = validate_and_transform_args(None, None, s1[:64], s2[:64], **kw)
    tables = CostTables(cmat, goc)
    eng = _engine(monkeypatch, td)
    try:
        eng.load(tables.codes(s1), tables.codes(s2), tables, **load_kw)
        return int(eng.fill(traceback=False)[0]), cmat, goc
    finally:
        eng.close()


@pytest.mark.parametrize("td", [1, 2, 4])
@pytest.mark.parametrize("m,n", [(5, 130), (17, 513), (31, 64), (300, 2049), (2049, 1023), (1000, 5000),
                                 (130, 8 * 256 + 3), (3000, 300)])
def test_diag_cost_vs_oracle(monkeypatch, td, m, n):
    seed = 11 * m + n + td
    s1, s2 = splitmix_seq(m, seed, "dna"), splitmix_seq(n, seed + 1, "dna")
    got, cmat, goc = _fill(monkeypatch, td, s1, s2, SCORING)
    assert got == _oracle_cost(s1, s2, cmat, goc)


@pytest.mark.parametrize("td", [1, 2, 4])
def test_diag_wide_gap_int16_profile(monkeypatch, td):
    """Substitution costs past int8 (mismatch -300): the int16 query profile."""
    s1, s2 = splitmix_seq(900, 5, "dna"), splitmix_seq(1700, 6, "dna")
    kw = dict(match_score=200, mismatch_score=-300, gap_open_score=-50, gap_extension_score=-7)
    got, cmat, goc = _fill(monkeypatch, td, s1, s2, kw)
    assert got == _oracle_cost(s1, s2, cmat, goc)


@pytest.mark.parametrize("td", [1, 2, 4])
def test_diag_custom_boundary(monkeypatch, td):
    rng = np.random.default_rng(td)
    m, n = 700, 5000
    s1, s2 = splitmix_seq(m, 71, "dna"), splitmix_seq(n, 72, "dna")
    row0 = rng.integers(0, 60, size=3 * (n + 1)).astype(np.int64)
    col0 = rng.integers(0, 60, size=3 * (m + 1)).astype(np.int64)
    row0[:3] = col0[:3] = 0
    got, cmat, goc = _fill(monkeypatch, td, s1, s2, SCORING, row0=row0, col0=col0)
    assert got == _oracle_cost(s1, s2, cmat, goc, row0, col0)


@pytest.mark.parametrize("m,n", [(20_000, 3_000), (9_000, 2_100 + 37)])
def test_auto_tall_score_vs_oracle(monkeypatch, m, n):
    """No override: a score-only fill with m >= 4n takes the anti-diagonal kernel by itself (TD = 1 up to
    131k columns); its cost must equal the oracle's like every other fill's."""
    from globalign_amd import _native
    from globalign_amd._native import CostTables
    from globalign_amd.scoring import validate_and_transform_args
    del_knob(monkeypatch, "GA_FILL_MODE", raising=False)
    del_knob(monkeypatch, "GA_DIAG_COLS_PER_LANE", raising=False)
    s1, s2 = splitmix_seq(m, m + 3, "dna"), splitmix_seq(n, n + 5, "dna")
    _, _, _, cmat, _, goc, _ = validate_and_transform_args(None, None, s1[:64], s2[:64], **SCORING)
    tables = CostTables(cmat, goc)
    eng = _native.Engine(0)
    try:
        eng.load(tables.codes(s1), tables.codes(s2), tables)
        got = int(eng.fill(traceback=False)[0])
    finally:
        eng.close()
    assert got == _oracle_cost(s1, s2, cmat, goc)
