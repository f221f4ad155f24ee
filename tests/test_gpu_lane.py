"""GPU parity of the lane-skewed score-only fill (fill_lane_kernel, ga_lane.hip),
forced through GA_FILL_MODE=lane at every columns-per-lane width (GA_LANE_COLS_PER_LANE) and both
workgroup sizes (GA_FILL_NWC): the cost against the CPU oracle (oracle/ga_oracle.c, the restatement of
dp_array_forward globaligner.py:366-392) on shapes with a partial last stripe, n < 64*TD, rows shorter
than the 64-step lane skew, chains of several workgroups, a protein alphabet (BLOSUM62, K = 25),
host-supplied boundary triples and the finite `big` sentinel of very unequal lengths."""
import numpy as np
import pytest

from tests.conftest import splitmix_seq

pytestmark = pytest.mark.gpu

SCORING = dict(match_score=2, mismatch_score=-3, gap_open_score=-5, gap_extension_score=-1)


def _oracle_cost(s1, s2, cmat, goc, row0=None, col0=None):
    from oracle import core
    tab = core.Tables(cmat)
    a, b = tab.codes(s1), tab.codes(s2)
    if row0 is None:
        big = (tab.max_cost + 1) * max(len(s1), len(s2))
        row0, col0 = core.boundary(tab, a, b, goc, big)
    return int(min(core.fill_score(tab, a, b, goc, row0, col0)))


def _fill(monkeypatch, td, nwc, s1, s2, kw, **load_kw):
    from globalign_amd import _native
    from globalign_amd._native import CostTables
    from globalign_amd.scoring import validate_and_transform_args
    monkeypatch.setenv("GA_FILL_MODE", "lane")
    monkeypatch.setenv("GA_LANE_COLS_PER_LANE", str(td))
    monkeypatch.setenv("GA_FILL_NWC", str(nwc))
    _, _, _, cmat, _, goc, _ = validate_and_transform_args(None, None, s1[:64], s2[:64], **kw)
    tables = CostTables(cmat, goc)
    eng = _native.Engine(0)
    try:
        eng.load(tables.codes(s1), tables.codes(s2), tables, **load_kw)
        cost = int(eng.fill(traceback=False)[0])
        kind = eng.fill_kind()
    finally:
        eng.close()
    assert kind[0] == "lane" and kind[1] == td and kind[3] == nwc, kind
    return cost, cmat, goc


@pytest.mark.parametrize("td", [1, 2, 4, 8])
@pytest.mark.parametrize("nwc", [4, 8])
@pytest.mark.parametrize("m,n", [(1, 1), (5, 130), (17, 513), (63, 64), (64, 1000), (300, 2049), (2049, 1023),
                                 (1000, 5000), (130, 8 * 512 + 3), (3000, 300)])
def test_lane_cost_vs_oracle(monkeypatch, td, nwc, m, n):
    seed = 13 * m + n + td + nwc
    s1, s2 = splitmix_seq(m, seed, "dna"), splitmix_seq(n, seed + 1, "dna")
    got, cmat, goc = _fill(monkeypatch, td, nwc, s1, s2, SCORING)
    assert got == _oracle_cost(s1, s2, cmat, goc)


@pytest.mark.parametrize("td", [1, 8])
def test_lane_many_workgroups(monkeypatch, td):
    """More stripes than one workgroup holds many times over: the workgroup hand-off rows chain."""
    m, n = 1500, 64 * td * 4 * 40 + 17
    s1, s2 = splitmix_seq(m, 91 + td, "dna"), splitmix_seq(n, 92 + td, "dna")
    got, cmat, goc = _fill(monkeypatch, td, 4, s1, s2, SCORING)
    assert got == _oracle_cost(s1, s2, cmat, goc)


@pytest.mark.parametrize("td", [2, 8])
def test_lane_protein_blosum62(monkeypatch, td):
    s1, s2 = splitmix_seq(1200, 31, "protein"), splitmix_seq(2500, 32, "protein")
    kw = dict(scoring_mat_name="BLOSUM62", gap_open_score=-10)
    got, cmat, goc = _fill(monkeypatch, td, 8, s1, s2, kw)
    assert got == _oracle_cost(s1, s2, cmat, goc)


@pytest.mark.parametrize("td", [1, 4])
def test_lane_custom_boundary(monkeypatch, td):
    rng = np.random.default_rng(td)
    m, n = 700, 5000
    s1, s2 = splitmix_seq(m, 71, "dna"), splitmix_seq(n, 72, "dna")
    row0 = rng.integers(0, 60, size=3 * (n + 1)).astype(np.int64)
    col0 = rng.integers(0, 60, size=3 * (m + 1)).astype(np.int64)
    row0[:3] = col0[:3] = 0
    got, cmat, goc = _fill(monkeypatch, td, 4, s1, s2, SCORING, row0=row0, col0=col0)
    assert got == _oracle_cost(s1, s2, cmat, goc, row0, col0)


@pytest.mark.parametrize("m,n", [(40, 9000), (9000, 40)])
def test_lane_sentinel_unequal(monkeypatch, m, n):
    """Very unequal lengths: the boundary's finite `big` sentinel (make_dp_array :756-821) in range."""
    s1, s2 = splitmix_seq(m, m + 1, "dna"), splitmix_seq(n, n + 2, "dna")
    got, cmat, goc = _fill(monkeypatch, 2, 4, s1, s2, SCORING)
    assert got == _oracle_cost(s1, s2, cmat, goc)
