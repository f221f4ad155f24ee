"""GPU parity of the blocked fill (T columns per lane) for every T the engine
builds, forced through GA_COLS_PER_LANE on a fresh context: full alignment (cost, strings, final
random state) and score-only cost vs the CPU oracle, on shapes that exercise a partial last stripe
(n not a multiple of 64*T, n < 64*T), multi-workgroup chains, ragged m and a row m inside the
last 16-row chunk at every offset."""
import random

import numpy as np
import pytest

from tests.conftest import splitmix_seq, set_knob

pytestmark = pytest.mark.gpu

SCORING = dict(match_score=2, mismatch_score=-3, gap_open_score=-5, gap_extension_score=-1)


def _tables(seq_1, seq_2, scoring=SCORING):
    from globalign_amd._native import CostTables
    from globalign_amd.scoring import validate_and_transform_args
    _, _, _, cmat, _, goc, _ = validate_and_transform_args(None, None, seq_1[:64], seq_2[:64], **scoring)
    return CostTables(cmat, goc), cmat, goc


def _engine(monkeypatch, T):
    from globalign_amd import _native
    set_knob(monkeypatch, "GA_COLS_PER_LANE", str(T))
    return _native.Engine(0)


@pytest.mark.parametrize("T", [2, 4, 8])
@pytest.mark.parametrize("m,n", [(5, 130), (17, 513), (31, 64), (300, 2049), (2049, 1023), (1000, 5000),
                                 (130, 4 * 512 + 3)])
def test_blocked_align_vs_oracle(monkeypatch, T, m, n):
    from oracle import core
    seed = 7 * m + n + T
    s1, s2 = splitmix_seq(m, seed, "dna"), splitmix_seq(n, seed + 1, "dna")
    tables, cmat, goc = _tables(s1, s2)
    random.seed(seed)
    mt = np.array(random.getstate()[1], dtype=np.uint32)
    ref = core.align(s1, s2, cmat, goc, mt)
    eng = _engine(monkeypatch, T)
    try:
        eng.load(tables.codes(s1), tables.codes(s2), tables)
        cost, strings, status, mt_after = eng.align(mt, s1, s2)
        score_cost = eng.fill(traceback=False)[0]
    finally:
        eng.close()
    assert status == 0
    assert int(cost) == ref["cost"] and int(score_cost) == ref["cost"]
    assert tuple(strings) == tuple(ref["strings"])
    assert np.asarray(mt_after, dtype=np.uint32).tolist() == np.asarray(ref["mt_out"], dtype=np.uint32).tolist()


@pytest.mark.parametrize("T", [2, 4, 8])
def test_blocked_protein_vs_oracle(monkeypatch, T):
    """BLOSUM62 (25-letter profile, asymmetric gap costs, int8 profile), open -10."""
    from oracle import core
    from tests.conftest import load_matrix
    from oracle import transform
    s1, s2 = splitmix_seq(700, 3, "protein"), splitmix_seq(1300, 4, "protein")
    kw = dict(scoring_mat_name="BLOSUM62", gap_open_score=-10)
    a1, a2, smat, cmat, gos, goc = transform.settings(dict(kw, seq_1=s1, seq_2=s2), blosum=load_matrix("BLOSUM62"))
    tables, _, _ = _tables(s1, s2, kw)
    random.seed(11)
    mt = np.array(random.getstate()[1], dtype=np.uint32)
    ref = core.align(a1, a2, cmat, goc, mt)
    eng = _engine(monkeypatch, T)
    try:
        eng.load(tables.codes(s1), tables.codes(s2), tables)
        cost, strings, status, _ = eng.align(mt, s1, s2)
    finally:
        eng.close()
    assert status == 0 and int(cost) == ref["cost"] and tuple(strings) == tuple(ref["strings"])


@pytest.mark.parametrize("T", [4, 8])
def test_blocked_multi_round_score_vs_oracle(monkeypatch, T):
    """More workgroup slabs than CUs with blocked stripes (the C4 shape, shortened): 600 x 1.2M."""
    from oracle import core
    s1, s2 = splitmix_seq(600, 51, "dna"), splitmix_seq(1_200_000 + 77, 52, "dna")
    tables, cmat, goc = _tables(s1, s2)
    eng = _engine(monkeypatch, T)
    try:
        eng.load(tables.codes(s1), tables.codes(s2), tables)
        cost = eng.fill(traceback=False)[0]
    finally:
        eng.close()
    tab = core.Tables(cmat)
    a, b = tab.codes(s1), tab.codes(s2)
    big = (tab.max_cost + 1) * max(len(s1), len(s2))
    row0, col0 = core.boundary(tab, a, b, goc, big)
    assert int(cost) == int(min(core.fill_score_parallel(tab, a, b, goc, row0, col0, 8)))


@pytest.mark.parametrize("T", [1, 2, 4, 8])
def test_blocked_custom_boundary_vs_oracle(monkeypatch, T):
    """Host-supplied row-0 / column-0 triples (dp_array_forward on a caller's dp_array, globaligner.py:366-392):
    every workgroup's first row takes its corner from the top row, at every stripe width."""
    from oracle import core
    rng = np.random.default_rng(T)
    m, n = 700, 5000
    s1, s2 = splitmix_seq(m, 61, "dna"), splitmix_seq(n, 62, "dna")
    tables, cmat, goc = _tables(s1, s2)
    row0 = rng.integers(0, 60, size=3 * (n + 1)).astype(np.int64)
    col0 = rng.integers(0, 60, size=3 * (m + 1)).astype(np.int64)
    row0[:3] = col0[:3] = 0
    tab = core.Tables(cmat)
    want = int(min(core.fill_score(tab, tab.codes(s1), tab.codes(s2), goc, row0, col0)))
    eng = _engine(monkeypatch, T)
    try:
        eng.load(tables.codes(s1), tables.codes(s2), tables, row0=row0, col0=col0)
        got = int(eng.fill(traceback=False)[0])
    finally:
        eng.close()
    assert got == want
