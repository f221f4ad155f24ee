"""GPU parity of the lane-skewed score-only fill (fill_lane_kernel, ga_lane.hip),
forced through GA_FILL_MODE=lane at every columns-per-lane width (GA_LANE_COLS_PER_LANE) and both
workgroup sizes (GA_FILL_NWC): the cost against the CPU oracle (oracle/ga_oracle.c, the restatement of
dp_array_forward globaligner.py:366-392) on shapes with a partial last stripe, n < 64*TD, rows shorter
than the 64-step lane skew, chains of several workgroups, a protein alphabet (BLOSUM62, K = 25),
host-supplied boundary triples and the finite `big` sentinel of very unequal lengths."""
import numpy as np
import pytest

from tests.conftest import splitmix_seq, set_knob

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
    set_knob(monkeypatch, "GA_FILL_MODE", "lane")
    set_knob(monkeypatch, "GA_LANE_COLS_PER_LANE", str(td))
    set_knob(monkeypatch, "GA_FILL_NWC", str(nwc))
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


@pytest.mark.parametrize("td", [1, 2])
def test_lane_rounds(monkeypatch, td):
    """More stripes than 4-wave workgroups can hold at once (one per CU): workgroups run in ticket-ordered
    rounds, a later round reading hand-off rows the earlier one wrote long before (the C4 schedule)."""
    m, n = 400, 64 * td * 4 * 300 + 21
    s1, s2 = splitmix_seq(m, 93 + td, "dna"), splitmix_seq(n, 94 + td, "dna")
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


# ---------------------------------------------------------------- traceback words (ga_lane.hip LkRot)
def _align_lane(monkeypatch, s1, s2, kw, seed, td, nwc=4, protein=False, band_rows=None, tb_sub=None):
    """Fill with the lane kernel's traceback words + the walk, against the oracle's dp_array_backward
    (globaligner.py:395-593): cost, the three alignment strings and the final random state."""
    import random
    from globalign_amd import _native
    from globalign_amd.scoring import validate_and_transform_args
    from oracle import core, transform
    from tests.conftest import load_matrix
    a1, a2, smat, cmat, gos, goc = transform.settings(dict(kw, seq_1=s1, seq_2=s2),
                                                      blosum=load_matrix("BLOSUM62") if protein else None)
    random.seed(seed)
    mt = np.array(random.getstate()[1], dtype=np.uint32)
    ref = core.align(a1, a2, cmat, goc, mt)
    _, _, _, cmat2, _, goc2, _ = validate_and_transform_args(None, None, s1[:64], s2[:64], **kw)
    tables = _native.CostTables(cmat2, goc2)
    set_knob(monkeypatch, "GA_FILL_MODE", "lane")
    set_knob(monkeypatch, "GA_LANE_COLS_PER_LANE", str(td))
    set_knob(monkeypatch, "GA_FILL_NWC", str(nwc))
    if band_rows:
        set_knob(monkeypatch, "GA_TB_BAND_ROWS", str(band_rows))
    if tb_sub:
        set_knob(monkeypatch, "GA_LANE_TB_SUB", str(tb_sub))
    eng = _native.Engine(0)
    try:
        eng.load(tables.codes(a1), tables.codes(a2), tables)
        cost, strings, status, mt_after = eng.align(mt, a1, a2)
        kind = eng.fill_kind()
    finally:
        eng.close()
    assert kind[0] == "lane" and kind[1] == td, kind
    assert status == 0
    assert int(cost) == ref["cost"]
    assert tuple(strings) == tuple(ref["strings"])
    assert np.asarray(mt_after, dtype=np.uint32).tolist() == np.asarray(ref["mt_out"], dtype=np.uint32).tolist()


@pytest.mark.parametrize("tb_sub", [8, 16])
@pytest.mark.parametrize("td", [1, 2, 4])
@pytest.mark.parametrize("m,n", [(1, 1), (7, 300), (63, 64), (200, 2049), (1000, 1300), (2049, 700), (3000, 5000)])
def test_lane_traceback_dna_vs_oracle(monkeypatch, td, m, n, tb_sub):
    """One-byte words through 8-step sub-chunk pairs and 16-step sub-chunks (one window each)."""
    s1, s2 = splitmix_seq(m, m + 17, "dna"), splitmix_seq(n, n + 19, "dna")
    _align_lane(monkeypatch, s1, s2, SCORING, seed=m ^ n ^ td, td=td, tb_sub=tb_sub)


@pytest.mark.parametrize("td", [1, 2])
@pytest.mark.parametrize("o", [10, 300])
def test_lane_traceback_word_widths(monkeypatch, td, o):
    """2- and 4-byte traceback words (o + 1 >= 8 / >= 128): the window rotation over 8 / 16 dwords."""
    s1, s2 = splitmix_seq(900, 31 + o, "dna"), splitmix_seq(1700, 32 + o, "dna")
    kw = dict(match_score=2, mismatch_score=-3, gap_open_score=-o, gap_extension_score=-1)
    _align_lane(monkeypatch, s1, s2, kw, seed=o + td, td=td)


@pytest.mark.parametrize("td,nwc", [(1, 8), (2, 8), (2, 4)])
def test_lane_traceback_protein(monkeypatch, td, nwc):
    s1, s2 = splitmix_seq(1500, 3, "protein"), splitmix_seq(2600, 4, "protein")
    _align_lane(monkeypatch, s1, s2, dict(scoring_mat_name="BLOSUM62", gap_open_score=-10), seed=td,
                td=td, nwc=nwc, protein=True)


@pytest.mark.parametrize("td", [1, 4])
def test_lane_traceback_similar_pair(monkeypatch, td):
    """A near-diagonal path through many ties (draw_two_random_seqs-like similar pair)."""
    s1 = splitmix_seq(4000, 5, "dna")
    s2 = s1[:1500] + "ACGT" + s1[1500:3000] + s1[3100:]
    _align_lane(monkeypatch, s1, s2, SCORING, seed=11, td=td)


@pytest.mark.parametrize("td", [1, 2, 4])
@pytest.mark.parametrize("band_rows", [16, 96, 256])
def test_lane_traceback_banded(monkeypatch, td, band_rows):
    """Banded (linear-memory) traceback through the lane kernel: its score pass stores the checkpoint rows
    (one per lane window at most, band_rows >= 16), then lane-kernel refills from checkpoint tops over
    prefix columns."""
    s1, s2 = splitmix_seq(2049, 41, "dna"), splitmix_seq(3000, 42, "dna")
    _align_lane(monkeypatch, s1, s2, SCORING, seed=7 + band_rows, td=td, band_rows=band_rows)


@pytest.mark.parametrize("env", [{}, {"GA_LANE_DIRECT": "1"}, {"GA_LANE_DIRECT": "1", "GA_LANE_ASM": "0"}, {"GA_LANE_ASM": "0"},
                                 {"GA_LANE_LATE": "0"}])
@pytest.mark.parametrize("td", [1, 2, 4])
def test_lane_handover_variants(monkeypatch, env, td):
    """The edge hand-over variants over a chain of many workgroups with a partial last stripe:
    the lean asm sub-chunk (default), the IO wave's workgroup hand-off and the last compute wave's direct one
    (GA_LANE_DIRECT=1), the compiler's step (GA_LANE_ASM=0), early edge reads (GA_LANE_LATE=0)."""
    for k, v in env.items():
        set_knob(monkeypatch, k, v)
    m, n = 2100, 64 * td * 4 * 12 + 37
    s1, s2 = splitmix_seq(m, 301 + td, "dna"), splitmix_seq(n, 302 + td, "dna")
    got, cmat, goc = _fill(monkeypatch, td, 4, s1, s2, SCORING)
    assert got == _oracle_cost(s1, s2, cmat, goc)
