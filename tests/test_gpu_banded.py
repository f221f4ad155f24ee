"""GPU parity of the banded traceback: a score-only fill that checkpoints the
(H', h2') row every Bh rows, then band-by-band refills with traceback words and a walk handed on
at each band's top row.  Bands are forced small through GA_TB_BAND_ROWS so that walks cross many
band boundaries; the result must equal the single-problem oracle exactly (cost, the three
alignment strings, the final random state)."""
import random

import numpy as np
import pytest

from tests.conftest import splitmix_seq, set_knob, del_knob

pytestmark = pytest.mark.gpu


def _align(monkeypatch, s1, s2, kw, seed, band_rows, protein=False):
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
    set_knob(monkeypatch, "GA_TB_BAND_ROWS", str(band_rows))
    eng = _native.Engine(0)
    try:
        eng.load(tables.codes(a1), tables.codes(a2), tables)
        cost, strings, status, mt_after = eng.align(mt, a1, a2)
    finally:
        eng.close()
    assert status == 0
    assert int(cost) == ref["cost"]
    assert tuple(strings) == tuple(ref["strings"])
    assert np.asarray(mt_after, dtype=np.uint32).tolist() == np.asarray(ref["mt_out"], dtype=np.uint32).tolist()


DNA = dict(match_score=2, mismatch_score=-3, gap_open_score=-5, gap_extension_score=-1)


@pytest.mark.parametrize("m,n,bh", [(300, 500, 64), (133, 90, 64), (1000, 1300, 128), (777, 2049, 96), (65, 100, 32),
                                    (5000, 200, 512), (2049, 3000, 16)])
def test_banded_dna_vs_oracle(monkeypatch, m, n, bh):
    s1, s2 = splitmix_seq(m, m + 7, "dna"), splitmix_seq(n, n + 9, "dna")
    _align(monkeypatch, s1, s2, DNA, seed=m ^ n, band_rows=bh)


@pytest.mark.parametrize("m,n,bh", [(6000, 300, 512), (9000, 640, 2048), (4096, 1024, 16)])
def test_banded_lane_checkpoint_pass_vs_oracle(monkeypatch, m, n, bh):
    """Tall shapes, whose score-only checkpoint pass takes the lane-skewed kernel, the band
    refills the row scan."""
    s1, s2 = splitmix_seq(m, m + 3, "dna"), splitmix_seq(n, n + 5, "dna")
    _align(monkeypatch, s1, s2, DNA, seed=m ^ bh, band_rows=bh)


@pytest.mark.parametrize("o", [10, 300])
def test_banded_word_widths_vs_oracle(monkeypatch, o):
    """2- and 4-byte traceback words (o + 1 >= 8 / >= 128)."""
    s1, s2 = splitmix_seq(900, 31, "dna"), splitmix_seq(700, 32, "dna")
    kw = dict(match_score=2, mismatch_score=-3, gap_open_score=-o, gap_extension_score=-1)
    _align(monkeypatch, s1, s2, kw, seed=o, band_rows=64)


def test_banded_protein_vs_oracle(monkeypatch):
    s1, s2 = splitmix_seq(1200, 3, "protein"), splitmix_seq(1000, 4, "protein")
    _align(monkeypatch, s1, s2, dict(scoring_mat_name="BLOSUM62", gap_open_score=-10), seed=5, band_rows=128,
           protein=True)


def test_banded_similar_pair_vs_oracle(monkeypatch):
    """Long diagonal runs that cross band tops with the walk inside a match streak."""
    from globalign_amd.random_seqs import draw_two_random_seqs
    orig = random.seed
    monkeypatch.setattr(random, "seed", lambda a=None, version=2: orig(77 if a is None else a, version))
    s1, s2 = draw_two_random_seqs(list("ACGT"), 3000, 3000, 3100, 3100, 0.05, 41, 42)
    monkeypatch.setattr(random, "seed", orig)
    _align(monkeypatch, s1, s2, DNA, seed=9, band_rows=256)


def test_banded_matches_unbanded_100k(monkeypatch):
    """C3 size: the banded traceback (13 bands of 8192 rows) against the one-pass traceback, whose cost the
    C oracle pins (test_gpu_parity.test_large_100k_score_vs_oracle): identical strings and random state."""
    import bench
    from globalign_amd import _native
    wl = bench.WORKLOADS["c3"]
    s1, s2 = bench.workload_pair(wl)
    tables, _ = bench.problem_tables(s1, s2, wl["scoring"])
    random.seed(0)
    mt = np.array(random.getstate()[1], dtype=np.uint32)
    out = []
    for rows in (None, 8192):
        if rows is None:
            del_knob(monkeypatch, "GA_TB_BAND_ROWS", raising=False)
        else:
            set_knob(monkeypatch, "GA_TB_BAND_ROWS", str(rows))
        eng = _native.Engine(0)
        try:
            eng.load(tables.codes(s1), tables.codes(s2), tables)
            out.append(eng.align(mt, s1, s2))
        finally:
            eng.close()
    (c0, st0, s0, mt0), (c1, st1, s1_, mt1) = out
    assert s0 == 0 and s1_ == 0 and int(c0) == int(c1)
    assert tuple(st0) == tuple(st1)
    assert np.asarray(mt0).tolist() == np.asarray(mt1).tolist()
