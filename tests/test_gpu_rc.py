"""GPU parity of the recompute walk: a score-only lane fill that leaves checkpoints (every
stripe's right edge, staircase lane states every GA_RC_EVERY steps), then one launch in which workgroup 0
walks while recompute workgroups rebuild the traceback words of the 64-row blocks ahead of it.  The result
must equal the single-problem oracle exactly: cost, the three alignment strings, the final random state.
GA_RC=1 forces the path at small sizes; the full-size C3 pin takes it by default
(test_gpu_parity.py::test_bench_workload_cost_matches_golden)."""
import os
import random

import numpy as np
import pytest

from tests.conftest import splitmix_seq, set_knob

pytestmark = pytest.mark.gpu

DNA = dict(match_score=2, mismatch_score=-3, gap_open_score=-5, gap_extension_score=-1)
JUMP_DEFAULT = "0"  # ga_host.cpp kRcJumpDefault


def _experiments():
    from globalign_amd import _native
    return _native.experiments_build()


# the tie-to-tie walk measured slower than the word walk and is compiled only into an experiments
# build (make EXPERIMENTS=1); its cases run there
needs_jump = pytest.mark.skipif("not __import__('globalign_amd._native', fromlist=['x']).experiments_build()",
                                reason="the tie-to-tie walk is in experiments builds only")


def _align(monkeypatch, s1, s2, kw, seed, env=None, protein=False):
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
    set_knob(monkeypatch, "GA_RC", "1")
    for k, v in (env or {}).items():
        set_knob(monkeypatch, k, str(v))
    eng = _native.Engine(0)
    try:
        eng.load(tables.codes(a1), tables.codes(a2), tables)
        cost, strings, status, mt_after = eng.align(mt, a1, a2)
        kind = eng.fill_kind()
        walk = eng.walk_kind()
    finally:
        eng.close()
    assert kind[0] == "rc", kind  # the recompute path really ran
    # the tie-to-tie walk (jump entries) wherever its workers fit: <= 4 columns per lane, o <= 14
    jump_ok = (_experiments() and kind[1] <= 4 and goc <= 14 and
               str((env or {}).get("GA_RC_JUMP", os.environ.get("GA_RC_JUMP", JUMP_DEFAULT))) != "0")
    assert walk == ("jump" if jump_ok else "rc"), (walk, kind, goc)
    assert status == 0
    assert int(cost) == ref["cost"]
    assert tuple(strings) == tuple(ref["strings"])
    assert np.asarray(mt_after, dtype=np.uint32).tolist() == np.asarray(ref["mt_out"], dtype=np.uint32).tolist()
    return kind


@pytest.mark.parametrize("m,n", [(256, 256), (300, 500), (1000, 1300), (777, 2049), (2049, 3000), (5000, 300),
                                 (300, 5000), (4097, 4097)])
def test_rc_dna_vs_oracle(monkeypatch, m, n):
    _align(monkeypatch, splitmix_seq(m, 11, "dna"), splitmix_seq(n, 12, "dna"), DNA, seed=m + n)


@pytest.mark.parametrize("td", [1, 2, 4, 8])
def test_rc_stripe_widths_vs_oracle(monkeypatch, td):
    """Every fill stripe width (64*TD columns): blocks of TD walker tiles, TD + 1 state pairs per lane."""
    kind = _align(monkeypatch, splitmix_seq(3000, 21, "dna"), splitmix_seq(2500 + 64 * td, 22, "dna"), DNA, seed=td,
                  env={"GA_LANE_COLS_PER_LANE": td})
    assert kind[1] == td


@pytest.mark.parametrize("env", [{"GA_LANE_DIRECT": 1}, {"GA_LANE_DIRECT": 1, "GA_LANE_ASM": 0}, {"GA_LANE_ASM": 0}])
def test_rc_handover_variants_vs_oracle(monkeypatch, env):
    """The checkpointing fill under each edge hand-over: the right-edge checkpoints are read back
    from lanes 48..63 of the lean sub-chunk or from the compiler steps' DPP shift registers (GA_LANE_ASM=0)."""
    _align(monkeypatch, splitmix_seq(3100, 51, "dna"), splitmix_seq(64 * 2 * 4 * 5 + 77, 52, "dna"), DNA, seed=3,
           env=dict(env, GA_LANE_COLS_PER_LANE=2))


@pytest.mark.parametrize("every", [128, 256])
def test_rc_checkpoint_spacing_vs_oracle(monkeypatch, every):
    """Sparser staircase checkpoints: a block is recomputed from up to every + 126 steps above it."""
    _align(monkeypatch, splitmix_seq(3000, 31, "dna"), splitmix_seq(3500, 32, "dna"), DNA, seed=every, env={"GA_RC_EVERY": every})


@pytest.mark.parametrize("td", ["narrow", 4])
@pytest.mark.parametrize("env", [{"GA_RC_SERVERS": 1, "GA_RC_WIN": 4},
                                 {"GA_RC_SERVERS": 2, "GA_RC_WIN": 64, "GA_RC_WPW": 6},
                                 {"GA_RC_SERVERS": 160, "GA_RC_WPW": 4},
                                 {"GA_RC_SERVERS": 1, "GA_RC_WIN": 4, "GA_RC_CONE": 1}])
def test_rc_worker_pools_vs_oracle(monkeypatch, env, td):
    """One worker behind a narrow window, a few many-worker groups, many groups racing for claims, at 2 columns per
    lane (GA_RC_NARROW's choice for DNA) and at 4: the window always offers the walker's own
    2 x 2 blocks first, so even one worker behind a 4-block window never starves it of the stripe to its left (round
    4 kept this case at TD < 4), whatever the cone that ranks the rest."""
    env = dict(env, GA_RC_NARROW=1) if td == "narrow" else dict(env, GA_LANE_COLS_PER_LANE=td)
    kind = _align(monkeypatch, splitmix_seq(2500, 41, "dna"), splitmix_seq(2600, 42, "dna"), DNA, seed=7, env=env)
    assert kind[1] == (2 if td == "narrow" else td), kind


@pytest.mark.parametrize("jump", [0, pytest.param(1, marks=needs_jump)])
def test_rc_lost_slot_tags_repaired_vs_oracle(monkeypatch, jump):
    """Cache slot owner tags (ga::rc_slot_tag): every 3rd block a worker writes is left without its tag,
    as if another block's worker had overwritten the slot; the walk's loaders must never use such a slot, reset the
    block's ready flag and wait for its recompute, and the alignment stays the oracle's, in both walks."""
    _align(monkeypatch, splitmix_seq(2200, 45, "dna"), splitmix_seq(2400, 46, "dna"), DNA, seed=45,
           env={"GA_RC_TAG_FAULT": 3, "GA_RC_JUMP": jump})


@pytest.mark.parametrize("o", [7, 130])
def test_rc_word_widths_vs_oracle(monkeypatch, o):
    """Two- and four-byte traceback words (gap open >= 7, >= 128)."""
    kw = dict(match_score=2, mismatch_score=-3, gap_open_score=-o, gap_extension_score=-1)
    _align(monkeypatch, splitmix_seq(1500, 51, "dna"), splitmix_seq(1700, 52, "dna"), kw, seed=o)


def test_rc_protein_blosum62_vs_oracle(monkeypatch):
    kw = dict(scoring_mat_name="BLOSUM62", gap_open_score=-10)
    _align(monkeypatch, splitmix_seq(1200, 3, "protein"), splitmix_seq(1400, 4, "protein"), kw, seed=3, protein=True)


def test_rc_long_gap_runs_vs_oracle(monkeypatch):
    """A pair whose path runs a long way along one edge: seq_2 = seq_1 plus 2000 extra columns (a
    horizontal gap run the window must follow sideways), then seq_1 much longer than seq_2."""
    a = splitmix_seq(2000, 61, "dna")
    _align(monkeypatch, a, splitmix_seq(1000, 62, "dna") + a + splitmix_seq(1000, 63, "dna"), DNA, seed=61)
    _align(monkeypatch, splitmix_seq(700, 64, "dna") + a + splitmix_seq(900, 65, "dna"), a, DNA, seed=62)


def test_rc_similar_pair_vs_oracle(monkeypatch):
    """Long diagonal match streaks (draw_two_random_seqs, 5 % divergence)."""
    from globalign_amd.random_seqs import draw_two_random_seqs
    orig = random.seed
    monkeypatch.setattr(random, "seed", lambda a=None, version=2: orig(777 if a is None else a, version))
    s1, s2 = draw_two_random_seqs(list("ACGT"), 3500, 3500, 3600, 3600, 0.05, 71, 72)
    monkeypatch.setattr(random, "seed", orig)
    _align(monkeypatch, s1, s2, DNA, seed=71)


def test_rc_repeated_calls_reuse_buffers(monkeypatch):
    """Consecutive calls on one context (new epochs over the same block flags and tile cache, shapes that
    shrink and grow) stay exact."""
    from globalign_amd import _native
    from globalign_amd.scoring import validate_and_transform_args
    from oracle import core, transform
    set_knob(monkeypatch, "GA_RC", "1")
    eng = _native.Engine(0)
    try:
        for k, (m, n) in enumerate([(2000, 2100), (900, 3000), (2000, 2100), (3100, 1200)]):
            s1, s2 = splitmix_seq(m, 81 + k, "dna"), splitmix_seq(n, 91 + k, "dna")
            a1, a2, smat, cmat, gos, goc = transform.settings(dict(DNA, seq_1=s1, seq_2=s2))
            random.seed(k)
            mt = np.array(random.getstate()[1], dtype=np.uint32)
            ref = core.align(a1, a2, cmat, goc, mt)
            _, _, _, cmat2, _, goc2, _ = validate_and_transform_args(None, None, s1[:64], s2[:64], **DNA)
            tables = _native.CostTables(cmat2, goc2)
            eng.load(tables.codes(a1), tables.codes(a2), tables)
            cost, strings, status, mt_after = eng.align(mt, a1, a2)
            assert eng.fill_kind()[0] == "rc"
            assert status == 0 and int(cost) == ref["cost"] and tuple(strings) == tuple(ref["strings"])
            assert np.asarray(mt_after, dtype=np.uint32).tolist() == np.asarray(ref["mt_out"], dtype=np.uint32).tolist()
    finally:
        eng.close()


def test_rc_worker_lds_caps_stripe_width(monkeypatch):
    """A block's staged codes must fit LDS: at 8 columns per lane and a 256-step checkpoint spacing (C4 on one GPU:
    219 KB) the fill narrows its stripes (4 columns per lane, 113 KB) instead of failing the walk's launch."""
    kind = _align(monkeypatch, splitmix_seq(3000, 31, "dna"), splitmix_seq(3100, 32, "dna"), DNA, seed=5,
                  env={"GA_LANE_COLS_PER_LANE": 8, "GA_RC_EVERY": 256})
    assert kind[1] == 4, kind


def test_rc_streamed_decode_check(monkeypatch):
    """The streamed level decode under its own detector: GA_RC_DECODE_CHECK records every level
    word as the host decodes it and fails the call if one changes afterwards (a block published before its
    stores landed); GA_RC_DECODE_LAG=1 holds the decode one 512-dispatch block behind the progress word."""
    _align(monkeypatch, splitmix_seq(4000, 91, "dna"), splitmix_seq(4000, 92, "dna"), DNA, seed=91,
           env={"GA_RC_DECODE_CHECK": 1, "GA_RC_DECODE_LAG": 1})
    _align(monkeypatch, splitmix_seq(4000, 93, "dna"), splitmix_seq(4000, 94, "dna"), DNA, seed=93,
           env={"GA_RC_DECODE_CHECK": 1})


@pytest.mark.parametrize("servers", [3, 200])
def test_rc_deep_window_many_block_rows(monkeypatch, servers):
    """4 columns per lane (blocks of 4 tiles) over ~190 block rows with the full 16 x 16-candidate
    window, so workers with stale views of the walker race to claim and write blocks 15 rows apart; the 32-deep
    cache and the write-time reach check must keep every block the walker reads its own."""
    _align(monkeypatch, splitmix_seq(12000, 95, "dna"), splitmix_seq(3300, 96, "dna"), DNA, seed=servers,
           env={"GA_LANE_COLS_PER_LANE": 4, "GA_RC_SERVERS": servers, "GA_RC_WIN": 64})


def test_rc_checkpoints_over_budget_fall_back(monkeypatch):
    """Checkpoints that do not fit the budget / the free device memory (GA_RC_BUDGET_MB=0 here) make
    ga_problem_align take another traceback path instead of failing; the result stays exact."""
    from globalign_amd import _native
    from globalign_amd.scoring import validate_and_transform_args
    from oracle import core, transform
    s1, s2 = splitmix_seq(2100, 97, "dna"), splitmix_seq(2300, 98, "dna")
    a1, a2, smat, cmat, gos, goc = transform.settings(dict(DNA, seq_1=s1, seq_2=s2))
    random.seed(4)
    mt = np.array(random.getstate()[1], dtype=np.uint32)
    ref = core.align(a1, a2, cmat, goc, mt)
    _, _, _, cmat2, _, goc2, _ = validate_and_transform_args(None, None, s1[:64], s2[:64], **DNA)
    tables = _native.CostTables(cmat2, goc2)
    set_knob(monkeypatch, "GA_RC", "1")
    set_knob(monkeypatch, "GA_RC_BUDGET_MB", "0")
    eng = _native.Engine(0)
    try:
        eng.load(tables.codes(a1), tables.codes(a2), tables)
        cost, strings, status, mt_after = eng.align(mt, a1, a2)
        kind = eng.fill_kind()
    finally:
        eng.close()
    assert kind[0] != "rc", kind
    assert status == 0 and int(cost) == ref["cost"] and tuple(strings) == tuple(ref["strings"])
    assert np.asarray(mt_after, dtype=np.uint32).tolist() == np.asarray(ref["mt_out"], dtype=np.uint32).tolist()


def _align_fallback(monkeypatch, env, seed):
    """A problem the recompute walk would take, under `env` that makes it decline: the call must fall back and
    still equal the oracle (cost, strings, random state)."""
    from globalign_amd import _native
    from globalign_amd.scoring import validate_and_transform_args
    from oracle import core, transform
    s1, s2 = splitmix_seq(1500, 61 + seed, "dna"), splitmix_seq(1700, 62 + seed, "dna")
    a1, a2, smat, cmat, gos, goc = transform.settings(dict(DNA, seq_1=s1, seq_2=s2))
    random.seed(seed)
    mt = np.array(random.getstate()[1], dtype=np.uint32)
    ref = core.align(a1, a2, cmat, goc, mt)
    _, _, _, cmat2, _, goc2, _ = validate_and_transform_args(None, None, s1[:64], s2[:64], **DNA)
    tables = _native.CostTables(cmat2, goc2)
    set_knob(monkeypatch, "GA_RC", "1")
    for k, v in env.items():
        set_knob(monkeypatch, k, str(v))
    eng = _native.Engine(0)
    try:
        eng.load(tables.codes(a1), tables.codes(a2), tables)
        for _ in range(2):  # the fallback twice on one context: nothing of the declined path is left behind
            cost, strings, status, mt_after = eng.align(mt, a1, a2)
            assert eng.fill_kind()[0] != "rc"
            assert status == 0 and int(cost) == ref["cost"]
            assert tuple(strings) == tuple(ref["strings"])
            assert np.asarray(mt_after, dtype=np.uint32).tolist() == np.asarray(ref["mt_out"], dtype=np.uint32).tolist()
    finally:
        eng.close()


def test_rc_checkpoint_alloc_failure_falls_back(monkeypatch):
    """a checkpoint allocation that fails after the other succeeded (GA_RC_FAIL_ALLOC=1) releases the
    recompute buffers and falls back to the stored-words path."""
    _align_fallback(monkeypatch, {"GA_RC_FAIL_ALLOC": 1}, seed=1)


def test_small_device_memory_bands(monkeypatch):
    """With little free device memory (GA_DEV_AVAIL_MB caps what the sizing sees) the recompute walk declines and
    the traceback words are banded to fit, instead of a stored-words fill that cannot allocate."""
    _align_fallback(monkeypatch, {"GA_DEV_AVAIL_MB": 1}, seed=2)


@pytest.mark.parametrize("jump", [0, pytest.param(1, marks=needs_jump)])
@pytest.mark.parametrize("m,n,seed", [(3000, 2600, 71), (2049, 4100, 72)])
def test_rc_jump_and_word_walks_vs_oracle(monkeypatch, jump, m, n, seed):
    """Both recompute walks on the same problems: the tie-to-tie walk (jump entries) and the walk of
    recomputed traceback words (GA_RC_JUMP=0)."""
    _align(monkeypatch, splitmix_seq(m, seed, "dna"), splitmix_seq(n, seed + 1, "dna"), DNA, seed=seed,
           env={"GA_RC_JUMP": jump})


@needs_jump
@pytest.mark.parametrize("o", [1, 2, 6, 14])
def test_rc_jump_gap_opens_vs_oracle(monkeypatch, o):
    """Gap opens across the jump LUT's range (X'-H', Y'-H' saturated at o+1 <= 15), incl. o = 1 and the largest, 14."""
    kw = dict(match_score=2, mismatch_score=-3, gap_open_score=-o, gap_extension_score=-1)
    _align(monkeypatch, splitmix_seq(1800, 81 + o, "dna"), splitmix_seq(1900, 82 + o, "dna"), kw, seed=o,
           env={"GA_RC_JUMP": 1})
