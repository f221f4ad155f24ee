"""GPU parity: the HIP path (through the C ABI) vs the reference's golden
vectors and the CPU oracle.  Bit-exact for costs, scores, alignment strings
and the global random state after the traceback's random.choice calls.
"""
import json
import os
import random

import numpy as np
import pytest

from tests.conftest import GOLDEN, aln_digest, load_matrix, splitmix_seq, state_digest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ga():
    import globalign_amd
    from globalign_amd import _native
    assert _native.device_count() >= 1
    return globalign_amd


def _kwargs(rec, tmp_path):
    kw = {k: v for k, v in rec["kwargs"].items()}
    if "mtx" in rec:
        letters, S = rec["mtx"]["letters"], rec["mtx"]["scores"]
        path = tmp_path / "m.mtx"
        lines = ["  ".join(letters)] + [letters[x] + " " + " ".join(str(v) for v in S[x]) for x in range(len(letters))]
        path.write_text("\n".join(lines) + "\n")
        kw["scoring_mat_path"] = str(path)
    return kw


def _check_api(ga, rec, tmp_path):
    random.seed(rec["seed"])
    kw = _kwargs(rec, tmp_path)
    if "error" in rec:
        import builtins
        with pytest.raises(getattr(builtins, rec["error"])) as ei:
            ga.find_global_alignment(**kw)
        assert type(ei.value).__name__ == rec["error"]
    else:
        r = ga.find_global_alignment(**kw)
        assert (r.seq_1_aligned, r.middle_part, r.seq_2_aligned) == (
            rec["seq_1_aligned"], rec["middle_part"], rec["seq_2_aligned"]), rec
        assert r.cost == rec["cost"] and r.score == rec["score"]
        assert r.gap_open_score == rec["gap_open_score"] and r.gap_open_cost == rec["gap_open_cost"]
        if "costing_mat" in rec:
            assert r.costing_mat == rec["costing_mat"] and r.scoring_mat == rec["scoring_mat"]
    assert state_digest() == rec["state_after"]


def test_kat_reference_suite(ga, tmp_path):
    """tests/globaligner_test.py:40-383 and tutorial.qmd known answers (+ strings under seed 0)."""
    kat = json.load(open(os.path.join(GOLDEN, "kat.json")))
    for rec in kat["api"]:
        _check_api(ga, rec, tmp_path)


def test_kat_dp_array_forward(ga):
    """tests/globaligner_test.py:6-37: the reference's hand-written 3x3 boundary."""
    rec = json.load(open(os.path.join(GOLDEN, "kat.json")))["fill"]
    dp = [[tuple(c) if c is not None else None for c in row] for row in rec["dp_in"]]
    ga.dp_array_forward(dp, rec["seq_1"], rec["seq_2"], rec["costing_mat"], rec["gap_open_cost"])
    assert [[list(c) for c in row] for row in dp] == rec["dp_out"]


def test_random_fill_fixtures(ga):
    for rec in json.load(open(os.path.join(GOLDEN, "random_fill.json"))):
        dp = [[tuple(c) if c is not None else None for c in row] for row in rec["dp_in"]]
        ga.dp_array_forward(dp, rec["seq_1"], rec["seq_2"], rec["costing_mat"], rec["gap_open_cost"])
        assert [[list(c) for c in row] for row in dp] == rec["dp_out"]


def test_random_api_fixtures(ga, tmp_path):
    """700 reference calls: all settings branches, degenerate lengths (IndexError quirk)."""
    for rec in json.load(open(os.path.join(GOLDEN, "random_api.json"))):
        _check_api(ga, rec, tmp_path)


def _splitmix_case(ga, rec):
    s1 = splitmix_seq(rec["m"], rec["seeds"][0], rec["alphabet"])
    s2 = splitmix_seq(rec["n"], rec["seeds"][1], rec["alphabet"])
    random.seed(rec["seed"])
    r = ga.GlobalAligner(max_seq_len_prod=None, **rec["kwargs"]).align(s1, s2)
    assert r.cost == rec["cost"] and r.score == rec["score"]
    assert len(r.middle_part) == rec["aln_len"]
    assert aln_digest(r.seq_1_aligned, r.middle_part, r.seq_2_aligned) == rec["aln_sha16"]
    assert state_digest() == rec["state_after"]


def test_splitmix_golden(ga):
    """SURVEY 8d synthetic configs vs the reference (1k DNA/protein, 1.5k x 0.7k, 2k, and 10k when generated)."""
    for rec in json.load(open(os.path.join(GOLDEN, "splitmix.json"))):
        _splitmix_case(ga, rec)


# ---------------------------------------------------------------- vs the CPU oracle
def _oracle_case(ga, s1, s2, kw, seed, mode="auto"):
    from oracle import core, transform
    blosum = load_matrix(kw["scoring_mat_name"]) if kw.get("scoring_mat_name") else None
    full_kw = dict(kw, seq_1=s1, seq_2=s2)
    a1, a2, smat, cmat, gos, goc = transform.settings(full_kw, blosum=blosum)
    random.seed(seed)
    ref = core.align(a1, a2, cmat, goc, core.mt_state_array(), mode=mode)
    random.seed(seed)
    r = ga.GlobalAligner(max_seq_len_prod=None, **kw).align(s1, s2)
    assert r.cost == ref["cost"]
    assert (r.seq_1_aligned, r.middle_part, r.seq_2_aligned) == ref["strings"]
    assert state_digest() == state_digest(core.mt_state_tuple(ref["mt_out"]))
    return r


def _rand(rng, alpha, n):
    return "".join(rng.choice(alpha) for _ in range(n))


@pytest.mark.parametrize("m,n", [(1, 1), (2, 2), (3, 70), (63, 64), (64, 65), (65, 63), (100, 449), (449, 100),
                                 (448, 448), (130, 1000), (1000, 130), (777, 1555), (2049, 1023)])
def test_shapes_vs_oracle(ga, m, n):
    """Partial stripes, one/many workgroups, m < 64 skew-only rows, m or n == 1."""
    rng = random.Random(m * 1000 + n)
    s1, s2 = _rand(rng, "ACGT", m), _rand(rng, "ACGT", n)
    kw = dict(match_score=2, mismatch_score=-3, gap_open_score=-5, gap_extension_score=-1)
    if min(m, n) == 1:
        pytest.skip("m or n == 1 covered by the fixture quirk cases")
    _oracle_case(ga, s1, s2, kw, seed=m + n)


@pytest.mark.parametrize("o", [0, 1, 6, 7, 10, 126, 127, 300])
def test_gap_open_word_widths(ga, o):
    """1-, 2- and 4-byte traceback words (o+1 < 8, < 128, otherwise)."""
    rng = random.Random(o)
    s1, s2 = _rand(rng, "ACGT", 300), _rand(rng, "ACGT", 211)
    _oracle_case(ga, s1, s2, dict(match_score=3, mismatch_score=-2, gap_open_score=-o, gap_extension_score=-1), seed=o)


def test_sentinel_leak_cases(ga):
    """Short sequences with a large gap-open: the finite sentinel big leaks into the optimum."""
    rng = random.Random(5)
    for k in range(40):
        s1, s2 = _rand(rng, "ACGT", rng.randint(2, 9)), _rand(rng, "ACGT", rng.randint(2, 9))
        _oracle_case(ga, s1, s2, dict(match_score=1, mismatch_score=-1, gap_open_score=-rng.choice([20, 40, 60]),
                                      gap_extension_score=-1), seed=k)


def test_protein_blosum62_open10(ga):
    """Config C5 shape at 3k x 2.5k: BLOSUM62 costs gH=9, gV=10 (asymmetric), open cost 10 (2-byte words)."""
    s1, s2 = splitmix_seq(3000, 3, "protein"), splitmix_seq(2500, 4, "protein")
    _oracle_case(ga, s1, s2, dict(scoring_mat_name="BLOSUM62", gap_open_score=-10), seed=1, mode="sets")


@pytest.mark.slow
def test_dna_6k_vs_oracle(ga):
    s1, s2 = splitmix_seq(6000, 11, "dna"), splitmix_seq(5000, 12, "dna")
    _oracle_case(ga, s1, s2, dict(match_score=2, mismatch_score=-3, gap_open_score=-5, gap_extension_score=-1), seed=9,
                 mode="sets")


def test_score_only_matches_traceback_cost(ga):
    s1, s2 = splitmix_seq(3000, 1, "dna"), splitmix_seq(2000, 2, "dna")
    kw = dict(match_score=2, mismatch_score=-3, gap_open_score=-5, gap_extension_score=-1)
    random.seed(0)
    r1 = ga.GlobalAligner(max_seq_len_prod=None, **kw).align(s1, s2)
    r2 = ga.GlobalAligner(max_seq_len_prod=None, traceback=False, **kw).align(s1, s2)
    assert r1.cost == r2.cost and r1.score == r2.score and r2.seq_1_aligned is None


def test_alignment_rescoring(ga):
    """The emitted alignment costs exactly the reported optimum (recomputed from the strings)."""
    s1, s2 = splitmix_seq(4000, 21, "dna"), splitmix_seq(3500, 22, "dna")
    kw = dict(match_score=2, mismatch_score=-3, gap_open_score=-5, gap_extension_score=-1)
    random.seed(3)
    r = ga.GlobalAligner(max_seq_len_prod=None, **kw).align(s1, s2)
    C, o = r.costing_mat, r.gap_open_cost
    cost, prev = 0, None
    for x, y in zip(r.seq_1_aligned, r.seq_2_aligned):
        kind = 0 if (x != "-" and y != "-") else (1 if x == "-" else 2)
        cost += C[x][y] if kind == 0 else (C["-"][y] if kind == 1 else C[x]["-"])
        if kind != 0 and kind != prev:
            cost += o
        prev = kind
    assert cost == r.cost
    assert r.seq_1_aligned.replace("-", "") == s1 and r.seq_2_aligned.replace("-", "") == s2


def test_large_100k_score_vs_oracle(ga):
    """Config C3 size: 100k x 100k DNA fill + traceback on the GPU; cost vs the C oracle's O(n)-memory fill,
    and the alignment must re-derive the sequences (size-independent properties)."""
    from oracle import core
    s1 = _fast_splitmix(100_000, 1)
    s2 = _fast_splitmix(100_000, 2)
    kw = dict(match_score=2, mismatch_score=-3, gap_open_score=-5, gap_extension_score=-1)
    random.seed(0)
    r = ga.GlobalAligner(max_seq_len_prod=None, **kw).align(s1, s2)
    tab = core.Tables(r.costing_mat)
    a, b = tab.codes(s1), tab.codes(s2)
    big = (tab.max_cost + 1) * 100_000
    row0, col0 = core.boundary(tab, a, b, r.gap_open_cost, big)
    last = core.fill_score(tab, a, b, r.gap_open_cost, row0, col0)
    assert r.cost == int(min(last))
    assert r.seq_1_aligned.replace("-", "") == s1 and r.seq_2_aligned.replace("-", "") == s2
    assert len(r.middle_part) == len(r.seq_1_aligned) == len(r.seq_2_aligned)


def _fast_splitmix(length, seed, alphabet="dna"):
    """numpy SplitMix64 (same stream as tests.conftest.splitmix_seq)."""
    with np.errstate(over="ignore"):
        k = np.arange(1, length + 1, dtype=np.uint64)
        z = np.uint64(seed) + k * np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    if alphabet == "dna":
        idx = (z >> np.uint64(62)).astype(np.int64)
        return "".join(np.array(list("ACGT"))[idx])
    idx = (((z >> np.uint64(32)) * np.uint64(20)) >> np.uint64(32)).astype(np.int64)
    return "".join(np.array(list("ARNDCQEGHILKMFPSTWYV"))[idx])


def test_fast_splitmix_matches_reference_generator():
    assert _fast_splitmix(500, 1) == splitmix_seq(500, 1, "dna")
    assert _fast_splitmix(300, 4, "protein") == splitmix_seq(300, 4, "protein")


def _rescore(r):
    """Cost of an emitted alignment recomputed from its strings (affine gaps: open paid per gap run)."""
    C, o = r.costing_mat, r.gap_open_cost
    cost, prev = 0, None
    for x, y in zip(r.seq_1_aligned, r.seq_2_aligned):
        kind = 0 if (x != "-" and y != "-") else (1 if x == "-" else 2)
        cost += C[x][y] if kind == 0 else (C["-"][y] if kind == 1 else C[x]["-"])
        if kind != 0 and kind != prev:
            cost += o
        prev = kind
    return cost


def test_multi_round_slabs_vs_oracle(ga):
    """More workgroup slabs than CUs (ticket-ordered rounds, as C4 runs on one GPU): 1000 x 200k DNA is
    3125 stripes = 391 slabs of 8 waves.  Cost vs the C oracle's O(n)-memory fill; the alignment must
    re-derive both sequences and rescore to the same cost."""
    from oracle import core
    s1, s2 = _fast_splitmix(1000, 31), _fast_splitmix(200_000, 32)
    kw = dict(match_score=2, mismatch_score=-3, gap_open_score=-5, gap_extension_score=-1)
    random.seed(4)
    r = ga.GlobalAligner(max_seq_len_prod=None, **kw).align(s1, s2)
    tab = core.Tables(r.costing_mat)
    a, b = tab.codes(s1), tab.codes(s2)
    big = (tab.max_cost + 1) * 200_000
    row0, col0 = core.boundary(tab, a, b, r.gap_open_cost, big)
    assert r.cost == int(min(core.fill_score(tab, a, b, r.gap_open_cost, row0, col0)))
    assert r.seq_1_aligned.replace("-", "") == s1 and r.seq_2_aligned.replace("-", "") == s2
    assert _rescore(r) == r.cost


def test_tall_narrow_vs_oracle(ga):
    """200k x 1000 (16 stripes, 4 slabs): long stripes, many 16-row chunks, ring wrap-around."""
    from oracle import core
    s1, s2 = _fast_splitmix(200_000, 33), _fast_splitmix(1000, 34)
    kw = dict(match_score=2, mismatch_score=-3, gap_open_score=-5, gap_extension_score=-1)
    random.seed(5)
    r = ga.GlobalAligner(max_seq_len_prod=None, **kw).align(s1, s2)
    tab = core.Tables(r.costing_mat)
    a, b = tab.codes(s1), tab.codes(s2)
    big = (tab.max_cost + 1) * 200_000
    row0, col0 = core.boundary(tab, a, b, r.gap_open_cost, big)
    assert r.cost == int(min(core.fill_score(tab, a, b, r.gap_open_cost, row0, col0)))
    assert r.seq_1_aligned.replace("-", "") == s1 and r.seq_2_aligned.replace("-", "") == s2
    assert _rescore(r) == r.cost


# ---------------------------------------------------------------- bench workloads vs the oracle's cost goldens
@pytest.mark.parametrize("name", ["c2", "c5", "c3", "c4", "c4tb"])
def test_bench_workload_cost_matches_golden(ga, name):
    """Each bench.py workload at its full BASELINE size (C4 = 10^12 cells, score only) against the cost
    the threaded C oracle produced (tests/golden/make_cost_golden.py, make_c4_golden.py); traceback
    workloads also walk, must reproduce both inputs, and must equal the oracle's alignment strings and
    final random state (tests/golden/make_aln_golden.py: <name>_aln.json digests, random.seed(0)).  c4tb: C4 with
    full traceback on one GPU (the recompute walk), its 1,222,001-column alignment pinned by the oracle's
    checkpoint-and-recompute walk (gao_align_ckpt)."""
    import bench
    from globalign_amd import _native
    wl = bench.WORKLOADS[name]
    gold = json.load(open(os.path.join(GOLDEN, f"{wl.get('golden', name)}_cost.json")))["cost"]
    s1, s2 = bench.workload_pair(wl)
    tables, _ = bench.problem_tables(s1, s2, wl["scoring"])
    eng = _native.Engine(0)
    try:
        eng.load(tables.codes(s1), tables.codes(s2), tables)
        if wl["traceback"]:
            random.seed(0)
            mt = np.array(random.getstate()[1], dtype=np.uint32)
            cost, (a, mid, b), status, mt_after = eng.align(mt, s1, s2)
            assert status == 0 and a.replace("-", "") == s1 and b.replace("-", "") == s2
            pin = os.path.join(GOLDEN, f"{name}_aln.json")
            if os.path.exists(pin):
                g = json.load(open(pin))
                st = random.getstate()
                assert len(mid) == g["aln_len"]
                assert aln_digest(a, mid, b) == g["aln_sha16"]
                assert state_digest((st[0], tuple(int(x) for x in mt_after), st[2])) == g["state_sha32"]
        else:
            cost = eng.fill(traceback=False)[0]
    finally:
        eng.close()
    assert int(cost) == gold


@pytest.mark.parametrize("div,lens", [(0.0, (3000, 3400)), (0.05, (4000, 4000)), (0.3, (2500, 2000))])
def test_similar_pairs_vs_oracle(ga, monkeypatch, div, lens):
    """Similar pairs from draw_two_random_seqs (reference start.py:724-867): long diagonal runs with
    sparse indels, the opposite of the i.i.d. inputs -- long match streaks through the walk."""
    from globalign_amd.random_seqs import draw_two_random_seqs
    orig = random.seed
    monkeypatch.setattr(random, "seed", lambda a=None, version=2: orig(4242 if a is None else a, version))
    s1, s2 = draw_two_random_seqs(list("ACGT"), lens[0], lens[0], lens[1], lens[1], div, 41, 42)
    monkeypatch.setattr(random, "seed", orig)
    _oracle_case(ga, s1, s2, dict(match_score=2, mismatch_score=-3, gap_open_score=-5, gap_extension_score=-1),
                 seed=int(div * 100) + 1)


# ---------------------------------------------------------------- the walker's lane select
@pytest.mark.parametrize("n", [5000, 40_000])
def test_walk_long_diagonal_runs_index_carries(ga, n):
    """The walker advances its v_readlane lane select unmasked: the index's low byte is the window offset and its
    upper bytes carry every move's advance (0x080109 >> 8L, ga_walk.h), which the lane select ignores (only its low
    6 bits count; tools/micro/readlane_idx2.hip).  A pure-diagonal path -- identical sequences, no tie anywhere, every
    move 0x080109 -- sets those upper bytes on every readlane of the walk: the alignment must be n matches and the
    random state the one n dispatches (18 draws each, globaligner.py:595-685) leave.  5000: the stored-words walk;
    40 000: the recompute walk."""
    s = _fast_splitmix(n, 77)
    kw = dict(match_score=2, mismatch_score=-3, gap_open_score=-5, gap_extension_score=-1)
    random.seed(9)
    r = ga.GlobalAligner(max_seq_len_prod=None, **kw).align(s, s)
    after = random.getstate()
    assert r.cost == 0 and r.score == 2 * n
    assert r.middle_part == "|" * n and r.seq_1_aligned == s and r.seq_2_aligned == s
    random.seed(9)
    sizes = (3, 2, 2, 2, 3, 2, 2, 2, 3) * 2
    for _ in range(n):
        for k in sizes:
            random.choice(range(k))
    assert after == random.getstate()


@pytest.mark.parametrize("every,ins", [(97, False), (53, True)])
def test_walk_diagonal_runs_with_gaps_vs_oracle(ga, every, ins):
    """Long diagonal runs broken by single gaps (every 97th residue deleted / a residue inserted every 53rd): the
    index advances of up (0x08) and left (0x0801) moves between diagonal runs, against the oracle."""
    s1 = _fast_splitmix(6000, 78)
    if ins:
        s2 = "".join(c + ("G" if k % every == every - 1 else "") for k, c in enumerate(s1))
    else:
        s2 = "".join(c for k, c in enumerate(s1) if k % every != every - 1)
    _oracle_case(ga, s1, s2, dict(match_score=2, mismatch_score=-3, gap_open_score=-5, gap_extension_score=-1),
                 seed=every)
