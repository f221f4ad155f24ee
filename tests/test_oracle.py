"""Pin the CPU oracle against the reference's own golden vectors (CPU only).

The oracle (oracle/) is the checker for every GPU parity test, so it is
itself checked here against fixtures that were produced by running the
reference (tests/golden/make_golden.py):
  * kat.json          -- the reference test-suite's known answers
                         (tests/globaligner_test.py:6-37, :40-383) and the
                         tutorial's (reference/tutorial.qmd:10-24, :126-150)
  * random_api.json   -- 700 random find_global_alignment calls incl.
                         degenerate lengths that raise IndexError (A.5)
  * random_fill.json  -- dp_array_forward on arbitrary boundaries
  * splitmix.json     -- SURVEY 8d synthetic configs (1k, 2k, 10k)
"""
import json
import os
import random

import numpy as np
import pytest

from oracle import core, transform
from tests.conftest import GOLDEN, load_matrix, state_digest


def _smat_for(rec):
    kw = rec["kwargs"]
    if kw.get("scoring_mat_name"):
        return load_matrix(kw["scoring_mat_name"]), None
    if "mtx" in rec:
        return None, transform.read_mtx_rows(rec["mtx"]["letters"], rec["mtx"]["scores"])
    return None, None


def _run_oracle(rec, mode="auto", **kw):
    blosum, mtx = _smat_for(rec)
    s1, s2, smat, cmat, gos, goc = transform.settings(rec["kwargs"], blosum=blosum, mtx=mtx)
    random.seed(rec["seed"])
    res = core.align(s1, s2, cmat, goc, core.mt_state_array(), mode=mode, **kw)
    res["score"] = transform.cost_to_score(res["cost"], len(s1), len(s2), transform.max_val(smat))
    res["smat"], res["cmat"], res["gos"], res["goc"] = smat, cmat, gos, goc
    return res


def _check(rec, res):
    digest = state_digest(core.mt_state_tuple(res["mt_out"]))
    assert res["ndispatch"] * 18 == rec["choices"]
    assert digest == rec["state_after"]
    if "error" in rec:
        assert res["status"] == rec["error"]
        return
    assert res["status"] == "ok"
    assert res["cost"] == rec["cost"]
    assert res["score"] == rec["score"]
    assert res["strings"] == (rec["seq_1_aligned"], rec["middle_part"], rec["seq_2_aligned"])
    if "costing_mat" in rec:
        assert res["cmat"] == rec["costing_mat"]
        assert res["smat"] == rec["scoring_mat"]
    assert res["gos"] == rec["gap_open_score"] and res["goc"] == rec["gap_open_cost"]


def test_oracle_kat_api():
    kat = json.load(open(os.path.join(GOLDEN, "kat.json")))
    for rec in kat["api"]:
        _check(rec, _run_oracle(rec))
    # the reference test-suite's own expected (score, cost) pairs
    expected = [(-1, 7), (-9, 24), (-15, 56), (-21, 62), (-20, 102), (-18, 28), (-18, 26), (-21, 31), (-21, 31),
                (0, 7), (-2, 8)]
    assert [(r["score"], r["cost"]) for r in kat["api"]] == expected


def test_oracle_kat_fill():
    rec = json.load(open(os.path.join(GOLDEN, "kat.json")))["fill"]
    _check_fill(rec)


def _check_fill(rec):
    tab = core.Tables(rec["costing_mat"])
    a, b = tab.codes(rec["seq_1"]), tab.codes(rec["seq_2"])
    m, n = len(a), len(b)
    dp = np.zeros((m + 1, n + 1, 3), np.int64)
    for i in range(m + 1):
        for j in range(n + 1):
            if i == 0 or j == 0:
                dp[i, j] = rec["dp_in"][i][j]
    core.fill_full(tab, a, b, rec["gap_open_cost"], dp)
    assert dp.tolist() == rec["dp_out"]


def test_oracle_random_fill():
    for rec in json.load(open(os.path.join(GOLDEN, "random_fill.json"))):
        _check_fill(rec)


@pytest.mark.parametrize("mode", ["full", "sets", "ckpt"])
def test_oracle_random_api(mode):
    """Every reference-run API case through each walk of the oracle; "ckpt" (the checkpoint-and-recompute walk that
    pins the C4 full-traceback alignment, gao_align_ckpt) with tiny tiles and three threads, so that walks cross many
    tiles and the forward pass many slab boundaries."""
    cases = json.load(open(os.path.join(GOLDEN, "random_api.json")))
    n_err = 0
    kw = dict(threads=3, tile=(3, 5)) if mode == "ckpt" else {}
    for rec in cases:
        if "error" in rec and rec["error"] != "IndexError":
            continue  # validation errors are host-side, checked in test_api.py
        n_err += "error" in rec
        _check(rec, _run_oracle(rec, mode=mode, **kw))
    assert n_err >= 3  # the degenerate IndexError quirk is exercised


@pytest.mark.parametrize("mode,okw", [("sets", {}), ("ckpt", dict(threads=4, tile=(61, 97))), ("ckpt", dict(threads=1, tile=(1000, 7)))])
def test_oracle_splitmix(mode, okw):
    for rec in json.load(open(os.path.join(GOLDEN, "splitmix.json"))):
        if rec["m"] * rec["n"] > 5_000_000:
            continue  # 10k x 10k is pinned in the GPU suite (needs ~2 GB of traceback sets)
        from tests.conftest import splitmix_seq
        s1 = splitmix_seq(rec["m"], rec["seeds"][0], rec["alphabet"])
        s2 = splitmix_seq(rec["n"], rec["seeds"][1], rec["alphabet"])
        kw = dict(rec["kwargs"], seq_1=s1, seq_2=s2)
        r = dict(rec, kwargs=kw)
        res = _run_oracle(r, mode=mode, **okw)
        a, mid, b = res["strings"]
        assert res["cost"] == rec["cost"] and res["score"] == rec["score"]
        assert len(mid) == rec["aln_len"]
        from tests.conftest import aln_digest
        assert aln_digest(a, mid, b) == rec["aln_sha16"]
        assert res["ndispatch"] * 18 == rec["choices"]
        assert state_digest(core.mt_state_tuple(res["mt_out"])) == rec["state_after"]


def test_mt_emulation_matches_cpython():
    """random.choice on sizes 2/3 == oracle's MT19937 + _randbelow emulation."""
    sizes = np.array([3, 2, 2, 2, 3, 2, 2, 2, 3] * 2 * 300, dtype=np.int32)
    for seed in (0, 1, 12345):
        random.seed(seed)
        st = core.mt_state_array()
        want = [random.choice(range(s)) for s in sizes]
        got = np.zeros(len(sizes), np.int32)
        core.lib().gao_mt_draws(st, len(sizes), sizes, got)
        assert got.tolist() == want
        assert state_digest(core.mt_state_tuple(st)) == state_digest()


def test_pyport_matches_oracle():
    """The CPU-baseline port (oracle/pyport.py) computes the same alignments as the oracle."""
    from oracle import pyport
    rng = random.Random(42)
    for k in range(60):
        s1 = "".join(rng.choice("ACGT") for _ in range(rng.randint(2, 60)))
        s2 = "".join(rng.choice("ACGT") for _ in range(rng.randint(2, 60)))
        kw = dict(seq_1=s1, seq_2=s2, match_score=2, mismatch_score=-3, gap_open_score=-rng.randint(0, 8),
                  gap_extension_score=-1)
        _, _, smat, cmat, gos, goc = transform.settings(kw)
        random.seed(k)
        ref = core.align(s1, s2, cmat, goc, core.mt_state_array())
        random.seed(k)
        T = pyport.fill(s1, s2, cmat, goc, transform.max_val(cmat))
        a, mid, b, cost = pyport.traceback(T, s1, s2, cmat, goc)
        assert cost == ref["cost"] and (a, mid, b) == ref["strings"]
        assert state_digest() == state_digest(core.mt_state_tuple(ref["mt_out"]))


def test_oracle_reproduces_c2_cost_golden():
    """The threaded score-only fill that pins the bench workloads' costs (tests/golden/*_cost.json),
    re-run at C2 (10^8 cells, well under a second)."""
    import json
    import os
    from tests.golden.make_cost_golden import cost_of
    import bench
    gold = json.load(open(os.path.join(GOLDEN, "c2_cost.json")))["cost"]
    assert cost_of(bench.WORKLOADS["c2"], 4) == gold
