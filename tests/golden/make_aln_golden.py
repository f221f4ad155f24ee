"""Pins the full-size ALIGNMENT of a traceback bench workload with the C oracle (sets fill + walk):

    python tests/golden/make_aln_golden.py c3   ->  tests/golden/c3_aln.json   (10^10 cells, ~20 GB of sets)
    python tests/golden/make_aln_golden.py c5   ->  tests/golden/c5_aln.json
    python tests/golden/make_aln_golden.py c4tb ->  tests/golden/c4tb_aln.json (10^12 cells: the checkpoint-and-
        recompute walk gao_align_ckpt on 8 threads, 12 GB of row / column checkpoints, ~20 min here)

The walk runs under random.seed(0) exactly as bench.py / the GPU test do; the record holds the
alignment length, the sha256 digests of the three strings (tests/conftest.py aln_digest) and of the
random state afterwards (state_digest), plus the cost.  The oracle restates dp_array_backward
(globaligner.py:395-593) and is pinned by the reference's own fixtures up to 10k x 10k
(tests/test_oracle.py, golden/splitmix.json).  Test infrastructure only."""
import json
import os
import random
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from oracle import core, transform  # noqa: E402
from tests.conftest import aln_digest, load_matrix, state_digest  # noqa: E402


def aln_record(name):
    wl = bench.WORKLOADS[name]
    s1, s2 = bench.workload_pair(wl)
    mat = wl["scoring"].get("scoring_mat_name")
    _, _, _, cmat, _, goc = transform.settings(dict(wl["scoring"], seq_1=s1[:64], seq_2=s2[:64]),
                                               blosum=load_matrix(mat) if mat else None)
    random.seed(0)
    t0 = time.time()
    # 10^12 cells (C4 with full traceback): no m x n sets; the checkpoint-and-recompute walk, which reproduces the
    # sets walk's C3 alignment and random state exactly (tests/test_oracle.py runs it on every reference-run case)
    ckpt = wl["m"] * wl["n"] > 10**11
    mode = "ckpt" if ckpt else "sets"
    r = core.align(s1, s2, cmat, goc, core.mt_state_array(), mode=mode, threads=int(os.environ.get("ORACLE_THREADS", 8)))
    a, mid, b = r["strings"]
    st = random.getstate()
    after = (st[0], tuple(int(x) for x in r["mt_out"]), st[2])
    return {"workload": wl["desc"], "m": wl["m"], "n": wl["n"], "seed": 0, "cost": r["cost"],
            "status": r["status"], "ndispatch": r["ndispatch"], "aln_len": len(mid),
            "aln_sha16": aln_digest(a, mid, b), "state_sha32": state_digest(after),
            "oracle": "oracle/ga_oracle.c " + ("gao_align_ckpt (4096 x 4096 tiles)" if ckpt else
                                               "gao_fill_sets + gao_traceback_sets"),
            "seconds": round(time.time() - t0, 1)}


if __name__ == "__main__":
    name = sys.argv[1] if len(sys.argv) > 1 else "c5"
    rec = aln_record(name)
    print(json.dumps(rec))
    json.dump(rec, open(os.path.join(ROOT, "tests", "golden", f"{name}_aln.json"), "w"), indent=1)
