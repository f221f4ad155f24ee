"""Pins the cost of a bench workload (BASELINE configs, SplitMix64 inputs, bench.WORKLOADS) with the C
oracle's score-only fill on host threads:

    python tests/golden/make_cost_golden.py c3 [threads]   ->  tests/golden/c3_cost.json

The oracle is pinned by the reference's own fixtures (tests/test_oracle.py); this runs it at sizes the
reference cannot reach (C3 is 10^10 cells, C4 10^12).  Test infrastructure: never shipped or imported by
the product path (bench.py only reads the committed JSON to report cost_matches_oracle)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from oracle import core, transform  # noqa: E402
from tests.conftest import load_matrix  # noqa: E402


def cost_of(wl, threads):
    s1, s2 = bench.workload_pair(wl)
    name = wl["scoring"].get("scoring_mat_name")
    blosum = load_matrix(name) if name else None
    _, _, _, cmat, _, goc = transform.settings(dict(wl["scoring"], seq_1=s1[:64], seq_2=s2[:64]), blosum=blosum)
    tab = core.Tables(cmat)
    a, b = tab.codes(s1), tab.codes(s2)
    big = (tab.max_cost + 1) * max(wl["m"], wl["n"])
    row0, col0 = core.boundary(tab, a, b, goc, big)
    return int(min(core.fill_score_parallel(tab, a, b, goc, row0, col0, threads)))


if __name__ == "__main__":
    name = sys.argv[1] if len(sys.argv) > 1 else "c3"
    threads = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    wl = bench.WORKLOADS[name]
    t0 = time.time()
    cost = cost_of(wl, threads)
    rec = {"workload": wl["desc"], "m": wl["m"], "n": wl["n"], "cost": cost,
           "oracle": "oracle/ga_oracle.c gao_fill_score_parallel (gao_cell per cell)", "threads": threads,
           "seconds": round(time.time() - t0, 1)}
    print(json.dumps(rec))
    json.dump(rec, open(os.path.join(ROOT, "tests", "golden", f"{name}_cost.json"), "w"), indent=1)
