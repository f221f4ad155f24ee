"""Pins the C4 cost (1M x 1M DNA, SplitMix64 seeds 1/2, match 2 / mismatch -3 / open -5 / ext -1,
BASELINE configs[3]) with the C oracle's score-only fill on host threads.

    python tests/golden/make_c4_golden.py [side] [threads]   ->  tests/golden/c4_cost.json

The oracle is pinned by the reference's own fixtures (tests/test_oracle.py); this only runs it at a size
the reference itself cannot reach (~10^12 cells).  Test infrastructure: never shipped or imported by the
product path."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from oracle import core, transform  # noqa: E402


def cost_of(side, threads, seeds=(1, 2)):
    s1, s2 = bench.splitmix(side, seeds[0]), bench.splitmix(side, seeds[1])
    _, _, _, cmat, _, goc = transform.settings(dict(bench.SCORING, seq_1=s1[:64], seq_2=s2[:64]))
    tab = core.Tables(cmat)
    a, b = tab.codes(s1), tab.codes(s2)
    big = (tab.max_cost + 1) * side
    row0, col0 = core.boundary(tab, a, b, goc, big)
    last = core.fill_score_parallel(tab, a, b, goc, row0, col0, threads)
    return int(min(last))


if __name__ == "__main__":
    side = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
    threads = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    t0 = time.time()
    cost = cost_of(side, threads)
    rec = {"config": "C4" if side == 1_000_000 else f"{side}x{side}", "m": side, "n": side, "seeds": [1, 2],
           "scoring": bench.SCORING, "cost": cost, "score": 2 * side - cost,
           "oracle": "oracle/ga_oracle.c gao_fill_score_parallel (gao_cell per cell)", "threads": threads,
           "seconds": round(time.time() - t0, 1)}
    print(json.dumps(rec))
    if side == 1_000_000:
        json.dump(rec, open(os.path.join(ROOT, "tests", "golden", "c4_cost.json"), "w"), indent=1)
