"""C4 with full traceback through the recompute walk: walk time by recompute-worker count (GA_RC_SERVERS) or, with
"win" first, by recompute window (GA_RC_WIN)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

import bench  # noqa: E402
from globalign_amd import _native  # noqa: E402

wl = bench.WORKLOADS["c4tb"]
s1, s2 = bench.workload_pair(wl)
tables, _ = bench.problem_tables(s1, s2, wl["scoring"])
mt0 = np.random.RandomState(0).randint(0, 2**32, size=625, dtype=np.uint64).astype(np.uint32)
mt0[624] = 624
eng = _native.Engine(0)
eng.load(tables.codes(s1), tables.codes(s2), tables)
args = sys.argv[1:] or ["64", "96", "128", "192", "255"]
knob = "GA_RC_SERVERS"
if args[0] == "win":
    knob, args = "GA_RC_WIN", args[1:]
for ns in args:
    os.environ[knob] = ns
    for rep in range(2):
        cost, (a, mid, b), status, mt = eng.align(mt0, s1, s2)
        t = eng.timings()
        print(f"{knob}={ns} cost={cost} len={len(mid)} fill={t['fill_ms']:.1f} walk={t['walk_ms']:.1f} call={t['call_ms']:.1f}",
              flush=True)
eng.close()
