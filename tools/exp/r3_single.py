"""Round 3: single-call timings (ga_problem_align) of C3 / C5 / C2 and score-only fills, per kernel.

    python tools/exp/r3_single.py [workload ...]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from globalign_amd import _native  # noqa: E402
import numpy as np  # noqa: E402

for wl in (sys.argv[1:] or ["c3"]):
    cfg = bench.WORKLOADS[wl]
    s1, s2 = bench.workload_pair(cfg)
    tables, _ = bench.problem_tables(s1, s2, cfg["scoring"])
    eng = _native.Engine(0)
    eng.load(tables.codes(s1), tables.codes(s2), tables)
    mt = np.random.RandomState(0).randint(0, 2**32, size=625, dtype=np.uint64).astype(np.uint32)
    mt[624] = 624
    for k in range(6):
        t0 = time.perf_counter()
        r = eng.align(mt, s1, s2)
        dt = (time.perf_counter() - t0) * 1e3
        print(wl, "align wall %.2f ms" % dt, "cost", r[0], "timings(fill, walk, table, wall)",
              {k: round(v, 3) for k, v in eng.timings().items()}, "kind", eng.fill_kind(), flush=True)
    if cfg["m"] * cfg["n"] <= 10**10:
        for k in range(3):
            cost, _ = eng.fill(traceback=False)
            print(wl, "score-only fill %.3f ms" % eng.kernel_ms()[0], "kind", eng.fill_kind(), flush=True)
