"""Diagnostic: time K fills of an m x n SplitMix64 DNA pair (score only or with traceback words).

    python tools/fill_sweep.py m n K tb(0|1)

Prints one JSON line: cost, per-launch fill ms (HIP events), cells/s.  Used to sweep launch
settings given through the environment (GA_FILL_MODE, GA_LANE_COLS_PER_LANE, GA_FILL_NWC,
GA_FILL_LDS_FLOOR)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from globalign_amd import _native  # noqa: E402

m, n, K, tb = (int(x) for x in sys.argv[1:5])
s1, s2 = bench.splitmix(m, 1), bench.splitmix(n, 2)
tables, _ = bench.problem_tables(s1, s2)
eng = _native.Engine(0)
eng.load(tables.codes(s1), tables.codes(s2), tables)
ms = []
for _ in range(K):
    cost, _ = eng.fill(traceback=bool(tb))
    ms.append(eng.kernel_ms()[0])
best = min(ms[1:] if K > 1 else ms)
print(json.dumps({"m": m, "n": n, "tb": tb, "kind": eng.fill_kind(), "mode": os.environ.get("GA_FILL_MODE"),
                  "floor": os.environ.get("GA_FILL_LDS_FLOOR"), "cost": int(cost),
                  "fill_ms": ms, "best_cells_per_s": m * n / (best * 1e-3)}), flush=True)
