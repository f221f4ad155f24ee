"""Diagnostic: per tile the traceback walker needs, how long it waited (s_memrealtime, 100 MHz).

    python tools/walk_tiles.py [m] [n]
Prints wait statistics split by the move that led into the tile (diagonal / up / left / same)."""
import ctypes as C
import json
import os
import random
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from globalign_amd import _native  # noqa: E402

m = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000
n = int(sys.argv[2]) if len(sys.argv) > 2 else 100_000
s1, s2 = bench.splitmix(m, 1), bench.splitmix(n, 2)
tables, _ = bench.problem_tables(s1, s2)
eng = _native.Engine(0)
eng.load(tables.codes(s1), tables.codes(s2), tables)
L = _native.load_library()
L.ga_debug_stamps.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_int64]
L.ga_debug_walk_tiles.argtypes = [C.c_void_p, C.c_void_p]
L.ga_debug_stamps(eng._h, 1, None, 0)
random.seed(0)
eng.align(np.array(random.getstate()[1], dtype=np.uint32), s1, s2)
rec = np.zeros(4 * 8192, dtype=np.uint32)
L.ga_debug_walk_tiles(eng._h, rec.ctypes.data)
rec = rec.reshape(-1, 4)
rec = rec[rec[:, 0] != 0xFFFFFFFF].astype(np.int64)
ti, tj, D, wt = rec[:, 0], rec[:, 1], rec[:, 2], rec[:, 3] / 100.0  # us
out = {"needs": int(len(rec)), "waited": int((wt > 0.05).sum()), "wait_us_total": float(wt.sum()),
       "walk_ms": eng.timings()["walk_ms"]}
# classify each need by its relation to the previous need
kinds = {}
for k in range(1, len(rec)):
    di, dj = ti[k - 1] - ti[k], tj[k - 1] - tj[k]
    key = f"d({di},{dj})"
    e = kinds.setdefault(key, [0, 0.0, 0])
    e[0] += 1
    e[1] += wt[k]
    e[2] += int(wt[k] > 0.05)
out["by_relation"] = {k: {"count": v[0], "wait_us": round(v[1], 1), "waited": v[2]} for k, v in
                      sorted(kinds.items(), key=lambda kv: -kv[1][1])[:12]}
# wait distribution
out["wait_us_percentiles"] = {p: float(np.percentile(wt, p)) for p in (50, 75, 90, 99)}
out["first_20"] = [[int(a), int(b), int(c), round(float(d), 2)] for a, b, c, d in zip(ti[:20], tj[:20], D[:20], wt[:20])]
print(json.dumps(out, indent=1))
