"""Diagnostic: one full alignment of a bench workload and the walker's own accounting.

    python tools/walk_diag.py [c3|c5|c2]
Prints fill / walk / tie-break ms and the walk kernel's tile-wait, ring-wait, tile loads and clock."""
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

name = sys.argv[1] if len(sys.argv) > 1 else "c5"
wl = bench.WORKLOADS[name]
s1, s2 = bench.workload_pair(wl)
tables, _ = bench.problem_tables(s1, s2, wl["scoring"])
eng = _native.Engine(0)
eng.load(tables.codes(s1), tables.codes(s2), tables)
random.seed(0)
mt = np.array(random.getstate()[1], dtype=np.uint32)
out = []
for _ in range(3):
    cost, strings, status, _ = eng.align(mt, s1, s2)
    L = _native.load_library()
    L.ga_debug_walk.argtypes = [C.c_void_p, C.c_void_p]
    w = np.zeros(8, dtype=np.int32)
    L.ga_debug_walk(eng._h, w.ctypes.data)
    steps = len(strings[0])
    out.append(dict(eng.timings(), cost=int(cost), steps=steps, tile_wait_sleeps=int(w[0]), tiles=int(w[1]),
                    tile_wait_us=w[2] / 100.0, ring_wait_us=w[3] / 100.0, walker_us=w[4] / 100.0,
                    walker_clk_per_step=float(w[5]) * 16 / max(1, steps), loads=int(w[7]),
                    load_us_per_tile=float(w[6]) / 100.0 / max(1, int(w[7]))))
print(json.dumps({"workload": name, "runs": out}))
