"""Diagnostic: where the traceback walk spends its time.

    python tools/walk_diag.py [m] [n] [reps]
Prints walk kernel ms, walker-side wait time on tiles and on the tie-break /
level rings (s_memrealtime), tiles entered and steps."""
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
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
s1, s2 = bench.splitmix(m, 1), bench.splitmix(n, 2)
tables, _ = bench.problem_tables(s1, s2)
eng = _native.Engine(0)
eng.load(tables.codes(s1), tables.codes(s2), tables)
L = _native.load_library()
L.ga_debug_walk.argtypes = [C.c_void_p, C.c_void_p]
random.seed(0)
mt0 = np.array(random.getstate()[1], dtype=np.uint32)
rows = []
for _ in range(reps):
    cost, (a, mid, b), st, _ = eng.align(mt0, s1, s2)
    tm = eng.timings()
    d = np.zeros(8, np.int32)
    L.ga_debug_walk(eng._h, d.ctypes.data)
    steps = len(a)
    rows.append(dict(walk_ms=tm["walk_ms"], fill_ms=tm["fill_ms"], rng_ms=tm["rng_ms"], call_ms=tm["call_ms"],
                     steps=steps, tile_spins=int(d[0]), tiles=int(d[1]), tile_wait_ms=d[2] / 1e5,
                     ring_wait_ms=d[3] / 1e5, walker_ms=d[4] / 1e5,
                     tiles_loaded=int(d[7]), us_per_tile_load=(d[6] / 100.0 / d[7]) if d[7] else None,
                     clock_mhz=d[5] * 16 / (d[4] / 1e5) / 1e3 if d[4] else None, ns_per_step=tm["walk_ms"] * 1e6 / steps))
print(json.dumps({"m": m, "n": n, "cost": cost, "runs": rows}, indent=1))
