"""Diagnostic: per-step time of fill-kernel ablation variants (timing only; outputs garbage).

    python tools/fill_ablation.py [m] [n] [--tb]"""
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from globalign_amd import _native  # noqa: E402

m = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000
n = int(sys.argv[2]) if len(sys.argv) > 2 else 100_000
tb = "--tb" in sys.argv
s1, s2 = bench.splitmix(m, 1), bench.splitmix(n, 2)
tables, _ = bench.problem_tables(s1, s2)
eng = _native.Engine(0)
eng.load(tables.codes(s1), tables.codes(s2), tables)
L = _native.load_library()
L.ga_debug_stamps.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_int64]
L.ga_debug_ablation.argtypes = [C.c_void_p, C.c_int]
ns = (n + 63) // 64
res = {}
names = {0: "product", 1: "no_ring_write", 2: "no_dpp", 4: "no_ring_read", 8: "no_qp_load", 16: "no_waits",
         17: "no_waits+no_write", 21: "no_waits/write/read", 29: "no_waits/write/read/qp", 31: "all_off"}
for abl in [0, 1, 2, 4, 8, 16, 17, 21, 29, 31]:
    L.ga_debug_ablation(eng._h, abl)
    L.ga_debug_stamps(eng._h, 1, None, 0)
    eng.fill(traceback=tb)
    buf = np.zeros(4 * ns, dtype=np.uint64)
    L.ga_debug_stamps(eng._h, 0, buf.ctypes.data, buf.size)
    st = buf.reshape(ns, 4).astype(np.int64)
    dur = (st[:, 2] - st[:, 0]) / 100.0
    start = (st[:, 0] - st[:, 0].min()) / 100.0
    res[names[abl]] = dict(kernel_ms=round(eng.kernel_ms()[0], 3), step_ns=round(float(np.median(dur)) * 1e3 / (m + 63), 2),
                           lag_us=round(float(np.mean(np.diff(start))), 3))
L.ga_debug_ablation(eng._h, -1)
print(json.dumps({"m": m, "n": n, "tb": tb, "variants": res}))
