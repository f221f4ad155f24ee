"""Diagnostic: per-stripe timestamps of one fill (s_memrealtime, 100 MHz).

    python tools/fill_stamps.py [m] [n] [--tb]
Prints the stripe start lag (ramp), per-stripe duration and the implied time per row."""
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
eng.fill(traceback=tb)
L.ga_debug_stamps(eng._h, 1, None, 0)
cost, _ = eng.fill(traceback=tb)
L.ga_debug_geometry.argtypes = [C.c_void_p, C.c_void_p]
geo = np.zeros(4, dtype=np.int32)
L.ga_debug_geometry(eng._h, geo.ctypes.data)
T, ns, nwc = int(geo[0]), int(geo[1]), int(geo[2])
buf = np.zeros(8 * ns, dtype=np.uint64)
L.ga_debug_stamps(eng._h, 0, buf.ctypes.data, buf.size)
st = buf.reshape(ns, 8).astype(np.int64)
t0 = st[:, 0].min()
start, mid, end = (st[:, 0] - t0) / 100.0, (st[:, 1] - t0) / 100.0, (st[:, 2] - t0) / 100.0  # microseconds
f_ms = eng.kernel_ms()[0]
dur = end - start
step_ns = dur * 1e3 / m
out = {
    "m": m, "n": n, "tb": tb, "cost": cost, "fill_kernel_ms": f_ms, "nstripes": ns,
    "last_stripe_start_us": float(start[-1]), "last_end_us": float(end.max()),
    "lag_per_stripe_us_mean": float(np.mean(np.diff(start))),
    "lag_intra_slab_us": float(np.mean([start[k + 1] - start[k] for k in range(ns - 1) if (k + 1) % nwc != 0])),
    "lag_cross_slab_us": float(np.mean([start[k + 1] - start[k] for k in range(ns - 1) if (k + 1) % nwc == 0])),
    "stripe_duration_us_median": float(np.median(dur)),
    "row_ns_median": float(np.median(step_ns)),
    "first_half_vs_second_half": float(np.median((mid - start) / np.maximum(end - mid, 1e-9))),
    "start_us_samples": [float(x) for x in start[:: max(1, ns // 12)]],
    "latest_ends": [[int(k), round(float(start[k]), 1), round(float(end[k]), 1)] for k in np.argsort(end)[-5:]],
    "max_start_us": float(start.max()),
    "row_ns_samples": [round(float(x), 1) for x in step_ns[:: max(1, ns // 12)]],
    "wait_frac_samples": [round(float(x), 3) for x in (st[:: max(1, ns // 12), 4] / np.maximum(st[:: max(1, ns // 12), 3], 1))],
    # shader clocks (s_memtime) over the same span as end - start: the in-kernel clock and cycles per row
    "clock_ghz_median": float(np.median(st[:, 3] / np.maximum(dur * 1e3, 1e-9))),
    "cycles_per_row_median": float(np.median(st[:, 3] / m)),
    "first_stripes_row_ns": [float(x) for x in step_ns[:10]],
    "row_ns_min": float(np.min(step_ns)),
    "cols_per_lane": T, "nwc": nwc,
    # blocked stripes (T > 1): shader clocks waiting for edges in / ring space out / the profile
    "wait_frac_edges_in": float(np.median(st[:, 4] / np.maximum(st[:, 3], 1))),
    "wait_frac_ring_out": float(np.median(st[:, 5] / np.maximum(st[:, 3], 1))),
    "wait_frac_profile": float(np.median(st[:, 6] / np.maximum(st[:, 3], 1))),
    "sleeps_per_row": float(np.median(st[:, 7] / m)),
    # by position in the workgroup chain: the waves that wait least set the chain's pace
    "wait_frac_edges_in_by_wave": [round(float(np.median(st[k::nwc, 4] / np.maximum(st[k::nwc, 3], 1))), 3)
                                   for k in range(nwc)],
    "cycles_per_row_by_wave": [round(float(np.median(st[k::nwc, 3] / m)), 1) for k in range(nwc)],
}
# one align for the walk diagnostics
import random  # noqa: E402
random.seed(0)
if tb:
    eng.align(np.array(random.getstate()[1], dtype=np.uint32), s1, s2)
    L.ga_debug_walk.argtypes = [C.c_void_p, C.c_void_p]
    w2 = np.zeros(8, dtype=np.int32)
    L.ga_debug_walk(eng._h, w2.ctypes.data)
    out["walk"] = dict(eng.timings(), tile_wait_sleeps=int(w2[0]), tiles=int(w2[1]),
                       tile_wait_us=float(w2[2]) / 100.0, ring_wait_us=float(w2[3]) / 100.0,
                       walker_us=float(w2[4]) / 100.0, walker_cycles=int(w2[5]), load_ticks=int(w2[6]),
                       loads=int(w2[7]))
print(json.dumps(out))
