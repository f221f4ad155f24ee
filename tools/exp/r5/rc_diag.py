"""Round 5: the recompute walk's accounting at C3 (walker tile waits, tile loads, blocks recomputed and their time)
per GA_RC_SERVERS:GA_RC_WIN[:GA_RC_CONE] config, one context per config (knobs are read when a context is created).

    python tools/exp/r5/rc_diag.py [m] [servers:win[:cone] ...]"""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

import bench  # noqa: E402
from globalign_amd import _native  # noqa: E402

m = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000
cfgs = sys.argv[2:] or ["64:64"]
wl = bench.WORKLOADS.get(os.environ.get("RC_WL", ""))  # (RC_WL=c5: that workload's alphabet, seeds and scoring)
if wl:
    s1, s2 = bench.splitmix(m, wl["seeds"][0], wl["alphabet"]), bench.splitmix(m, wl["seeds"][1], wl["alphabet"])
    tables, _ = bench.problem_tables(s1, s2, wl["scoring"])
else:
    s1, s2 = bench.splitmix(m, 1), bench.splitmix(m, 2)
    tables, _ = bench.problem_tables(s1, s2)
L = _native.load_library()
L.ga_debug_walk.argtypes = [C.c_void_p, C.c_void_p]
L.ga_debug_rc.argtypes = [C.c_void_p, C.c_void_p]
L.ga_debug_walk_jump.argtypes = [C.c_void_p, C.c_void_p]
mt0 = np.random.RandomState(0).randint(0, 2**32, size=625, dtype=np.uint64).astype(np.uint32)
mt0[624] = 624
os.environ["GA_RC"] = "1"
for cfg in cfgs:
    ns, win, *rest = cfg.split(":")
    os.environ["GA_RC_SERVERS"] = ns
    os.environ["GA_RC_WIN"] = win
    os.environ["GA_RC_CONE"] = rest[0] if rest else "1"
    eng = _native.Engine(0)
    eng.load(tables.codes(s1), tables.codes(s2), tables)
    for rep in range(2):
        r = eng.align(mt0, s1, s2)
        t = eng.timings()
        w = np.zeros(8, dtype=np.int32)
        L.ga_debug_walk(eng._h, w.ctypes.data)
        rc = np.zeros(4, dtype=np.uint32)
        L.ga_debug_rc(eng._h, rc.ctypes.data)
        steps = len(r[1][0])
        jd = np.zeros(3, dtype=np.int32)
        L.ga_debug_walk_jump(eng._h, jd.ctypes.data)
        print(f"steps={steps} ns_per_step={t['walk_ms'] * 1e6 / steps:.1f} servers={ns} win={win} cone={os.environ['GA_RC_CONE']} fill={t['fill_ms']:.3f} "
              f"walk={t['walk_ms']:.3f} call={t['call_ms']:.3f} kind={eng.fill_kind()} waits={w[0]} tiles={w[1]} "
              f"t_tile_ms={w[2] / 1e5:.3f} t_total_ms={w[4] / 1e5:.3f} loads={w[7]} load_us_avg={w[6] / max(w[7], 1) / 100:.2f} "
              f"| rc blocks={rc[2]} block_us_avg={rc[3] / max(rc[2], 1) / 100:.2f} | jump trips={jd[0]} rechecks={jd[1]} ties={jd[2]} "
              f"moves_per_trip={steps / max(jd[0], 1):.2f} walk_ns_per_trip_ex_waits={(w[4] - w[2]) * 10.0 / max(jd[0], 1):.1f}", flush=True)
    eng.close()
