"""Round 6: the recompute walk's accounting at C3 (walker tile waits, tile loads, blocks recomputed and their time) per
config, each config a list of context options (GA_NAME=VALUE, comma-separated; knobs are read when a context is
created), e.g.

    python tools/exp/r6/rc_diag.py 100000 GA_LANE_COLS_PER_LANE=4 GA_LANE_COLS_PER_LANE=2,GA_RC_CONE=2"""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

import bench  # noqa: E402
from globalign_amd import _native  # noqa: E402

m = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000
cfgs = sys.argv[2:] or ["GA_RC=1"]
s1, s2 = bench.splitmix(m, 1), bench.splitmix(m, 2)
tables, _ = bench.problem_tables(s1, s2)
L = _native.load_library()
L.ga_debug_walk.argtypes = [C.c_void_p, C.c_void_p]
L.ga_debug_rc.argtypes = [C.c_void_p, C.c_void_p]
mt0 = np.random.RandomState(0).randint(0, 2**32, size=625, dtype=np.uint64).astype(np.uint32)
mt0[624] = 624
for cfg in cfgs:
    opts = dict(kv.split("=", 1) for kv in cfg.split(",") if kv)
    opts.setdefault("GA_RC", "1")
    eng = _native.Engine(0, options=opts)
    eng.load(tables.codes(s1), tables.codes(s2), tables)
    for rep in range(3):
        r = eng.align(mt0, s1, s2)
        t = eng.timings()
        w = np.zeros(8, dtype=np.int32)
        L.ga_debug_walk(eng._h, w.ctypes.data)
        rc = np.zeros(4, dtype=np.uint32)
        L.ga_debug_rc(eng._h, rc.ctypes.data)
        steps = len(r[1][0])
        print(f"{cfg} steps={steps} ns_per_step={t['walk_ms'] * 1e6 / steps:.1f} fill={t['fill_ms']:.3f} "
              f"walk={t['walk_ms']:.3f} call={t['call_ms']:.3f} kind={eng.fill_kind()} waits={w[0]} tiles={w[1]} "
              f"t_tile_ms={w[2] / 1e5:.3f} t_total_ms={w[4] / 1e5:.3f} loads={w[7]} load_us_avg={w[6] / max(w[7], 1) / 100:.2f} "
              f"| rc blocks={rc[2]} block_us_avg={rc[3] / max(rc[2], 1) / 100:.2f}", flush=True)
    eng.close()
