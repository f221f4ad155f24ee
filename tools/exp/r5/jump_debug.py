"""Round 5 diagnostics: the tie-to-tie walk on a small problem; its entry cache (every block resident) against the
CPU emulation of the workers' build (tools/jump_model.py semantics, the kernel's LUT / selector encoding), and its
alignment against the oracle.  python tools/exp/r5/jump_debug.py [N]"""
import ctypes as C
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

import bench  # noqa: E402
from globalign_amd import _native  # noqa: E402
from oracle import core, transform  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 256
os.environ["GA_RC"] = "1"
os.environ["GA_RC_JUMP"] = "1"
wl = bench.WORKLOADS["c3"]
s1, s2 = bench.workload_pair(dict(wl, m=N, n=N))
tables, _ = bench.problem_tables(s1, s2)
eng = _native.Engine(0)
eng.load(tables.codes(s1), tables.codes(s2), tables)
random.seed(0)
mt = np.array(random.getstate()[1], dtype=np.uint32)
cost, strings, status, mt_after = eng.align(mt, s1, s2)
print("kind", eng.fill_kind(), "walk", eng.walk_kind(), "cost", cost)
TD = eng.fill_kind()[1]
L = _native.load_library()
L.ga_debug_rc_cache.argtypes = [C.c_void_p, C.c_void_p, C.c_int64]
nb = 32 * 32 * 4 * TD * 6144
buf = np.zeros(nb, dtype=np.uint8)
_native._check(L.ga_debug_rc_cache(eng._h, buf.ctypes.data, nb))
ent = buf.view(np.uint16)


def gpu_entry(p, i, j):
    ti, tj = (i - 1) >> 5, (j - 1) >> 5
    bi, tr, td2 = ti >> 1, ti & 1, 2 * TD
    bs, tc = tj // td2, tj % td2
    tile = ((bi % 32) * 32 + bs % 32) * (2 * td2) + tr * td2 + tc
    return int(ent[tile * 3072 + p * 1024 + ((i - 1) & 31) * 32 + ((j - 1) & 31)])


# CPU emulation of the build (as /tmp/emu.py)
sys.argv = [sys.argv[0], str(N)]
_, _, _, cmat, _, o = transform.settings(dict(wl["scoring"], seq_1=s1[:64], seq_2=s2[:64]))
tab = core.Tables(cmat)
a, b = tab.codes(s1), tab.codes(s2)
m, n = len(a), len(b)
big = (tab.max_cost + 1) * max(m, n)
row0, col0 = core.boundary(tab, a, b, o, big)
dp = np.zeros((m + 1, n + 1, 3), np.int64)
dp[0, :, :] = row0.reshape(n + 1, 3)
dp[:, 0, :] = col0.reshape(m + 1, 3)
core.fill_full(tab, a, b, o, dp)


def perm(x, y, sel):
    src = [(y >> (8 * k)) & 0xff for k in range(4)] + [(x >> (8 * k)) & 0xff for k in range(4)]
    out = 0
    for k in range(4):
        s = (sel >> (8 * k)) & 0xff
        out |= (src[s] if s < 8 else (0 if s == 12 else 0xff)) << (8 * k)
    return out


def lut_entry(idx):
    fx, fy, zM, mm = idx & 15, (idx >> 4) & 15, ((idx >> 8) & 1) ^ 1, (idx >> 9) & 1
    zX, zY = int(fx == 0), int(fy == 0)
    leX, geX, leY, geY = int(fx <= o), int(fx >= o), int(fy <= o), int(fy >= o)
    S = [zM | (zX << 1) | (zY << 2), (zM & geX) | (leX << 1) | ((zY & geX) << 2), (zM & geY) | ((zX & geY) << 1) | (leY << 2)]
    sel, tw = [], []
    for x in S:
        if x in (1, 2, 4):
            sel.append({1: 0x0504, 2: 0x0706, 4: 0x0100}[x])
            tw.append(0)
        else:
            sel.append(0x0c0c)
            tw.append(((2 * x - 2 + 14 * mm) << 2) if x else 0x7c)
    return (sel[0] | (sel[1] << 16), sel[2] | (0x0c0c << 16), tw[0] | (tw[1] << 16), tw[2])


LUT = [lut_entry(q) for q in range(1024)]
SC = 64 * TD
bad = 0
shown = 0
for R0 in range(0, m, 64):
    for j0 in range(0, n, SC):
        e0p, e1, e2p = {}, {}, {}
        for i in range(R0 + 1, min(R0 + 64, m) + 1):
            for j in range(j0 + 1, min(j0 + SC, n) + 1):
                M, X, Y = (int(v) for v in dp[i, j])
                H = min(M, X, Y)
                idx = min(X - H, o + 1) | (min(Y - H, o + 1) << 4) | (min(M - H, 1) << 8) | (int(a[i - 1] != b[j - 1]) << 9)
                f = LUT[idx]
                Pd = ((e0p.get((i - 1, j - 1), 0) << 2) | 3)
                Pl = ((e1.get((i, j - 1), 0) << 2) | 1)
                Pu = ((e2p.get((i - 1, j), 0) << 2) | 2)
                src0 = perm(Pl & 0xffffffff, Pd & 0xffffffff, 0x05040100)
                E01, E2v = perm(src0, Pu & 0xffffffff, f[0]), perm(src0, Pu & 0xffffffff, f[1])
                S01, S2 = E01 | f[2], E2v | f[3]
                e0p[(i, j)], e1[(i, j)], e2p[(i, j)] = E01 & 0xffff, E01 >> 16, E2v
                exp = (S01 & 0xffff, S01 >> 16, S2 & 0xffff)
                got = tuple(gpu_entry(p, i, j) for p in range(3))
                if exp != got:
                    bad += 1
                    if shown < 12:
                        print(f"cell ({i},{j}) exp {[hex(x) for x in exp]} got {[hex(x) for x in got]}")
                        shown += 1
print("entries differing:", bad, "of", 3 * m * n)
random.seed(0)
r = core.align(s1, s2, cmat, o, core.mt_state_array())
print("strings equal:", tuple(strings) == tuple(r["strings"]), "cost", r["cost"])
ga, gm, gb = strings
ra, rm, rb = r["strings"]
q = next((k for k in range(min(len(gm), len(rm))) if (ga[k], gm[k], gb[k]) != (ra[k], rm[k], rb[k])), None)
print("first string difference at column", q, "of", len(rm))
