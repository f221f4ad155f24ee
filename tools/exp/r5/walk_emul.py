"""Round 5: CPU emulation of the walker's interior (ga_walk.h walk_body) with the u64 lane-delta table, against a plain
per-step walk over the same rank sets and table.  Test infrastructure (imports the oracle).

    python tools/exp/r5/walk_emul.py [m n seed]
"""
import ctypes as C
import os
import random
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, ROOT)
from oracle import core, transform  # noqa: E402
from tests.conftest import splitmix_seq  # noqa: E402

TV = (25, 17, 8)
M32, M64 = 0xffffffff, 0xffffffffffffffff


def tab_field(S, mm):
    return {1: 8, 2: 9, 4: 10}.get(S, 4 * mm + {3: 0, 5: 1, 6: 2, 7: 3}.get(S, 3))


def main(m=300, n=400, seed=5):
    DNA = dict(match_score=2, mismatch_score=-3, gap_open_score=-5, gap_extension_score=-1)
    s1, s2 = splitmix_seq(m, 11, "dna"), splitmix_seq(n, 12, "dna")
    a1, a2, smat, cmat, gos, o = transform.settings(dict(DNA, seq_1=s1, seq_2=s2))
    tab = core.Tables(cmat)
    a, b = tab.codes(a1), tab.codes(a2)
    big = (tab.max_cost + 1) * max(m, n)
    row0, col0 = core.boundary(tab, a, b, o, big)
    dp = np.zeros((m + 1, n + 1, 3), np.int64)
    dp[0, :, :] = row0.reshape(n + 1, 3)
    dp[:, 0, :] = col0.reshape(m + 1, 3)
    core.fill_full(tab, a, b, o, dp)
    # rank sets per cell and entering level
    cell = np.zeros((m + 1, n + 1), np.int64)
    sets = {}
    for i in range(1, m + 1):
        for j in range(1, n + 1):
            M, X, Y = (int(x) for x in dp[i, j])
            mm = int(a[i - 1] != b[j - 1])
            u = 0
            for L, c in enumerate(((M, X, Y), (M + o, X, Y + o), (M + o, X + o, Y))):
                h = min(c)
                S = sum(1 << k for k in range(3) if c[k] == h)
                sets[(i, j, L)] = S
                u |= (3 * tab_field(S, mm)) << (5 * L)
            cell[i, j] = u
    # the table
    lib = C.CDLL(os.path.join(ROOT, "globalign_amd", "_lib", "libglobalign_amd.so"))
    lib.ga_debug_rng.argtypes = [C.c_void_p, C.c_int64, C.c_void_p, C.c_int64, C.c_void_p, C.c_void_p]
    random.seed(seed)
    st = np.array(random.getstate()[1], dtype=np.uint32)
    steps = m + n + 64
    T = np.zeros(steps, np.uint64)
    out = np.zeros(625, np.uint32)
    ms = C.c_double(0)
    assert lib.ga_debug_rng(st.ctypes.data, steps, T.ctypes.data, 0, out.ctypes.data, C.byref(ms)) == 0
    T = [int(x) for x in T]

    def level_at(i, j, L, D):
        fa = (int(cell[i, j]) >> (5 * L)) & 31
        V = (T[D] >> (2 * fa)) & M32
        return (~(V >> 3)) & 3

    # plain per-step walk (interior only: stop at i == 0 or j == 0)
    ref = []
    i, j, L, D = m, n, 0, 0
    while i >= 1 and j >= 1:
        lv = level_at(i, j, L, D)
        # the level must be in the rank set
        assert (sets[(i, j, L)] >> lv) & 1, (i, j, L, lv)
        ref.append(lv)
        D += 1
        i -= lv != 1
        j -= lv != 2
        L = lv
    # the device walker: per-step until D % 16 == 0, then groups of 4 with windows
    dev = []
    i, j, L, D = m, n, 0, 0
    while (D & 15) != 0 or D == 0:
        lv = level_at(i, j, L, D)
        dev.append(lv)
        D += 1
        i -= lv != 1
        j -= lv != 2
        L = lv
        if i == 0 or j == 0:
            break
    lanes = [(((ln - 17 * (ln & 7)) & 63) >> 3, ln & 7) for ln in range(64)]  # (lr, lc)

    def window(pi, pj):
        w = []
        for (lr, lc) in lanes:
            ci, cj = pi - lr, pj - lc
            w.append(int(cell[ci, cj]) if ci >= 1 and cj >= 1 else 0)
        return w

    def widen(w):
        return [(((u & 31) << 26) | ((u & 0x3e0) << 13) | ((u & 0x7c00) >> 1)) & M32 for u in w]

    if i >= 1 and j >= 1:
        wcw = widen(window(i, j))
        rel, Lx = 0, TV[L]
        done = False
        while not done:
            check = min(i, j) <= 16
            for g in range(4):
                wcur = wcw
                wnext = window(i, j)
                ix, A, ri, cj = rel, 0, 0, 0
                ended = 0
                for k in range(4):
                    v = wcur[ix & 63]
                    if k == 3:
                        wcw = widen(wnext)
                    f = (v >> (Lx & 31)) & M32
                    V = (T[D + 4 * g + k - 0] >> (f & 63)) & M32 if False else (T[D + 4 * g + k] >> (f & 63)) & M32
                    ix = (ix + V) & M32
                    Lx = V
                    code = (V >> 3) & 3
                    A = (A * 4 + code) & M32
                    dev.append((~code) & 3)
                    if check:
                        ri += code & 1
                        cj += code >> 1
                        if ri == i or cj == j:
                            i -= ri
                            j -= cj
                            ended = k + 1
                            break
                if ended:
                    done = True
                    break
                i -= bin(A & 0x55).count("1")
                j -= bin(A & 0xaa).count("1")
                rel = (ix - rel) & M32
            D += 16
    n_ok = next((k for k in range(min(len(dev), len(ref))) if dev[k] != ref[k]), None)
    print(m, n, "moves ref", len(ref), "dev", len(dev), "first diff", n_ok, "end", (i, j))
    return n_ok is None and len(dev) == len(ref)


if __name__ == "__main__":
    args = [int(x) for x in sys.argv[1:]]
    ok = main(*args) if args else all(main(m, n, s) for m, n, s in [(300, 400, 5), (256, 256, 512), (100, 120, 220)])
    print("OK" if ok else "MISMATCH")
