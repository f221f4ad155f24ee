"""ctypes front-end of the C oracle (ga_oracle.c).  TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import
this module, and only as the checker.  It builds oracle/_build/libga_oracle.so
on first use when gcc is available.
"""
import ctypes as C
import os
import random
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "_build", "libga_oracle.so")
_lib = None

i64p = np.ctypeslib.ndpointer(dtype=np.int64, flags="C_CONTIGUOUS")
u8p = np.ctypeslib.ndpointer(dtype=np.uint8, flags="C_CONTIGUOUS")
u16p = np.ctypeslib.ndpointer(dtype=np.uint16, flags="C_CONTIGUOUS")
u32p = np.ctypeslib.ndpointer(dtype=np.uint32, flags="C_CONTIGUOUS")
i32p = np.ctypeslib.ndpointer(dtype=np.int32, flags="C_CONTIGUOUS")
I64 = C.c_int64


def build():
    src = os.path.join(HERE, "ga_oracle.c")
    if not os.path.exists(LIB_PATH) or os.path.getmtime(LIB_PATH) < os.path.getmtime(src):
        subprocess.check_call(["make", "-s", "-C", HERE])


def lib():
    global _lib
    if _lib is None:
        build()
        L = C.CDLL(LIB_PATH)
        L.gao_boundary.argtypes = [u8p, I64, u8p, I64, i64p, i64p, I64, I64, i64p, i64p]
        L.gao_fill_full.argtypes = [u8p, I64, u8p, I64, i64p, C.c_int, i64p, i64p, I64, i64p]
        L.gao_fill_sets.argtypes = [u8p, I64, u8p, I64, i64p, C.c_int, i64p, i64p, I64, i64p, i64p, u16p, i64p]
        L.gao_fill_score.argtypes = [u8p, I64, u8p, I64, i64p, C.c_int, i64p, i64p, I64, i64p, i64p, i64p]
        L.gao_fill_slab.argtypes = [u8p, I64, u8p, I64, i64p, C.c_int, i64p, i64p, I64, i64p, i64p, i64p]
        L.gao_fill_score_parallel.argtypes = [u8p, I64, u8p, I64, i64p, C.c_int, i64p, i64p, I64, i64p, i64p, C.c_int,
                                              i64p]
        L.gao_traceback_full.argtypes = [i64p, I64, I64, I64, u8p, u8p, C.c_char_p, C.c_char_p, i64p, C.c_int,
                                         i64p, u32p, C.c_char_p, C.c_char_p, C.c_char_p, C.POINTER(I64), C.POINTER(I64)]
        L.gao_traceback_sets.argtypes = [u16p, i64p, i64p, I64, I64, I64, u8p, u8p, C.c_char_p, C.c_char_p, i64p,
                                         C.c_int, i64p, u32p, C.c_char_p, C.c_char_p, C.c_char_p, C.POINTER(I64),
                                         C.POINTER(I64)]
        L.gao_mt_draws.argtypes = [u32p, C.c_int, i32p, i32p]
        L.gao_align_ckpt.argtypes = [u8p, I64, u8p, I64, C.c_char_p, C.c_char_p, i64p, C.c_int, i64p, i64p, I64, i64p,
                                     i64p, C.c_int, I64, I64, u32p, C.c_char_p, C.c_char_p, C.c_char_p, C.POINTER(I64),
                                     C.POINTER(I64), i64p, C.POINTER(I64)]
        _lib = L
    return _lib


class Tables:
    """Integer tables derived from a costing dict (keys in dict order)."""

    def __init__(self, cmat):
        self.keys = list(cmat.keys())
        self.code = {k: i for i, k in enumerate(self.keys)}
        K = self.K = len(self.keys)
        self.sub = np.array([[cmat[x][y] for y in self.keys] for x in self.keys], dtype=np.int64).reshape(-1)
        self.gh = np.array([cmat["-"][y] for y in self.keys], dtype=np.int64)
        self.gv = np.array([cmat[x]["-"] for x in self.keys], dtype=np.int64)
        self.max_cost = int(max(max(r.values()) for r in cmat.values()))
        assert self.sub.size == K * K

    def codes(self, s):
        return np.array([self.code[ch] for ch in s], dtype=np.uint8)


def mt_state_array(state=None):
    st = random.getstate() if state is None else state
    return np.array(st[1], dtype=np.uint32)


def mt_state_tuple(arr):
    return (3, tuple(int(x) for x in arr), None)


def boundary(tab, a, b, o, big):
    m, n = len(a), len(b)
    row0 = np.zeros(3 * (n + 1), np.int64)
    col0 = np.zeros(3 * (m + 1), np.int64)
    lib().gao_boundary(a, m, b, n, tab.gh, tab.gv, o, big, row0, col0)
    return row0, col0


def fill_full(tab, a, b, o, dp):
    """dp: int64 array (m+1, n+1, 3) with row 0 / column 0 set; filled in place."""
    m, n = len(a), len(b)
    lib().gao_fill_full(a, m, b, n, tab.sub, tab.K, tab.gh, tab.gv, o, dp.reshape(-1))
    return dp


def fill_score(tab, a, b, o, row0, col0):
    last = np.zeros(3, np.int64)
    lib().gao_fill_score(a, len(a), b, len(b), tab.sub, tab.K, tab.gh, tab.gv, o, row0, col0, last)
    return last


def fill_score_parallel(tab, a, b, o, row0, col0, threads=8):
    """fill_score on `threads` host threads (column slabs x row bands wavefront); same cells (gao_cell)."""
    last = np.zeros(3, np.int64)
    lib().gao_fill_score_parallel(a, len(a), b, len(b), tab.sub, tab.K, tab.gh, tab.gv, o, row0, col0, threads, last)
    return last


def fill_slab(tab, a, b, o, row0, col0):
    right = np.zeros(3 * (len(a) + 1), np.int64)
    lib().gao_fill_slab(a, len(a), b, len(b), tab.sub, tab.K, tab.gh, tab.gv, o, row0, col0, right)
    return right


def align(seq_1, seq_2, cmat, o, mt_words, mode="auto", threads=8, tile=(4096, 4096)):
    """Oracle of make_dp_array + dp_array_forward + dp_array_backward.

    mode "full" (the whole triple array), "sets" (m x n rank sets), "ckpt" (every tile[0]-th row and tile[1]-th
    column of triples from a forward pass on `threads` threads; the walk recomputes one tile's sets at a time:
    memory (m/BH)(n+1) + (n/CW)(m+1) triples, for 1M x 1M at 4096 x 4096 12 GB).
    Returns dict(cost, strings, status ('ok'|'IndexError'), ndispatch, mt_out)."""
    tab = Tables(cmat)
    a, b = tab.codes(seq_1), tab.codes(seq_2)
    m, n = len(a), len(b)
    big = (tab.max_cost + 1) * max(m, n)
    row0, col0 = boundary(tab, a, b, o, big)
    if mode == "auto":
        mode = "full" if (m + 1) * (n + 1) <= 4_000_000 else "sets"
    mt = np.array(mt_words, dtype=np.uint32).copy()
    cap = m + n + 2
    oa, om, ob = C.create_string_buffer(cap), C.create_string_buffer(cap), C.create_string_buffer(cap)
    ln, nd = I64(0), I64(0)
    a_chr, b_chr = seq_1.encode(), seq_2.encode()
    if mode == "full":
        dp = np.zeros((m + 1, n + 1, 3), np.int64)
        dp[0, :, :] = row0.reshape(n + 1, 3)
        dp[:, 0, :] = col0.reshape(m + 1, 3)
        fill_full(tab, a, b, o, dp)
        last = dp[m, n]
        st = lib().gao_traceback_full(dp.reshape(-1), m, n, o, a, b, a_chr, b_chr, tab.sub, tab.K, tab.gh, mt,
                                      oa, om, ob, C.byref(ln), C.byref(nd))
    elif mode == "ckpt":
        last = np.zeros(3, np.int64)
        nt = I64(0)
        st = lib().gao_align_ckpt(a, m, b, n, a_chr, b_chr, tab.sub, tab.K, tab.gh, tab.gv, o, row0, col0, threads,
                                  tile[0], tile[1], mt, oa, om, ob, C.byref(ln), C.byref(nd), last, C.byref(nt))
        if st < 0:
            raise MemoryError("gao_align_ckpt: checkpoints do not fit in host memory")
    else:
        sets = np.zeros(m * n, np.uint16)
        last = np.zeros(3, np.int64)
        lib().gao_fill_sets(a, m, b, n, tab.sub, tab.K, tab.gh, tab.gv, o, row0, col0, sets, last)
        st = lib().gao_traceback_sets(sets, row0, col0, m, n, o, a, b, a_chr, b_chr, tab.sub, tab.K, tab.gh, mt,
                                      oa, om, ob, C.byref(ln), C.byref(nd))
    L = ln.value
    return {
        "cost": int(min(last)),
        "strings": (oa.raw[:L].decode(), om.raw[:L].decode(), ob.raw[:L].decode()),
        "status": "ok" if st == 0 else "IndexError",
        "ndispatch": nd.value,
        "mt_out": mt,
    }
