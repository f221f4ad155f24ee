"""ctypes binding of the MI355X engine (include/globalign_amd.h).

The product path has no CPU fallback: if the HIP library is missing or no
GPU is visible, every entry point raises.  The shared library is built
in-tree by ``__graft_entry__.build()`` (``make -C globalign_amd/csrc``).
"""
import ctypes as C
import os
import threading

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("GA_LIB_PATH") or os.path.join(_HERE, "_lib", "libglobalign_amd.so")

GA_FILL_TRACEBACK = 1
GA_FILL_FULL = 2
GA_E_NOMEM = -6
GA_TB_OK = 0
GA_TB_INDEX_ERROR = 1

_lib = None
_lib_lock = threading.Lock()


class GaCosts(C.Structure):
    _fields_ = [
        ("K", C.c_int32),
        ("sub", C.POINTER(C.c_int32)),
        ("gap_h", C.POINTER(C.c_int32)),
        ("gap_v", C.POINTER(C.c_int32)),
        ("gap_open", C.c_int32),
        ("max_cost", C.c_int32),
    ]


class EngineError(RuntimeError):
    pass


# every symbol include/globalign_amd.h declares (tests check the exports)
EXPORTS = [
    "ga_last_error", "ga_device_count", "ga_ctx_create", "ga_ctx_create_opts", "ga_ctx_destroy", "ga_build_flags", "ga_problem_set", "ga_problem_fill", "ga_problem_set_cells",
    "ga_problem_traceback", "ga_problem_align", "ga_problem_align_many", "ga_problem_set_slab", "ga_slab_buffers", "ga_slab_bind_halos",
    "ga_slab_link", "ga_slab_link_export", "ga_slab_link_import", "ga_enable_peer_access",
    "ga_slab_fill_launch", "ga_slab_fill_finish", "ga_slab_walk_prepare", "ga_slab_walk", "ga_slab_mt_state",
    "ga_stream_wait_ge", "ga_stream_write", "ga_ctx_stream", "ga_ctx_wait_stream", "ga_ctx_stream_priority",
    "ga_last_kernel_ms", "ga_last_timings",
]


class WalkState(C.Structure):
    """ga_walk_state: the traceback walk handed from slab to slab (right to left)."""
    _fields_ = [("i", C.c_int64), ("j", C.c_int64), ("D", C.c_int64), ("h", C.c_int64), ("L", C.c_int32),
                ("first", C.c_int32), ("reason", C.c_int32), ("pad", C.c_int32)]

    def as_list(self):
        return [self.i, self.j, self.D, self.h, self.L, self.first, self.reason]

    @classmethod
    def from_list(cls, v):
        return cls(int(v[0]), int(v[1]), int(v[2]), int(v[3]), int(v[4]), int(v[5]), int(v[6]), 0)


def _preload_hip_runtime():
    """Keep ONE HIP runtime per process.

    PyTorch-ROCm ships its own libamdhip64.so and resolves it by path, while
    this library links libamdhip64.so.7.  If ours were loaded first and torch
    imported later, the process would hold two HIP runtimes.  So when torch is
    installed, load torch's runtime first (without importing torch): our
    library then binds to it by SONAME, and torch finds it already loaded."""
    import importlib.util
    try:
        spec = importlib.util.find_spec("torch")
    except (ImportError, ValueError):
        spec = None
    if spec is None or not spec.origin:
        return
    cand = os.path.join(os.path.dirname(spec.origin), "lib", "libamdhip64.so")
    if os.path.exists(cand):
        C.CDLL(cand, mode=C.RTLD_GLOBAL)


def load_library():
    """Load libglobalign_amd.so (raises ImportError when it has not been built)."""
    global _lib
    with _lib_lock:
        if _lib is not None:
            return _lib
        _preload_hip_runtime()
        if not os.path.exists(LIB_PATH):
            raise ImportError(
                f"{LIB_PATH} not found: build the HIP engine first (python -c 'import __graft_entry__ as g; g.build()')")
        L = C.CDLL(LIB_PATH)
        i64, i32, vp = C.c_int64, C.c_int32, C.c_void_p
        p32, pu32, pi64 = C.POINTER(C.c_int32), C.POINTER(C.c_uint32), C.POINTER(C.c_int64)
        L.ga_last_error.restype = C.c_char_p
        L.ga_device_count.argtypes = [C.POINTER(C.c_int)]
        L.ga_ctx_create.argtypes = [C.c_int, C.POINTER(vp)]
        L.ga_ctx_create_opts.argtypes = [C.c_int, C.c_char_p, C.POINTER(vp)]
        L.ga_build_flags.argtypes = [p32]
        L.ga_ctx_destroy.argtypes = [vp]
        L.ga_ctx_destroy.restype = None
        L.ga_problem_set.argtypes = [vp, C.c_char_p, i64, C.c_char_p, i64, C.POINTER(GaCosts), p32, p32]
        L.ga_problem_fill.argtypes = [vp, i32, pi64, p32]
        L.ga_problem_set_cells.argtypes = [vp, p32, pi64]
        L.ga_problem_traceback.argtypes = [vp, pu32, C.c_char_p, C.c_char_p, C.c_char_p, C.c_char_p, C.c_char_p, i64,
                                           pi64, p32]
        L.ga_problem_align.argtypes = [vp, pu32, C.c_char_p, C.c_char_p, C.c_char_p, C.c_char_p, C.c_char_p, i64,
                                       pi64, p32, pi64]
        L.ga_problem_align_many.argtypes = [vp, i32, pu32, C.c_char_p, C.c_char_p, C.c_char_p, C.c_char_p,
                                            C.c_char_p, i64, pi64, p32, pi64]
        L.ga_problem_set_slab.argtypes = [vp, C.c_char_p, i64, C.c_char_p, i64, C.POINTER(GaCosts), i64, i64]
        L.ga_slab_buffers.argtypes = [vp, C.POINTER(vp), C.POINTER(vp), C.POINTER(vp), C.POINTER(vp)]
        L.ga_slab_bind_halos.argtypes = [vp, vp, vp]
        L.ga_slab_link.argtypes = [vp, vp]
        L.ga_slab_link_export.argtypes = [vp, C.c_char_p]
        L.ga_slab_link_import.argtypes = [vp, C.c_char_p]
        L.ga_enable_peer_access.argtypes = [C.c_int, C.c_int]
        L.ga_slab_walk_prepare.argtypes = [vp, pu32]
        L.ga_slab_walk.argtypes = [vp, C.POINTER(WalkState), C.c_char_p, C.c_char_p, C.c_char_p, C.c_char_p,
                                   C.c_char_p, i64, pi64]
        L.ga_slab_mt_state.argtypes = [vp, i64, pu32]
        L.ga_slab_fill_launch.argtypes = [vp, i32]
        L.ga_slab_fill_finish.argtypes = [vp, pi64]
        L.ga_stream_wait_ge.argtypes = [vp, vp, C.c_uint32]
        L.ga_stream_write.argtypes = [vp, vp, C.c_uint32]
        L.ga_ctx_stream.argtypes = [vp]
        L.ga_ctx_stream.restype = vp
        L.ga_ctx_wait_stream.argtypes = [vp, vp]
        L.ga_ctx_stream_priority.argtypes = [vp, C.POINTER(C.c_int)]
        L.ga_last_kernel_ms.argtypes = [vp, C.POINTER(C.c_float), C.POINTER(C.c_float)]
        L.ga_last_timings.argtypes = [vp, C.POINTER(C.c_float)]
        _lib = L
        return L


def _check(rc):
    if rc != 0:
        msg = _lib.ga_last_error().decode(errors="replace")
        if rc == -1:
            raise ValueError(msg)
        if rc == GA_E_NOMEM:
            raise MemoryError(f"globalign_amd engine: {msg}")
        raise EngineError(f"globalign_amd engine error {rc}: {msg}")


# a progress word's value once the fill writing it (or the relay feeding it) has given up (ga_sync.h)
PROG_ABORT = 0xFFFFFFFF


def experiments_build():
    """True for a library built with make EXPERIMENTS=1 (the measured-and-dropped paths compiled in)."""
    L = load_library()
    f = (C.c_int32 * 1)()
    _check(L.ga_build_flags(f))
    return bool(f[0] & 1)


def device_count():
    L = load_library()
    n = C.c_int(0)
    _check(L.ga_device_count(C.byref(n)))
    return n.value


class CostTables:
    """Integer view of a costing dict: codes follow the dict's key order."""

    def __init__(self, costing_mat, gap_open_cost):
        self.keys = list(costing_mat.keys())
        if "-" not in costing_mat:
            raise KeyError("-")
        self.code = {k: i for i, k in enumerate(self.keys)}
        K = len(self.keys)
        self.sub = np.array([[int(costing_mat[x][y]) for y in self.keys] for x in self.keys], dtype=np.int32).reshape(-1)
        self.gap_h = np.array([int(costing_mat["-"][y]) for y in self.keys], dtype=np.int32)
        self.gap_v = np.array([int(costing_mat[x]["-"]) for x in self.keys], dtype=np.int32)
        self.max_cost = int(max(max(row.values()) for row in costing_mat.values()))
        self.gap_open = int(gap_open_cost)
        self.K = K
        p32 = C.POINTER(C.c_int32)
        self.struct = GaCosts(K, self.sub.ctypes.data_as(p32), self.gap_h.ctypes.data_as(p32),
                              self.gap_v.ctypes.data_as(p32), self.gap_open, self.max_cost)

    def codes(self, seq):
        code = self.code
        return bytes(code[ch] for ch in seq)


# Explicit context options (ga_ctx_create_opts): kernel variants for tests and tuning, fault injection,
# diagnostics.  The library reads only its shipped GA_* knobs from the environment; everything
# else is given here, e.g. OPTIONS["GA_LANE_ASM"] = "0", or per engine through Engine(options=...).
OPTIONS = {}


def options_string(options=None):
    merged = dict(OPTIONS)
    merged.update(options or {})
    return ";".join(f"{k}={v}" for k, v in sorted(merged.items()))


class Engine:
    """One HIP device context (ga_ctx)."""

    def __init__(self, device=0, options=None):
        L = load_library()
        if device_count() < 1:
            raise EngineError("no HIP device visible: the globalign_amd engine runs on MI355X (gfx950) only")
        self._L = L
        h = C.c_void_p()
        _check(L.ga_ctx_create_opts(int(device), options_string(options).encode(), C.byref(h)))
        self._h = h
        self.device = device
        self.m = self.n = 0

    def close(self):
        if getattr(self, "_h", None):
            self._L.ga_ctx_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -- problem -------------------------------------------------------------
    def load(self, a_codes, b_codes, tables, row0=None, col0=None):
        p32 = C.POINTER(C.c_int32)
        r0 = c0 = None
        if row0 is not None:
            self._row0 = np.ascontiguousarray(row0, dtype=np.int32).reshape(-1)
            self._col0 = np.ascontiguousarray(col0, dtype=np.int32).reshape(-1)
            r0, c0 = self._row0.ctypes.data_as(p32), self._col0.ctypes.data_as(p32)
        self._tables = tables
        _check(self._L.ga_problem_set(self._h, a_codes, len(a_codes), b_codes, len(b_codes), C.byref(tables.struct),
                                      r0, c0))
        self.m, self.n = len(a_codes), len(b_codes)

    def fill(self, traceback=False, full=False):
        flags = (GA_FILL_TRACEBACK if traceback else 0) | (GA_FILL_FULL if full else 0)
        cost = C.c_int64(0)
        out = None
        ptr = None
        if full:
            out = np.zeros((self.m + 1, self.n + 1, 3), dtype=np.int32)
            ptr = out.ctypes.data_as(C.POINTER(C.c_int32))
        _check(self._L.ga_problem_fill(self._h, flags, C.byref(cost), ptr))
        return cost.value, out

    def fill_kind(self):
        """The kernel and geometry of the last fill: (kind, T, nstripes, nwc, nslabs), kind 'row' / 'diag' / 'lane', or
        'rc' (the recompute walk's checkpointing lane fill)."""
        f = self._L.ga_debug_fill_kind
        f.argtypes = [C.c_void_p, C.c_void_p]
        f.restype = C.c_int
        out = np.zeros(5, dtype=np.int32)
        _check(f(self._h, out.ctypes.data))
        return (("row", "diag", "lane", "rc")[int(out[0])],) + tuple(int(x) for x in out[1:])

    def walk_kind(self):
        """The walk of the last traceback: 'stored' (traceback words), 'rc' (the recompute walk of words) or 'jump'
        (the tie-to-tie recompute walk)."""
        f = self._L.ga_debug_walk_kind
        f.argtypes = [C.c_void_p, C.c_void_p]
        f.restype = C.c_int
        out = np.zeros(1, dtype=np.int32)
        _check(f(self._h, out.ctypes.data))
        return ("stored", "rc", "jump")[int(out[0])]

    def set_cells(self, cells):
        """Use a filled (m+1, n+1, 3) int32 cell array for the next traceback (-> min of the last cell)."""
        arr = np.ascontiguousarray(cells, dtype=np.int32)
        if arr.shape != (self.m + 1, self.n + 1, 3):
            raise ValueError(f"cells must be ({self.m + 1}, {self.n + 1}, 3), got {arr.shape}")
        cost = C.c_int64(0)
        _check(self._L.ga_problem_set_cells(self._h, arr.ctypes.data_as(C.POINTER(C.c_int32)), C.byref(cost)))
        return cost.value

    def _tb_call(self, fn, mt_words, a_chr, b_chr, extra=()):
        mt = np.ascontiguousarray(mt_words, dtype=np.uint32).copy()
        cap = self.m + self.n + 2
        # output rows kept by the engine (unzeroed: the engine writes the first out_len bytes), the sequences' bytes
        # kept while the caller passes the same str objects (round 6: zeroing three 200 KB buffers, encoding both
        # sequences and copying whole buffers before slicing took ~0.1 ms of every C3 call)
        if getattr(self, "_obuf_cap", 0) < cap:
            self._obuf = tuple(np.empty(cap, dtype=np.uint8) for _ in range(3))
            self._obuf_cap = cap
        oa, om, ob = self._obuf
        enc = getattr(self, "_enc", None)
        if enc is None or enc[0] is not a_chr or enc[2] is not b_chr:
            enc = self._enc = (a_chr, a_chr.encode(), b_chr, b_chr.encode())
        ln, st = C.c_int64(0), C.c_int32(0)
        cp = C.c_char_p
        _check(fn(self._h, mt.ctypes.data_as(C.POINTER(C.c_uint32)), enc[1], enc[3], oa.ctypes.data_as(cp),
                  om.ctypes.data_as(cp), ob.ctypes.data_as(cp), cap, C.byref(ln), C.byref(st), *extra))
        L = ln.value
        strings = tuple(x[:L].tobytes().decode() for x in (oa, om, ob))
        return strings, st.value, mt

    def traceback(self, mt_words, a_chr, b_chr):
        """-> ((seq_1_aligned, middle, seq_2_aligned), status, mt_words_after)"""
        return self._tb_call(self._L.ga_problem_traceback, mt_words, a_chr, b_chr)

    def align(self, mt_words, a_chr, b_chr):
        """fill + traceback -> (cost, strings, status, mt_words_after)"""
        cost = C.c_int64(0)
        strings, st, mt = self._tb_call(self._L.ga_problem_align, mt_words, a_chr, b_chr, (C.byref(cost),))
        return cost.value, strings, st, mt

    def align_many(self, mt_words, a_chr, b_chr, count):
        """`count` consecutive alignments of the loaded pair, each from the random state the previous one left
        (as consecutive find_global_alignment calls); walk k overlaps fill k+1 on the device.
        -> ([(cost, strings, status)] * count, mt_words_after)"""
        mt = np.ascontiguousarray(mt_words, dtype=np.uint32).copy()
        cap = self.m + self.n + 2
        # unzeroed output rows (the engine writes each alignment's first out_len[k] bytes)
        oa, om, ob = (np.empty(cap * count, dtype=np.uint8) for _ in range(3))
        ln = np.zeros(count, dtype=np.int64)
        st = np.zeros(count, dtype=np.int32)
        cost = np.zeros(count, dtype=np.int64)
        p64, p32 = C.POINTER(C.c_int64), C.POINTER(C.c_int32)
        _check(self._L.ga_problem_align_many(self._h, int(count), mt.ctypes.data_as(C.POINTER(C.c_uint32)),
                                             a_chr.encode(), b_chr.encode(), oa.ctypes.data_as(C.c_char_p),
                                             om.ctypes.data_as(C.c_char_p), ob.ctypes.data_as(C.c_char_p), cap,
                                             ln.ctypes.data_as(p64),
                                             st.ctypes.data_as(p32), cost.ctypes.data_as(p64)))
        out = []
        for k in range(count):
            lo, L = k * cap, int(ln[k])
            out.append((int(cost[k]), tuple(x[lo:lo + L].tobytes().decode() for x in (oa, om, ob)), int(st[k])))
        return out, mt

    def timings(self):
        """{fill_ms, walk_ms, rng_ms (host tie-break table), call_ms} of the last call."""
        out = (C.c_float * 4)()
        _check(self._L.ga_last_timings(self._h, out))
        return dict(fill_ms=out[0], walk_ms=out[1], rng_ms=out[2], call_ms=out[3])

    def kernel_ms(self):
        f, w = C.c_float(0), C.c_float(0)
        _check(self._L.ga_last_kernel_ms(self._h, C.byref(f), C.byref(w)))
        return f.value, w.value

    # -- slabs (multi-GPU) ---------------------------------------------------
    def load_slab(self, a_codes, b_codes, tables, col_begin, col_end):
        self._tables = tables
        _check(self._L.ga_problem_set_slab(self._h, a_codes, len(a_codes), b_codes, len(b_codes),
                                           C.byref(tables.struct), int(col_begin), int(col_end)))
        self.m, self.n = len(a_codes), int(col_end - col_begin)

    def slab_buffers(self):
        """-> (halo_in device ptr, halo_in_prog HOST ptr, halo_out device ptr, halo_out_prog HOST ptr)"""
        vp = C.c_void_p
        hi, hip_, ho, hop = vp(), vp(), vp(), vp()
        _check(self._L.ga_slab_buffers(self._h, C.byref(hi), C.byref(hip_), C.byref(ho), C.byref(hop)))
        self._in_prog = C.c_uint32.from_address(hip_.value)
        self._out_prog = C.c_uint32.from_address(hop.value)
        return hi.value, hip_.value, ho.value, hop.value

    def slab_bind_halos(self, halo_in_ptr, halo_out_ptr):
        """Use caller-owned (m+1) x int2 buffers (device or pinned host memory) as the slab's edges."""
        _check(self._L.ga_slab_bind_halos(self._h, C.c_void_p(halo_in_ptr), C.c_void_p(halo_out_ptr)))

    def slab_link(self, right):
        """Join this slab (left) to its right neighbour's engine device to device (ga_slab_link)."""
        _check(self._L.ga_slab_link(self._h, right._h))

    def slab_link_export(self):
        """This (right) slab's side of a cross-process link -> the 64-byte IPC handle of its edge buffer."""
        buf = C.create_string_buffer(64)
        _check(self._L.ga_slab_link_export(self._h, buf))
        return buf.raw

    def slab_link_import(self, handle):
        """Map the right neighbour's edge buffer (its slab_link_export bytes) as this slab's right edge."""
        if len(handle) != 64:
            raise ValueError("an IPC handle has 64 bytes")
        _check(self._L.ga_slab_link_import(self._h, bytes(handle)))

    def slab_launch(self, traceback=False):
        _check(self._L.ga_slab_fill_launch(self._h, GA_FILL_TRACEBACK if traceback else 0))
        self.slab_buffers()

    def slab_finish(self):
        cost = C.c_int64(0)
        _check(self._L.ga_slab_fill_finish(self._h, C.byref(cost)))
        return cost.value

    # progress words of the running slab fill (pinned host memory shared with the kernel)
    def out_progress(self):
        v = self._out_prog.value
        if v == PROG_ABORT:
            raise EngineError("the slab fill gave up before its right edge was complete")
        return v

    def set_in_progress(self, rows):
        self._in_prog.value = int(rows)

    def slab_walk_prepare(self, mt_words):
        mt = np.ascontiguousarray(mt_words, dtype=np.uint32)
        _check(self._L.ga_slab_walk_prepare(self._h, mt.ctypes.data_as(C.POINTER(C.c_uint32))))

    def slab_walk(self, state, a_chr, b_chr):
        """Continue the walk (list state, see WalkState) on this slab -> (segment strings, new state)."""
        st = WalkState.from_list(state)
        cap = self.m + 2 * len(b_chr) + 2
        oa, om, ob = C.create_string_buffer(cap), C.create_string_buffer(cap), C.create_string_buffer(cap)
        ln = C.c_int64(0)
        _check(self._L.ga_slab_walk(self._h, C.byref(st), a_chr.encode(), b_chr.encode(), oa, om, ob, cap,
                                    C.byref(ln)))
        n = ln.value
        return (oa.raw[:n].decode(), om.raw[:n].decode(), ob.raw[:n].decode()), st.as_list()

    def slab_mt_state(self, D):
        out = np.zeros(625, dtype=np.uint32)
        _check(self._L.ga_slab_mt_state(self._h, int(D), out.ctypes.data_as(C.POINTER(C.c_uint32))))
        return out

    def stream(self):
        return self._L.ga_ctx_stream(self._h)

    def wait_stream(self, stream):
        """Order this context's stream after the work enqueued so far on `stream` (a hipStream_t handle)."""
        _check(self._L.ga_ctx_wait_stream(self._h, C.c_void_p(stream)))

    def stream_priority(self):
        pr = C.c_int(0)
        _check(self._L.ga_ctx_stream_priority(self._h, C.byref(pr)))
        return pr.value

    def stream_wait_ge(self, stream, prog_ptr, value):
        _check(self._L.ga_stream_wait_ge(C.c_void_p(stream), C.c_void_p(prog_ptr), int(value)))

    def stream_write(self, stream, prog_ptr, value):
        _check(self._L.ga_stream_write(C.c_void_p(stream), C.c_void_p(prog_ptr), int(value)))


_default = {}
_default_lock = threading.Lock()


def knob_fingerprint():
    """The GA_* overrides as the environment and OPTIONS hold them now.  A context reads them once, when it is
    created (ga_ctx_create_opts), so cached engines are keyed by them: changing one (tests, tuning) gets a fresh
    context, and a context's kernel choices never change under it."""
    return (tuple(sorted((k, v) for k, v in os.environ.items() if k.startswith("GA_"))),
            tuple(sorted((k, str(v)) for k, v in OPTIONS.items())))


def evict_stale(cache, key):
    """Drop the cached entries of key's (device(s), thread) whose GA_* fingerprint differs from key's: a context
    made under other knobs is never asked for again by this thread, and its device buffers (traceback words,
    checkpoints, tile cache) would otherwise stay allocated and shrink the free memory later calls size
    themselves by.  The context is destroyed once nothing else holds it (Engine.__del__)."""
    for k in [k for k in cache if k[:2] == key[:2] and k != key]:
        del cache[k]


def default_engine(device=0):
    """Process-wide engine per device and GA_* override set (contexts are not thread-safe: one per thread);
    one set per (device, thread) is kept, the current one."""
    key = (device, threading.get_ident(), knob_fingerprint())
    with _default_lock:
        eng = _default.get(key)
        if eng is None:
            evict_stale(_default, key)
            eng = Engine(device)
            _default[key] = eng
        return eng
