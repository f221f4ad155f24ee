"""CPU tests of the product's host side: library exports, the host tie-break table
(CPython MT19937 emulation) and argument validation -- no GPU needed."""
import ctypes as C
import random
import re

import numpy as np
import pytest

from tests.conftest import ROOT, state_digest, set_knob


@pytest.fixture(scope="module")
def lib():
    from globalign_amd import _native
    return _native.load_library()


def test_exports_match_header(lib):
    """Every function include/globalign_amd.h declares is exported by the library."""
    from globalign_amd import _native
    hdr = open(f"{ROOT}/include/globalign_amd.h").read()
    declared = set(re.findall(r"^\s*(?:const\s+)?[\w\*]+\s+\**(ga_\w+)\s*\(", hdr, re.M))
    assert declared == set(_native.EXPORTS)
    for name in declared:
        assert getattr(lib, name) is not None


def _choice_levels(r):
    """Level chosen per candidate set S (1..7) for one step's 18 draws (dispatcher order)."""
    out = []
    for half in (0, 1):
        q = r[9 * half: 9 * half + 9]
        lv = {1: 0, 2: 1, 3: q[1], 4: 2, 5: 2 * q[2], 6: 1 + q[3], 7: q[0]}
        out.append(lv)
    return out


@pytest.mark.parametrize("seed,steps", [(0, 1), (1, 37), (12345, 500), (7, 3000), (3, 5000), (11, 20000), (14, 4096)])
def test_tiebreak_table_matches_cpython(lib, seed, steps):
    lib.ga_debug_rng.argtypes = [C.c_void_p, C.c_int64, C.c_void_p, C.c_int64, C.c_void_p, C.c_void_p]
    random.seed(seed)
    for _ in range(seed % 5):          # start mid-block too
        random.random()
    st = np.array(random.getstate()[1], dtype=np.uint32)
    sizes = [3, 2, 2, 2, 3, 2, 2, 2, 3] * 2
    want, states = [], [random.getstate()]
    for _ in range(steps):
        r = [random.choice(range(s)) for s in sizes]
        lv = _choice_levels(r)
        e = 0
        for half in (0, 1):
            for S in range(1, 8):
                e |= lv[half][S] << (2 * S + 1 + 14 * half)
        want.append(e)
        states.append(random.getstate())
    for D in sorted({0, 1, steps // 2, steps}):
        tab = np.zeros(steps, np.uint32)
        out = np.zeros(625, np.uint32)
        ms = C.c_double(0)
        assert lib.ga_debug_rng(st.ctypes.data, steps, tab.ctypes.data, D, out.ctypes.data, C.byref(ms)) == 0
        assert tab.tolist() == want
        assert state_digest((3, tuple(int(x) for x in out), None)) == state_digest(states[D])


@pytest.mark.parametrize("seed,steps,chunk", [(2, 5000, 1), (5, 20000, 777), (9, 12000, 4000), (4, 3001, 3001)])
def test_tiebreak_stream_resumes_exactly(lib, seed, steps, chunk):
    """The resumable table stream (align_many's continuous tie-break table): built in chunks it equals the
    one-shot table, and its entries from any dispatch G on equal a fresh table started from the state
    after G dispatches (consecutive alignments share one stream)."""
    lib.ga_debug_rng.argtypes = [C.c_void_p, C.c_int64, C.c_void_p, C.c_int64, C.c_void_p, C.c_void_p]
    lib.ga_debug_rng_chunked.argtypes = [C.c_void_p, C.c_int64, C.c_int64, C.c_void_p, C.c_int64, C.c_void_p]
    random.seed(seed)
    st = np.array(random.getstate()[1], dtype=np.uint32)
    one = np.zeros(steps, np.uint32)
    s1 = np.zeros(625, np.uint32)
    ms = C.c_double(0)
    assert lib.ga_debug_rng(st.ctypes.data, steps, one.ctypes.data, steps, s1.ctypes.data, C.byref(ms)) == 0
    ch = np.zeros(steps, np.uint32)
    s2 = np.zeros(625, np.uint32)
    G = steps // 3
    assert lib.ga_debug_rng_chunked(st.ctypes.data, steps, chunk, ch.ctypes.data, G, s2.ctypes.data) == 0
    assert ch.tolist() == one.tolist()
    fresh = np.zeros(steps - G, np.uint32)
    s3 = np.zeros(625, np.uint32)
    assert lib.ga_debug_rng(s2.ctypes.data, steps - G, fresh.ctypes.data, 0, s3.ctypes.data, C.byref(ms)) == 0
    assert fresh.tolist() == one[G:].tolist()


def test_lane_asm_header_matches_generator(tmp_path):
    """The committed ga_lane_asm.h is exactly what tools/gen_lane_asm.py generates (no hand edits, no drift)."""
    import subprocess
    import sys
    out = tmp_path / "ga_lane_asm.h"
    subprocess.check_call([sys.executable, f"{ROOT}/tools/gen_lane_asm.py", str(out)], stdout=subprocess.DEVNULL)
    assert out.read_bytes() == open(f"{ROOT}/globalign_amd/csrc/ga_lane_asm.h", "rb").read()


def test_engine_cache_keeps_one_knob_set(monkeypatch):
    """default_engine / device_engines keep one context per (device(s), thread): a GA_* change drops the contexts
    made under the old set (they held their device buffers for the life of the process)."""
    import gc
    import weakref

    from globalign_amd import _native, distributed

    made = []

    class FakeEngine:
        def __init__(self, device):
            self.device = device
            made.append(weakref.ref(self))

    monkeypatch.setattr(_native, "Engine", FakeEngine)
    monkeypatch.setattr(_native, "_default", {})
    monkeypatch.setattr(distributed, "_device_engines", {})
    for k in range(5):
        set_knob(monkeypatch, "GA_RC_SERVERS", str(48 + k))
        e0 = _native.default_engine(0)
        assert _native.default_engine(0) is e0          # same knobs: the cached context
        _native.default_engine(1)
        distributed.device_engines([0, 1])
    assert len(_native._default) == 2                    # one per device for this thread
    assert len(distributed._device_engines) == 1
    del e0
    gc.collect()
    assert sum(r() is not None for r in made) == 4       # the current set's: 2 default + 2 slab engines


def _perm(a, b, sel):
    """v_perm_b32: byte k of the result is byte sel_k of {a, b} (b = bytes 0..3), 0x0c gives 0x00"""
    src = [(b >> (8 * k)) & 0xff for k in range(4)] + [(a >> (8 * k)) & 0xff for k in range(4)]
    return sum((src[s] if s < 8 else (0 if s == 12 else 0xff)) << (8 * k) for k, s in
               enumerate((sel >> (8 * k)) & 0xff for k in range(4)))


@pytest.mark.parametrize("o", [0, 1, 5, 10, 14])
def test_jump_lut_selects_the_singleton_move(lib, o):
    """The tie-to-tie walk's worker LUT (ga_host.cpp jump_lut_build): for every combination of
    saturated differences its selectors pick, per entering level, the candidate of the level's unique minimum (diag
    Pd / left Pl / up Pu) and a zero half plus the walk's tie word for a tie -- checked against the rank sets of the
    reference's rank test (argmin of (M, X, Y), (M+o, X, Y+o), (M+o, X+o, Y); globaligner.py:431-441, :490-514)."""
    lut = np.zeros(4096, dtype=np.uint32)
    lib.ga_debug_jump_lut.argtypes = [C.c_int32, C.c_void_p]
    assert lib.ga_debug_jump_lut(o, lut.ctypes.data) == 0
    Pd, Pl, Pu = 0x1113, 0x2221, 0x3332  # distinct 16-bit candidates
    src0 = _perm(Pl, Pd, 0x05040100)
    for dM in range(0, 3):
        for dX in range(0, o + 4):
            for dY in range(0, o + 4):
                if min(dM, dX, dY):
                    continue
                for mm in (0, 1):
                    H = 100
                    M, X, Y = H + dM, H + dX, H + dY
                    idx = min(dX, o + 1) | (min(dY, o + 1) << 4) | (min(dM, 1) << 8) | (mm << 9)
                    e01 = _perm(src0, Pu, int(lut[4 * idx])) | int(lut[4 * idx + 2])
                    e2 = _perm(src0, Pu, int(lut[4 * idx + 1])) | int(lut[4 * idx + 3])
                    got = (e01 & 0xffff, e01 >> 16, e2 & 0xffff)
                    for L, vals in enumerate(((M, X, Y), (M + o, X, Y + o), (M + o, X + o, Y))):
                        h = min(vals)
                        S = sum(1 << k for k in range(3) if vals[k] == h)
                        want = {1: Pd, 2: Pl, 4: Pu}.get(S, (2 * S - 2 + 14 * mm) << 2)
                        assert got[L] == want, (o, dM, dX, dY, mm, L, hex(got[L]), hex(want))
