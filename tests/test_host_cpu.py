"""CPU tests of the product's host side: library exports, the host tie-break table
(CPython MT19937 emulation) and argument validation -- no GPU needed."""
import ctypes as C
import random
import re

import numpy as np
import pytest

from tests.conftest import ROOT, state_digest


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
        monkeypatch.setenv("GA_RC_SERVERS", str(48 + k))
        e0 = _native.default_engine(0)
        assert _native.default_engine(0) is e0          # same knobs: the cached context
        _native.default_engine(1)
        distributed.device_engines([0, 1])
    assert len(_native._default) == 2                    # one per device for this thread
    assert len(distributed._device_engines) == 1
    del e0
    gc.collect()
    assert sum(r() is not None for r in made) == 4       # the current set's: 2 default + 2 slab engines
