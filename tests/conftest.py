import hashlib
import json
import os
import random
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI)")
    config.addinivalue_line("markers", "slow: long-running parity case")


def state_digest(state=None):
    st = random.getstate() if state is None else state
    return hashlib.sha256(",".join(str(w) for w in st[1]).encode()).hexdigest()[:32]


def aln_digest(a, mid, b):
    return hashlib.sha256("\n".join([a, mid, b]).encode()).hexdigest()[:16]


def load_matrix(name):
    d = json.load(open(os.path.join(ROOT, "globalign_amd", "data", name + ".json")))
    L = list(d["letters"])
    return {x: {y: d["scores"][i][j] for j, y in enumerate(L)} for i, x in enumerate(L)}


M64 = (1 << 64) - 1


def splitmix_seq(length, seed, alphabet):
    """SURVEY 8d generator (pure Python; small lengths only)."""
    state = seed & M64
    out = []
    for _ in range(length):
        state = (state + 0x9E3779B97F4A7C15) & M64
        z = state
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
        z = z ^ (z >> 31)
        out.append("ACGT"[z >> 62] if alphabet == "dna" else "ARNDCQEGHILKMFPSTWYV"[((z >> 32) * 20) >> 32])
    return "".join(out)


@pytest.fixture(autouse=True)
def _restore_random_state():
    st = random.getstate()
    yield
    random.setstate(st)


def set_knob(monkeypatch, name, value):
    """A GA_* option for engines created from here on, through _native.OPTIONS (ga_ctx_create_opts): the library
    reads only its shipped knobs from the environment, and none of the test variants or fault injections."""
    from globalign_amd import _native
    monkeypatch.setitem(_native.OPTIONS, name, str(value))


def del_knob(monkeypatch, name, raising=False):
    from globalign_amd import _native
    monkeypatch.delitem(_native.OPTIONS, name, raising=False)
    monkeypatch.delenv(name, raising=False)
