"""Round 3: the recompute walk (GA_RC=1) against the stored-words path (GA_RC=0) on the same inputs:
cost, strings and random state must be identical; then C3 timings of both.

    python tools/exp/r3_rc_check.py [quick]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

import bench  # noqa: E402
from globalign_amd import _native  # noqa: E402

mt0 = np.random.RandomState(0).randint(0, 2**32, size=625, dtype=np.uint64).astype(np.uint32)
mt0[624] = 624


def run(eng, s1, s2, rc):
    os.environ["GA_RC"] = "1" if rc else "0"
    t0 = time.perf_counter()
    r = eng.align(mt0, s1, s2)
    dt = (time.perf_counter() - t0) * 1e3
    return r, dt, eng.fill_kind(), eng.timings()


cases = [(300, 300, "dna", None), (1000, 777, "dna", None), (4097, 3000, "dna", None), (3000, 9000, "dna", None),
         (20000, 20000, "dna", None), (5000, 5000, "protein", bench.PROTEIN_SCORING),
         (2000, 2000, "dna", dict(match_score=1, mismatch_score=-1, gap_open_score=-20, gap_extension_score=-1))]
if len(sys.argv) < 2:
    cases.append((100000, 100000, "dna", None))
eng = _native.Engine(0)
ok = True
for m, n, alpha, scoring in cases:
    s1, s2 = bench.splitmix(m, 1, alpha), bench.splitmix(n, 2, alpha)
    tables, _ = bench.problem_tables(s1, s2, scoring)
    eng.load(tables.codes(s1), tables.codes(s2), tables)
    a, ta, ka, tma = run(eng, s1, s2, False)
    b, tb, kb, tmb = run(eng, s1, s2, True)
    same = a[0] == b[0] and a[1] == b[1] and a[2] == b[2] and np.array_equal(a[3], b[3])
    ok &= same
    print(f"{m}x{n} {alpha} same={same} cost={a[0]}/{b[0]} kinds={ka[0]}/{kb[0]} T={kb[1]} "
          f"wall_ms {ta:.2f}/{tb:.2f} fill {tma['fill_ms']:.3f}/{tmb['fill_ms']:.3f} walk {tma['walk_ms']:.3f}/{tmb['walk_ms']:.3f}",
          flush=True)
    if m * n >= 10**10:
        for _ in range(3):
            b, tb, kb, tmb = run(eng, s1, s2, True)
            print(f"  rc again wall {tb:.2f} ms fill {tmb['fill_ms']:.3f} walk {tmb['walk_ms']:.3f} call {tmb['call_ms']:.3f}",
                  flush=True)
print("ALL SAME" if ok else "MISMATCH", flush=True)
