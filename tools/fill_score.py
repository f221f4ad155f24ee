"""Diagnostic: K score-only fills of an m x n SplitMix64 DNA pair (the lane kernel under GA_FILL_MODE=lane), for
profilers (rocprofv3 --pmc passes of the fill alone).

    python tools/fill_score.py [m] [n] [K]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from globalign_amd import _native  # noqa: E402

m = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000
n = int(sys.argv[2]) if len(sys.argv) > 2 else 100_000
K = int(sys.argv[3]) if len(sys.argv) > 3 else 3
s1, s2 = bench.splitmix(m, 1), bench.splitmix(n, 2)
tables, _ = bench.problem_tables(s1, s2)
eng = _native.Engine(0)
eng.load(tables.codes(s1), tables.codes(s2), tables)
for _ in range(K):
    cost, _ = eng.fill(traceback=False)
print("cost", cost, "fill_ms", eng.kernel_ms()[0], "kind", eng.fill_kind())
