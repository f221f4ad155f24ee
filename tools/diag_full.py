"""Diagnostic: full (M, X, Y) matrices of the anti-diagonal kernel vs the row scan (GA_FILL_FULL);
prints the first differing cells."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from globalign_amd import _native  # noqa: E402


def full_with(mode, s1, s2, tables):
    os.environ["GA_FILL_MODE"] = mode
    eng = _native.Engine(0)
    try:
        eng.load(tables.codes(s1), tables.codes(s2), tables)
        return eng.fill(full=True)
    finally:
        eng.close()


for m, n in [(1, 64), (3, 64), (300, 130), (1100, 200)]:
    s1, s2 = bench.splitmix(m, 5), bench.splitmix(n, 6)
    tables, _ = bench.problem_tables(s1, s2)
    cr, fr = full_with("row", s1, s2, tables)
    cd, fd = full_with("diag", s1, s2, tables)
    bad = np.argwhere(fr[1:, 1:] != fd[1:, 1:])
    print(m, n, "cost row", cr, "diag", cd, "bad cells", len(bad), flush=True)
    for (i, j, k) in bad[:8]:
        print("   cell", i + 1, j + 1, "field", "MXY"[k], "row", fr[i + 1, j + 1, k], "diag", fd[i + 1, j + 1, k])
