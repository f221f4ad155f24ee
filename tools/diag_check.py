"""Diagnostic: score-only cost of the anti-diagonal kernel vs the row scan vs the C oracle.

    GA_FILL_MODE is set per engine here; prints one line per shape."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from globalign_amd import _native  # noqa: E402
from oracle import core  # noqa: E402


def cost_with(mode, s1, s2, tables, **env):
    os.environ["GA_FILL_MODE"] = mode
    for k, v in env.items():
        os.environ[k] = str(v)
    eng = _native.Engine(0)
    try:
        eng.load(tables.codes(s1), tables.codes(s2), tables)
        return int(eng.fill(traceback=False)[0])
    except Exception as e:  # noqa: BLE001
        return repr(e)
    finally:
        eng.close()
        for k in env:
            del os.environ[k]


for m, n in [(1, 64), (2, 64), (5, 64), (70, 64), (100, 63), (100, 130), (300, 1000), (1000, 1000), (3000, 5000),
             (4000, 60000)]:
    s1, s2 = bench.splitmix(m, 5), bench.splitmix(n, 6)
    tables, _ = bench.problem_tables(s1, s2)
    tab = core.Tables({x: {y: int(tables.sub[tables.code[x] * tables.K + tables.code[y]]) for y in tables.keys}
                       for x in tables.keys})
    a, b = tab.codes(s1), tab.codes(s2)
    big = (tab.max_cost + 1) * max(m, n)
    row0, col0 = core.boundary(tab, a, b, tables.gap_open, big)
    ref = int(min(core.fill_score(tab, a, b, tables.gap_open, row0, col0)))
    print(m, n, "oracle", ref, "row", cost_with("row", s1, s2, tables), "diag", cost_with("diag", s1, s2, tables),
          "diag_nwc4", cost_with("diag", s1, s2, tables, GA_FILL_NWC=4), flush=True)
