"""Round 3: steady-state score-only fill times of an m x n SplitMix64 DNA pair under the current GA_* knobs.

    GA_FILL_MODE=row GA_COLS_PER_LANE=2 python tools/exp/r3_fills.py [m] [n] [reps]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from globalign_amd import _native  # noqa: E402

m = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000
n = int(sys.argv[2]) if len(sys.argv) > 2 else 100_000
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 4
s1, s2 = bench.splitmix(m, 1), bench.splitmix(n, 2)
tables, _ = bench.problem_tables(s1, s2)
eng = _native.Engine(0)
eng.load(tables.codes(s1), tables.codes(s2), tables)
ts = []
for _ in range(reps):
    cost, _ = eng.fill(traceback=False)
    ts.append(eng.kernel_ms()[0])
knobs = {k: v for k, v in os.environ.items() if k.startswith("GA_")}
print(f"{m}x{n} {knobs} kind={eng.fill_kind()} cost={cost} fill_ms={[round(t, 3) for t in ts]}", flush=True)
