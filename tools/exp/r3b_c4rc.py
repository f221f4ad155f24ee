"""C4 with full traceback on one GPU: recompute walk at checkpoint spacings 256 / 128 / 64 against the banded path;
prints fill / walk ms and digests of the alignment and the final random state (all must agree)."""
import hashlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

import bench  # noqa: E402
from globalign_amd import _native  # noqa: E402

wl = bench.WORKLOADS["c4tb"]
s1, s2 = bench.workload_pair(wl)
tables, _ = bench.problem_tables(s1, s2, wl["scoring"])
mt0 = np.random.RandomState(0).randint(0, 2**32, size=625, dtype=np.uint64).astype(np.uint32)
mt0[624] = 624
for cfg in [("256", "1"), ("128", "1"), ("64", "1"), ("0", "0")]:
    os.environ["GA_RC_EVERY"], os.environ["GA_RC"] = cfg
    os.environ["GA_RC_BUDGET_MB"] = "200000"
    eng = _native.Engine(0)
    eng.load(tables.codes(s1), tables.codes(s2), tables)
    for rep in range(2):
        cost, (a, mid, b), status, mt = eng.align(mt0, s1, s2)
        t = eng.timings()
        assert status == 0 and a.replace("-", "") == s1 and b.replace("-", "") == s2
        dig = hashlib.sha256("\n".join([a, mid, b]).encode()).hexdigest()[:16]
        st = hashlib.sha256(",".join(str(int(w)) for w in mt).encode()).hexdigest()[:16]
        print(f"every={cfg[0]} rc={cfg[1]} cost={cost} len={len(mid)} aln={dig} state={st} fill={t['fill_ms']:.1f} "
              f"walk={t['walk_ms']:.1f} call={t['call_ms']:.1f} kind={eng.fill_kind()}", flush=True)
    eng.close()
