"""Round 5 debug: first difference between the device walk and the oracle on small problems (walker 3-op chain)."""
import random
import sys

import numpy as np

sys.path.insert(0, ".")
from globalign_amd import _native  # noqa: E402
from globalign_amd.scoring import validate_and_transform_args  # noqa: E402
from oracle import core, transform  # noqa: E402
from tests.conftest import splitmix_seq  # noqa: E402

DNA = dict(match_score=2, mismatch_score=-3, gap_open_score=-5, gap_extension_score=-1)
import os  # noqa: E402
for (m, n, rc, same) in [(256, 256, "1", "0"), (256, 256, "1", "1"), (1000, 1300, "1", "1")]:
    os.environ["GA_RC"] = rc
    if same == "1":
        os.environ["GA_DBG_UPLOAD_SAME"] = "1"
    else:
        os.environ.pop("GA_DBG_UPLOAD_SAME", None)
    s1, s2 = splitmix_seq(m, 11, "dna"), splitmix_seq(n, 12, "dna")
    a1, a2, smat, cmat, gos, goc = transform.settings(dict(DNA, seq_1=s1, seq_2=s2))
    random.seed(m + n)
    mt = np.array(random.getstate()[1], dtype=np.uint32)
    ref = core.align(a1, a2, cmat, goc, mt)
    _, _, _, cmat2, _, goc2, _ = validate_and_transform_args(None, None, s1[:64], s2[:64], **DNA)
    tables = _native.CostTables(cmat2, goc2)
    eng = _native.Engine(0)
    eng.load(tables.codes(a1), tables.codes(a2), tables)
    cost, strings, status, mt_after = eng.align(mt, a1, a2)
    kind = eng.fill_kind()
    eng.close()
    A, R = strings[0], ref["strings"][0]
    L = min(len(A), len(R))
    first = next((k for k in range(L) if strings[0][k] != R[k] or strings[1][k] != ref["strings"][1][k]
                  or strings[2][k] != ref["strings"][2][k]), None)
    print(m, n, "rc", rc, "same", same, kind, "cost", int(cost), ref["cost"], "len", len(A), len(R), "first diff", first)
    def levels(st):
        a, b = st[0][::-1], st[2][::-1]
        return [1 if x == "-" else 2 if y == "-" else 0 for x, y in zip(a, b)]
    ld, lr = levels(strings), levels(ref["strings"])
    fd = next((k for k in range(min(len(ld), len(lr))) if ld[k] != lr[k]), None)
    if fd is not None:
        i, j = m, n
        for k in range(fd):
            i -= lr[k] != 1
            j -= lr[k] != 2
        print("  first differing move D", fd, "at cell", (i, j), "dev", ld[max(0, fd - 8):fd + 8], "ref", lr[max(0, fd - 8):fd + 8])
    if first is not None:
        lo = max(0, first - 5)
        for k in range(3):
            print("  dev", strings[k][lo:first + 12])
            print("  ref", ref["strings"][k][lo:first + 12])
