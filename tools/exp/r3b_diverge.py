"""Round 3 (second session): where the GPU walk leaves the oracle's path (walk order), for random cases."""
import random
import sys
import os

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import globalign_amd as ga  # noqa: E402
from oracle import core, transform  # noqa: E402


def levels(s1a, s2a):
    return [0 if (x != "-" and y != "-") else (1 if x == "-" else 2) for x, y in zip(s1a, s2a)]


def case(s1, s2, kw, seed):
    a1, a2, smat, cmat, gos, goc = transform.settings(dict(kw, seq_1=s1, seq_2=s2))
    random.seed(seed)
    ref = core.align(a1, a2, cmat, goc, core.mt_state_array())
    random.seed(seed)
    r = ga.GlobalAligner(max_seq_len_prod=None, **kw).align(s1, s2)
    lr = levels(ref["strings"][0], ref["strings"][2])[::-1]
    lg = levels(r.seq_1_aligned, r.seq_2_aligned)[::-1]
    if lr == lg:
        return None
    k = next((q for q in range(min(len(lr), len(lg))) if lr[q] != lg[q]), min(len(lr), len(lg)))
    i, j = len(s1), len(s2)
    for q in range(k):
        i -= lr[q] != 1
        j -= lr[q] != 2
    return dict(k=k, i=i, j=j, i64=(i - 1) % 64, j64=(j - 1) % 64, ref=lr[k:k + 6], gpu=lg[k:k + 6], prev=lr[max(0, k - 4):k])


rng = random.Random(0)
bad = 0
for t in range(int(sys.argv[1]) if len(sys.argv) > 1 else 40):
    o = rng.choice([0, 1, 6, 7, 10, 126, 127, 300])
    m, n = rng.randint(50, 400), rng.randint(50, 400)
    s1 = "".join(rng.choice("ACGT") for _ in range(m))
    s2 = "".join(rng.choice("ACGT") for _ in range(n))
    res = case(s1, s2, dict(match_score=3, mismatch_score=-2, gap_open_score=-o, gap_extension_score=-1), t)
    if res:
        bad += 1
        print("MISMATCH", t, o, m, n, res, flush=True)
print("bad", bad)
