"""Run structure of a traceback walk (analysis for the tie-to-tie walker).

    python tools/walk_runs.py [N]      (default 20000: an N x N prefix of the C3 pair)

Fills the rank sets with the C oracle, walks with random.seed(0), rebuilds the path from the alignment
strings and reports: the share of steps whose set (at the entering level) is a tie, the run lengths
between ties, and how many jumps a walker needs when its jumps stop at ties, at tile edges of T cells
and after at most K moves.  Test/analysis infrastructure only (imports the oracle)."""
import os
import random
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from oracle import core, transform  # noqa: E402


def main():
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 20000
    wl = bench.WORKLOADS["c3"]
    s1, s2 = bench.workload_pair(dict(wl, m=N, n=N))
    _, _, _, cmat, _, o = transform.settings(dict(wl["scoring"], seq_1=s1[:64], seq_2=s2[:64]))
    tab = core.Tables(cmat)
    a, b = tab.codes(s1), tab.codes(s2)
    m, n = len(a), len(b)
    big = (tab.max_cost + 1) * max(m, n)
    row0, col0 = core.boundary(tab, a, b, o, big)
    sets = np.zeros(m * n, np.uint16)
    last = np.zeros(3, np.int64)
    core.lib().gao_fill_sets(a, m, b, n, tab.sub, tab.K, tab.gh, tab.gv, o, row0, col0, sets, last)
    random.seed(0)
    r = core.align(s1, s2, cmat, o, core.mt_state_array(), mode="sets")
    sa, mid, sb = r["strings"]
    # path from the end: the strings are in forward order; the walk visits them backwards
    i, j, L = m, n, 0
    states = []  # (i, j, L entering) per dispatch
    first = True
    for k in range(len(mid) - 1, -1, -1):
        if i == 0 or j == 0:
            break
        states.append((i, j, 0 if first else L))
        first = False
        if sa[k] == "-":
            lvl = 1
        elif sb[k] == "-":
            lvl = 2
        else:
            lvl = 0
        i -= lvl != 1
        j -= lvl != 2
        L = lvl
    S = np.array([(int(sets[(ii - 1) * n + jj - 1]) >> (3 * LL)) & 7 for ii, jj, LL in states])
    tie = np.array([bin(s).count("1") > 1 for s in S])
    nst = len(states)
    print(f"N={N} steps={nst} ties={tie.sum()} ({100 * tie.mean():.2f} %) ndispatch={r['ndispatch']}")
    # moves
    lv = [states[k + 1][2] for k in range(nst - 1)]
    print("moves diag/left/up:", [lv.count(x) for x in range(3)])
    # runs between ties
    idx = np.flatnonzero(tie)
    runs = np.diff(np.concatenate([[-1], idx, [nst]])) - 1
    print(f"run lengths: mean {runs.mean():.2f} median {np.median(runs)} p90 {np.percentile(runs, 90)}")
    for T in (32, 64):
        for K in (6, 7, 8, 15, 127):
            # a trip: the tie move at its start (if the walker stands on a tie), then the run of
            # deterministic moves until a tie, the tile's edge or K moves
            trips = 0
            k = 0
            while k < nst:
                if tie[k]:
                    k += 1
                ii, jj, _ = states[k] if k < nst else (0, 0, 0)
                ti, tj = (ii - 1) // T, (jj - 1) // T
                c = 0
                while k < nst and not tie[k] and c < K:
                    i2, j2, _ = states[k]
                    if (i2 - 1) // T != ti or (j2 - 1) // T != tj:
                        break
                    k += 1
                    c += 1
                trips += 1
            print(f"tile {T:3d} cap {K:3d}: {trips} trips, {nst / trips:.2f} moves per trip")

if __name__ == "__main__":
    main()
