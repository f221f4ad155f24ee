"""CPU model of the tie-to-tie walk: jump entries built per recompute block, a walker that
advances one entry per trip.  Checks that the trips reproduce the oracle's path move for move and counts them.

    python tools/jump_model.py [N] [TD]     (N x N prefix of the C3 pair; blocks of 64 rows x 64*TD columns)

Entry of state (cell, entering level L), 16 bits:
  * a tie (the rank set S_L has two or more members): bits 1:0 = 0, bits 6:2 = sh = 2S - 2 + 14*(a != b), the
    tie-break table shift the walk uses today (ga_walk.h);
  * otherwise up to 8 moves, move q in bits 2q+1:2q (bit 0: the move lowers j, bit 1: it lowers i; diag 3,
    left 1, up 2; 0 after the last move): the singleton choice x of (cell, L), then the moves of the entry of
    the successor state (cell - d(x), x) as it is built (16 bits kept), or nothing when that state is a tie or
    lies outside the block the entry is built in.
Every entry so built is a run of real moves of the deterministic walk (a valid jump), however its run was cut.
Analysis / test infrastructure only (imports the oracle)."""
import os
import random
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

CODE = {0: 3, 1: 1, 2: 2}     # level of a move -> its 2-bit code
LEVEL = {3: 0, 1: 1, 2: 2}


def build_entries(sets, a, b, m, n, R, C):
    """Entries [3][m][n] (uint16) from the rank sets (oracle layout: 9 bits per cell, 3 per level), built per
    region of R rows x C columns (the recompute blocks): a successor outside the region counts as empty."""
    E = np.zeros((3, m, n), dtype=np.int64)   # as built (the walker's view)
    S = np.zeros((3, m, n), dtype=np.int64)   # as a successor (0 for ties)
    st = sets.reshape(m, n).astype(np.int64)
    mm = (a[:, None] != b[None, :]).astype(np.int64)
    for L in range(3):
        pass
    for i in range(m):                        # row-major within the matrix: successors are up / left
        ri = i % R
        for j in range(n):
            cj = j % C
            for L in range(3):
                s = (st[i, j] >> (3 * L)) & 7
                if s & (s - 1):               # tie
                    E[L, i, j] = (2 * s - 2 + 14 * mm[i, j]) << 2
                    S[L, i, j] = 0
                    continue
                x = {1: 0, 2: 1, 4: 2}[s]
                si, sj = i - (x != 1), j - (x != 2)
                inside = si >= 0 and sj >= 0 and (x == 1 or ri > 0) and (x == 2 or cj > 0)
                succ = S[x, si, sj] if inside else 0
                v = ((succ << 2) | CODE[x]) & 0xFFFF
                E[L, i, j] = v
                S[L, i, j] = v
    return E


def walk(E, path_levels, m, n):
    """Trips from (m, n) entering level 0 (the walk's first step is at (m, n) with level 0), following the
    oracle's path at ties.  Returns (levels reproduced, trips)."""
    i, j, L = m, n, 0
    out = []
    trips = 0
    k = 0
    while i >= 1 and j >= 1 and k < len(path_levels):
        e = int(E[L, i - 1, j - 1])
        trips += 1
        if (e & 3) == 0:                     # tie: the oracle's move (the table decides in the kernel)
            x = path_levels[k]
            out.append(x)
            k += 1
            i, j, L = i - (x != 1), j - (x != 2), x
            if i < 1 or j < 1:
                break
            e = int(E[L, i - 1, j - 1])
            if (e & 3) == 0:
                continue                     # consecutive ties: the next trip resolves it
        q = 0
        while q < 8 and (e >> (2 * q)) & 3:
            x = LEVEL[(e >> (2 * q)) & 3]
            out.append(x)
            k += 1
            i, j, L = i - (x != 1), j - (x != 2), x
            q += 1
    return out, trips


def main():
    import bench
    from oracle import core, transform
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
    TD = int(sys.argv[2]) if len(sys.argv) > 2 else 4
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
    lv = []
    for k in range(len(mid) - 1, -1, -1):
        lv.append(1 if sa[k] == "-" else 2 if sb[k] == "-" else 0)
    E = build_entries(sets, a, b, m, n, 64, 64 * TD)
    got, trips = walk(E, lv, m, n)
    # the interior walk ends at row 0 / column 0; the reference then appends the edge run
    assert got == lv[:len(got)], "trip walk diverged from the oracle path"
    print(f"N={N} TD={TD} moves={len(got)} of {len(lv)} trips={trips} moves_per_trip={len(got) / trips:.2f}")


if __name__ == "__main__":
    main()
