"""Pure-Python port of globalign's DP loop.  TEST / BASELINE INFRASTRUCTURE ONLY.

Used by bench.py as the ``cpu_baseline`` (kind "port"): it keeps the
reference's data structures and per-cell costs -- a nested list of
(level0, level1, level2) tuples, one Python call per cell that takes three
``min`` over tuples and dict-of-dict cost lookups, and a traceback that
rebuilds an 18-``random.choice`` dispatcher per step -- so its cells/s is
representative of running the reference itself on the same host
(/root/reference/src/globalign/globaligner.py:317-392, :395-685, :756-821).
"""
import random


def next_costs(dp_array, i, j, seq_1, seq_2, costing_mat, gap_open_cost):
    """One cell, in the call shape of the reference's get_next_best_costs (globaligner.py:317-363):
    keyword arguments, nine nested-list reads of the three neighbours, three tuples, three min()."""
    a_idx, b_idx = i - 1, j - 1
    via_diag = (dp_array[i - 1][j - 1][0], dp_array[i - 1][j - 1][1], dp_array[i - 1][j - 1][2])
    via_left = (dp_array[i][j - 1][0] + gap_open_cost, dp_array[i][j - 1][1],
                dp_array[i][j - 1][2] + gap_open_cost)
    via_up = (dp_array[i - 1][j][0] + gap_open_cost, dp_array[i - 1][j][1] + gap_open_cost,
              dp_array[i - 1][j][2])
    return (min(via_diag) + costing_mat[seq_1[a_idx]][seq_2[b_idx]],
            min(via_left) + costing_mat["-"][seq_2[b_idx]],
            min(via_up) + costing_mat[seq_1[a_idx]]["-"])


def fill(a, b, C, o, max_cost):
    """make_dp_array (:756-821) + dp_array_forward (:366-392): one keyword call per cell."""
    m, n = len(a), len(b)
    T = [[None] * (n + 1) for _ in range(m + 1)]
    big = (max_cost + 1) * max(m, n)
    T[0][0] = (0, 0, 0)
    acc = o
    for j in range(1, n + 1):
        acc += C["-"][b[j - 1]]
        T[0][j] = (big, acc, big)
    acc = o
    for i in range(1, m + 1):
        acc += C[a[i - 1]]["-"]
        T[i][0] = (big, big, acc)
    for i in range(1, m + 1):
        for j in range(1, n + 1):
            T[i][j] = next_costs(dp_array=T, i=i, j=j, seq_1=a, seq_2=b, costing_mat=C, gap_open_cost=o)
    return T


_MOVES = {0: (-1, -1), 1: (0, -1), 2: (-1, 0)}


def _dispatch(ranks, is_match):
    ch = random.choice
    table = {}
    for flag in (True, False):
        mm = 0
        table[((0, 0, 0), flag)] = ch((mm, 1, 2))
        table[((0, 0, 2), flag)] = ch((mm, 1))
        table[((0, 2, 0), flag)] = ch((mm, 2))
        table[((2, 0, 0), flag)] = ch((1, 2))
        table[((1, 1, 1), flag)] = ch((mm, 1, 2))
        table[((1, 1, 2), flag)] = ch((mm, 1))
        table[((1, 2, 1), flag)] = ch((mm, 2))
        table[((2, 1, 1), flag)] = ch((1, 2))
        table[((2, 2, 2), flag)] = ch((mm, 1, 2))
    key = (tuple(ranks), is_match)
    if key in table:
        return table[key]
    lo = min(ranks)
    return ranks.index(lo)


def traceback(T, a, b, C, o):
    """Normal (min(m, n) >= 2) walk with the reference's tie-break draws."""
    m, n = len(a), len(b)
    out_a, out_m, out_b = [], [], []
    i, j, level, first = m, n, 0, True
    for _ in range(m + n + 1):
        v = T[i][j]
        if first or level == 0:
            c = v
        elif level == 1:
            c = (v[0] + o, v[1], v[2] + o)
        else:
            c = (v[0] + o, v[1] + o, v[2])
        s = sorted(c)
        ranks = [s.index(x) for x in c]
        x, y = a[i - 1], b[j - 1]
        level = _dispatch(ranks, x == y)
        if level == 0:
            out_a.append(x); out_m.append("|" if x == y else "*"); out_b.append(y)
        elif level == 1:
            out_a.append("-"); out_m.append(" "); out_b.append(y)
        else:
            out_a.append(x); out_m.append(" "); out_b.append("-")
        di, dj = _MOVES[level]
        i, j = i + di, j + dj
        if first:
            first = False
            if i == 0 and j == 0:
                break
            continue
        if i == 0:
            for jj in range(j, 0, -1):
                out_a.append("-"); out_m.append(" "); out_b.append(b[jj - 1])
            break
        if j == 0:
            for ii in range(i, 0, -1):
                out_a.append(a[ii - 1]); out_m.append(" "); out_b.append("-")
            break
    return "".join(reversed(out_a)), "".join(reversed(out_m)), "".join(reversed(out_b)), min(T[m][n])
