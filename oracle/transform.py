"""Score <-> cost transform restated for the oracle.  TEST INFRASTRUCTURE ONLY.

Restates /root/reference/src/globalign/start.py (branch selection of
validate_and_transform_args :236-343, create_scoring_mat :431-449,
create_costing_mat :451-468, get_max_val :488-497,
scoring_mat_to_costing_mat :500-557, costing_mat_to_scoring_mat :559-612,
read_scoring_mat :378-428) and conclude.py final_cost_to_score :154-177.
Argument *validation* (error cases) is not restated here; the product's own
validation is tested against the golden fixtures instead.
"""
import math


def max_val(mat):
    return max(max(row.values()) for row in mat.values())


def scores_to_costs(smat, b):
    dd, di = math.floor(b / 2), math.ceil(b / 2)
    out = {}
    for x, row in smat.items():
        out[x] = {}
        for y, s in row.items():
            if x == "-" and y != "-":
                out[x][y] = -s + dd
            elif y == "-" and x != "-":
                out[x][y] = -s + di
            else:
                out[x][y] = -s + dd + di
    return out


def costs_to_scores(cmat, b):
    dd, di = math.floor(b / 2), math.ceil(b / 2)
    out = {}
    for x, row in cmat.items():
        out[x] = {}
        for y, c in row.items():
            if x == "-" and y != "-":
                out[x][y] = dd - c
            elif y == "-" and x != "-":
                out[x][y] = di - c
            else:
                out[x][y] = dd + di - c
    return out


def simple_matrix(alphabet, same, gap, other):
    keys = list(alphabet) + ["-"]
    return {x: {y: (same if x == y else gap if "-" in (x, y) else other) for y in keys} for x in keys}


def read_mtx_rows(letters, scores):
    return {x: {y: scores[i][j] for j, y in enumerate(letters)} for i, x in enumerate(letters)}


def settings(kw, blosum=None, mtx=None):
    """Returns (seq_1, seq_2, scoring_mat, costing_mat, gap_open_score, gap_open_cost)
    for a valid kwargs dict, following start.py:236-343."""
    s1, s2 = kw["seq_1"].upper(), kw["seq_2"].upper()

    def iv(k, d):
        v = kw.get(k)
        return d if v is None else int(v)

    ms, mms, gos, ges = iv("match_score", 2), iv("mismatch_score", -3), iv("gap_open_score", -4), iv("gap_extension_score", -2)
    mc, goc, gec = iv("mismatch_cost", 5), iv("gap_open_cost", 4), iv("gap_extension_cost", 3)
    if kw.get("gap_open_score") is not None:
        goc = -gos
    else:
        gos = -goc
    alphabet = sorted(set(s1) | set(s2))
    if kw.get("scoring_mat_name") is not None:
        smat = blosum
        cmat = scores_to_costs(smat, max_val(smat))
    elif kw.get("scoring_mat_path") is not None:
        smat = mtx
        cmat = scores_to_costs(smat, max_val(smat))
    elif any(kw.get(k) is not None for k in ("mismatch_cost", "gap_open_cost", "gap_extension_cost")):
        cmat = simple_matrix(alphabet, 0, gec, mc)
        smat = costs_to_scores(cmat, ms)
    else:
        smat = simple_matrix(alphabet, ms, ges, mms)
        cmat = scores_to_costs(smat, ms)
    return s1, s2, smat, cmat, gos, goc


def cost_to_score(cost, m, n, b):
    return n * math.floor(b / 2) + m * math.ceil(b / 2) - cost
