#!/usr/bin/env python3
"""Optimal global alignment on MI355X -- drop-in for globalign's hot path.

Public surface (mirrors iamgiddyaboutgit/globalign src/globalign/globaligner.py):

  find_global_alignment(...) -> AlignmentResults        globaligner.py:132-314
  make_dp_array / dp_array_forward / dp_array_backward   globaligner.py:756-821, 366-392, 395-593
  main()  (the `globaligner` CLI)                        globaligner.py:23-129
plus GlobalAligner, a reusable façade bound to one GPU that can lift the
reference's m*n < 2e7 cap.

The three DP functions run on the GPU through the C ABI in
include/globalign_amd.h; there is no CPU fallback.  Tie-breaking consumes the
process-global ``random`` state exactly like the reference (18
``random.choice`` calls per traceback step), so with the same
``random.seed`` the alignment strings are identical.
"""
import argparse
import random
import sys
from pathlib import Path

import numpy as np

from . import _native
from .results import AlignmentResults, final_cost_to_score
from .scoring import MAX_SEQ_LEN_PROD, get_max_val, validate_and_transform_args

__version__ = "0.1.0"


def _mt_words():
    st = random.getstate()
    return np.array(st[1], dtype=np.uint32)


def _set_mt_words(words):
    # only the MT words move: random.choice leaves gauss_next (the state's third item) alone
    st = random.getstate()
    random.setstate((st[0], tuple(int(x) for x in words), st[2]))


class GlobalAligner:
    """Reusable aligner on one GPU or several.

    ``GlobalAligner(**settings).align(seq_1, seq_2)`` accepts the same keyword
    settings as find_global_alignment (scores, costs, matrix name/path, gap
    options) and returns an AlignmentResults.  ``max_seq_len_prod=None``
    lifts the reference's m*n < 2e7 API cap (the device path is sized for
    100k x 100k and beyond); ``traceback=False`` returns the score only.
    ``devices=[0, 1, ...]`` cuts seq_2's columns into one slab per listed GPU
    of this process (distributed.align_devices: each slab's fill writes its right
    edge straight into its neighbour's GPU memory over xGMI while both fills
    run, the walk is handed right to left);
    the result is identical to the one-GPU result.  For one process per GPU
    use globalign_amd.distributed (torch.distributed / RCCL).
    """

    def __init__(self, scoring_mat_name=None, scoring_mat_path=None, match_score=None, mismatch_score=None,
                 mismatch_cost=None, gap_open_score=None, gap_open_cost=None, gap_extension_score=None,
                 gap_extension_cost=None, device=0, max_seq_len_prod=MAX_SEQ_LEN_PROD, traceback=True, devices=None):
        self.settings = dict(scoring_mat_name=scoring_mat_name, scoring_mat_path=scoring_mat_path,
                             match_score=match_score, mismatch_score=mismatch_score, mismatch_cost=mismatch_cost,
                             gap_open_score=gap_open_score, gap_open_cost=gap_open_cost,
                             gap_extension_score=gap_extension_score, gap_extension_cost=gap_extension_cost)
        self.devices = [int(d) for d in devices] if devices is not None else [int(device)]
        if not self.devices:
            raise ValueError("devices must name at least one GPU")
        self.device = self.devices[0]
        self.max_seq_len_prod = max_seq_len_prod
        self.traceback = traceback

    def align(self, seq_1=None, seq_2=None, input_fasta=None, output=None):
        good = validate_and_transform_args(input_fasta, output, seq_1, seq_2, max_seq_len_prod=self.max_seq_len_prod,
                                           **self.settings)
        return _align_validated(good, device=self.device, traceback=self.traceback, devices=self.devices)


    def align_repeated(self, seq_1, seq_2, count):
        """`count` alignments of one pair, as `count` consecutive find_global_alignment calls make them: each
        starts from the global random state the previous one left, so the tie-breaks -- and with them the
        co-optimal alignment returned -- differ from call to call exactly as in the reference.  On one GPU
        the walk of alignment k runs beside the fill of alignment k+1 (ga_problem_align_many).
        -> list of AlignmentResults."""
        good = validate_and_transform_args(None, None, seq_1, seq_2, max_seq_len_prod=self.max_seq_len_prod,
                                           **self.settings)
        s1, s2, scoring_mat, costing_mat, gos, goc, output = good
        if int(count) <= 0:
            return []  # a loop of zero find_global_alignment calls
        if len(self.devices) > 1 or not self.traceback or min(len(s1), len(s2)) < 2:
            # (degenerate lengths may raise the reference's IndexError mid-way: one call at a time)
            return [_align_validated(good, device=self.device, traceback=self.traceback, devices=self.devices)
                    for _ in range(int(count))]
        tables = _native.CostTables(costing_mat, goc)
        eng = _native.default_engine(self.device)
        eng.load(tables.codes(s1), tables.codes(s2), tables)
        mt0 = _mt_words()
        runs, mt = eng.align_many(mt0, s1, s2, int(count))
        if any(status == _native.GA_TB_INDEX_ERROR for _, _, status in runs):
            # consecutive reference calls stop at the first IndexError, with the random state that call
            # left: replay them one at a time from the starting state (never reached for min(m, n) >= 2)
            _set_mt_words(mt0)
            return [_align_validated(good, device=self.device, traceback=True) for _ in range(int(count))]
        _set_mt_words(mt)
        out = []
        for cost, (a, mid, b), status in runs:
            score = final_cost_to_score(cost=cost, m=len(s1), n=len(s2), max_score=get_max_val(scoring_mat))
            out.append(AlignmentResults(a, mid, b, cost, score, scoring_mat, costing_mat, gos, goc, output))
        return out


def _align_validated(good, device=0, traceback=True, devices=None):
    seq_1, seq_2, scoring_mat, costing_mat, gap_open_score, gap_open_cost, output = good
    tables = _native.CostTables(costing_mat, gap_open_cost)
    if devices is not None and len(devices) > 1 and min(len(seq_1), len(seq_2)) >= 2 and len(seq_2) >= len(devices):
        from . import distributed
        cost, strings, status, mt = distributed.align_devices(devices, seq_1, seq_2, tables.codes(seq_1),
                                                              tables.codes(seq_2), tables, _mt_words(),
                                                              traceback=traceback)
        if traceback:
            _set_mt_words(mt)
            if status == _native.GA_TB_INDEX_ERROR:
                raise IndexError("string index out of range")
            a, mid, b = strings
        else:
            a = mid = b = None
        score = final_cost_to_score(cost=cost, m=len(seq_1), n=len(seq_2), max_score=get_max_val(scoring_mat))
        return AlignmentResults(a, mid, b, cost, score, scoring_mat, costing_mat, gap_open_score, gap_open_cost,
                                output)
    eng = _native.default_engine(device)
    eng.load(tables.codes(seq_1), tables.codes(seq_2), tables)
    if traceback:
        cost, (a, mid, b), status, mt = eng.align(_mt_words(), seq_1, seq_2)
        _set_mt_words(mt)  # the reference's random.choice calls advance the global state
        if status == _native.GA_TB_INDEX_ERROR:
            raise IndexError("string index out of range")  # reference behaviour for m==1 / n==1 walks (A.5)
    else:
        cost, _ = eng.fill(traceback=False)
        a = mid = b = None
    score = final_cost_to_score(cost=cost, m=len(seq_1), n=len(seq_2), max_score=get_max_val(scoring_mat))
    return AlignmentResults(a, mid, b, cost, score, scoring_mat, costing_mat, gap_open_score, gap_open_cost, output)


def find_global_alignment(input_fasta=None, output=None, seq_1=None, seq_2=None, scoring_mat_name=None,
                          scoring_mat_path=None, match_score=None, mismatch_score=None, mismatch_cost=None,
                          gap_open_score=None, gap_open_cost=None, gap_extension_score=None,
                          gap_extension_cost=None) -> AlignmentResults:
    """Optimal global alignment of seq_1 and seq_2 (Needleman-Wunsch / Gotoh affine gaps).

    Same arguments, defaults, validation and result as globalign's
    find_global_alignment; the DP fill and traceback run on the GPU."""
    good = validate_and_transform_args(input_fasta, output, seq_1, seq_2, scoring_mat_name, scoring_mat_path,
                                       match_score, mismatch_score, mismatch_cost, gap_open_score, gap_open_cost,
                                       gap_extension_score, gap_extension_cost)
    return _align_validated(good)


# --------------------------------------------------------------------------------
# The reference's DP building blocks, over its nested-list representation
# (list of rows of (level0, level1, level2) tuples).  They are thin shims over
# the same device kernels and exist so code written against globalign's
# internals (e.g. its own test-suite) keeps working.

def make_dp_array(seq_1, seq_2, costing_mat, max_cost, gap_open_cost):
    """(m+1) x (n+1) list with row 0 / column 0 set and None inside (globaligner.py:756-821)."""
    m, n = len(seq_1), len(seq_2)
    dp = [[None] * (n + 1) for _ in range(m + 1)]
    big = (max_cost + 1) * max(m, n)
    dp[0][0] = (0, 0, 0)
    if n >= 1:
        x = gap_open_cost + costing_mat["-"][seq_2[0]]
        dp[0][1] = (big, x, big)
        for j in range(2, n + 1):
            x += costing_mat["-"][seq_2[j - 1]]
            dp[0][j] = (big, x, big)
    else:
        return dp
    if m >= 1:
        y = gap_open_cost + costing_mat[seq_1[0]]["-"]
        dp[1][0] = (big, big, y)
        for i in range(2, m + 1):
            y += costing_mat[seq_1[i - 1]]["-"]
            dp[i][0] = (big, big, y)
    return dp


def _boundary_arrays(dp_array, m, n):
    row0 = np.array([dp_array[0][j] for j in range(n + 1)], dtype=np.int64).reshape(-1)
    col0 = np.array([dp_array[i][0] for i in range(m + 1)], dtype=np.int64).reshape(-1)
    if np.abs(np.concatenate([row0, col0])).max(initial=0) >= 2 ** 31:
        raise OverflowError("boundary values exceed the int32 range of the device path")
    return row0.astype(np.int32), col0.astype(np.int32)


def dp_array_forward(dp_array, seq_1, seq_2, costing_mat, gap_open_cost):
    """Fill dp_array[i][j] for i, j >= 1 in place from its row 0 / column 0 (globaligner.py:366-392)."""
    m, n = len(seq_1), len(seq_2)
    if m == 0 or n == 0:
        return None
    tables = _native.CostTables(costing_mat, gap_open_cost)
    row0, col0 = _boundary_arrays(dp_array, m, n)
    eng = _native.default_engine()
    eng.load(tables.codes(seq_1), tables.codes(seq_2), tables, row0=row0, col0=col0)
    _, full = eng.fill(full=True)
    for i in range(1, m + 1):
        row = dp_array[i]
        fi = full[i]
        for j in range(1, n + 1):
            row[j] = (int(fi[j, 0]), int(fi[j, 1]), int(fi[j, 2]))
    return None


def dp_array_backward(dp_array, seq_1, seq_2, costing_mat, gap_open_cost):
    """Traceback of a filled dp_array -> (seq_1_aligned, middle_part, seq_2_aligned, cost) (globaligner.py:395-593).

    Like the reference it walks the CALLER's cells (edited or hand-made ones included): the whole
    array goes to the device, a kernel derives every cell's traceback word from its (M, X, Y), and
    the walk kernel follows them.  Every interior cell must hold a triple (the reference would
    raise TypeError on a None it walks into; here any None raises it)."""
    m, n = len(seq_1), len(seq_2)
    tables = _native.CostTables(costing_mat, gap_open_cost)
    try:
        cells = np.array([[tuple(c) for c in row] for row in dp_array], dtype=np.int64)
    except TypeError:
        raise TypeError("'NoneType' object is not subscriptable") from None
    if cells.shape != (m + 1, n + 1, 3):
        raise IndexError("list index out of range")
    if np.abs(cells).max(initial=0) >= 2 ** 31:
        raise OverflowError("dp_array values exceed the int32 range of the device path")
    cells = cells.astype(np.int32)
    row0, col0 = cells[0].reshape(-1).copy(), cells[:, 0].reshape(-1).copy()
    eng = _native.default_engine()
    eng.load(tables.codes(seq_1), tables.codes(seq_2), tables, row0=row0, col0=col0)
    cost = eng.set_cells(cells)
    (a, mid, b), status, mt = eng.traceback(_mt_words(), seq_1, seq_2)
    _set_mt_words(mt)
    if status == _native.GA_TB_INDEX_ERROR:
        raise IndexError("string index out of range")
    return a, mid, b, cost


def _cli_version():
    """version('globalign') as the reference's --version prints it (globaligner.py:31-36): the installed
    globalign distribution's version, this package's own when globalign itself is not installed."""
    from importlib.metadata import PackageNotFoundError, version
    try:
        return version("globalign")
    except PackageNotFoundError:
        return __version__


def main(argv=None):
    """The `globaligner` command line (globaligner.py:23-129)."""
    parser = argparse.ArgumentParser(description="Perform optimal global alignment of two nucleotide or amino acid "
                                                 "sequences.")
    parser.add_argument("--version", action="version", version=_cli_version(), help="Prints the version and exits.")
    parser.add_argument("-i", "--input_fasta", required=False,
                        help="FASTA file with the two sequences to align (only the first 2 records are used).")
    parser.add_argument("-o", "--output", required=False,
                        help="Output file for the alignment; stdout when omitted.")
    parser.add_argument("--seq_1", required=False, help="First sequence to align.")
    parser.add_argument("--seq_2", required=False, help="Second sequence to align.")
    parser.add_argument("--scoring_mat_name", required=False, choices=["BLOSUM50", "BLOSUM62"],
                        help="Either 'BLOSUM50' or 'BLOSUM62'.")
    parser.add_argument("--scoring_mat_path", required=False, help="Path to a custom scoring matrix file.")
    parser.add_argument("--match_score", required=False, help="Score for a match (default 2).")
    parser.add_argument("--mismatch_score", required=False, help="Score for a mismatch (default -3).")
    parser.add_argument("--mismatch_cost", required=False, help="Cost for a mismatch (default 5).")
    parser.add_argument("--gap_open_score", required=False, help="Score for opening a run of gaps (default -4).")
    parser.add_argument("--gap_open_cost", required=False, help="Cost for opening a run of gaps (default 4).")
    parser.add_argument("--gap_extension_score", required=False, help="Score per gap (default -2).")
    parser.add_argument("--gap_extension_cost", required=False, help="Cost per gap (default 3).")
    args = parser.parse_args(argv)
    results = find_global_alignment(**vars(args))
    results.write()
    return None


if __name__ == "__main__":
    sys.exit(main())
