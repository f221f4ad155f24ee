"""Alignment result type and the cost -> score conversion.

Mirror of the reference's src/globalign/conclude.py: AlignmentResults
(:7-151, same ten fields, same printout), final_cost_to_score (:154-177),
final_score_to_cost (:179-202) and prettify_mat (:252-310).
"""
import math
from pathlib import Path
from typing import NamedTuple


def final_cost_to_score(cost, m, n, max_score, delta_d=None, delta_i=None):
    """score = n * floor(b/2) + m * ceil(b/2) - cost."""
    dd = math.floor(max_score / 2) if delta_d is None else delta_d
    di = math.ceil(max_score / 2) if delta_i is None else delta_i
    return n * dd + m * di - cost


def final_score_to_cost(score, m, n, max_score, delta_d=None, delta_i=None):
    dd = math.floor(max_score / 2) if delta_d is None else delta_d
    di = math.ceil(max_score / 2) if delta_i is None else delta_i
    return -score + n * dd + m * di


def print_nested_list_aligned(nested_list):
    """Print a list of equal-length rows with every column right-aligned to its widest cell + 1
    (conclude.py:204-249)."""
    widths = [max(len(str(row[j])) for row in nested_list) for j in range(len(nested_list[0]))]
    print("".join("".join(f"{str(c):>{w + 1}}" for c, w in zip(row, widths)) + "\n" for row in nested_list))


def prettify_mat(mat):
    """Right-aligned text table of a nested-dict matrix with row and column headers."""
    try:
        cols = list(list(mat.values())[0].keys())
    except Exception:
        print("mat does not appear to represent a matrix as a nested dictionary.")
        raise
    widths = [max([len(str(c))] + [len(str(mat[r][c])) for r in mat.keys()]) for c in cols]
    head_w = max(len(str(c)) for c in cols)
    parts = [" " * (head_w + 1)]
    parts += [f"{str(c):>{w + 1}}" for c, w in zip(cols, widths)]
    for r in mat.keys():
        parts.append("\n")
        parts.append(f"{str(r):<{head_w + 1}}")
        parts += [f"{str(mat[r][c]):>{w + 1}}" for c, w in zip(cols, widths)]
    return "".join(parts)


class AlignmentResults(NamedTuple):
    seq_1_aligned: str
    middle_part: str
    seq_2_aligned: str
    cost: int
    score: int
    scoring_mat: dict
    costing_mat: dict
    gap_open_score: int
    gap_open_cost: int
    output: Path

    def _generate_alignment_printout(self, desc_1="seq_1", desc_2="seq_2", chars_per_line=70):
        L = len(self.middle_part)
        blocks = math.ceil(L / chars_per_line)
        yield desc_1
        yield "\n"
        yield desc_2
        lo = 0
        hi = L if blocks == 1 else chars_per_line
        for _ in range(blocks):
            yield "\n\n"
            yield self.seq_1_aligned[lo:hi]
            yield "\n"
            yield self.middle_part[lo:hi]
            yield "\n"
            yield self.seq_2_aligned[lo:hi]
            lo, hi = hi, hi + chars_per_line
        yield "\n\n"
        yield f"score: {self.score}\n"
        yield f"cost: {self.cost}\n"
        yield "###########################################\n# Settings\n###########################################\n"
        yield "scoring_mat:\n"
        yield prettify_mat(self.scoring_mat)
        yield f"\n\ngap_open_score: {self.gap_open_score}\n"
        yield "\ncosting_mat:\n"
        yield prettify_mat(self.costing_mat)
        yield f"\n\ngap_open_cost: {self.gap_open_cost}\n"

    def __str__(self, desc_1="seq_1", desc_2="seq_2", chars_per_line=70):
        return "".join(self._generate_alignment_printout(desc_1=desc_1, desc_2=desc_2, chars_per_line=chars_per_line))

    def print(self, desc_1="seq_1", desc_2="seq_2", chars_per_line=70):
        print(self.__str__(desc_1=desc_1, desc_2=desc_2, chars_per_line=chars_per_line))

    def write(self, file=None, desc_1="seq_1", desc_2="seq_2", chars_per_line=70):
        """Write to `file`, else to self.output, else (or file == "stdout") to stdout."""
        if (file is None and self.output is None) or file == "stdout":
            self.print(desc_1=desc_1, desc_2=desc_2, chars_per_line=chars_per_line)
            return None
        target = self.output if file is None else file
        text = self.__str__(desc_1=desc_1, desc_2=desc_2, chars_per_line=chars_per_line)
        with open(file=target, mode="w+") as fh:
            fh.write(text)
        return None

    def cigar(self):
        """Extended CIGAR of the alignment (=: match, X: mismatch, D: gap in seq_2, I: gap in seq_1).

        Not part of the reference; derived from the middle line and the gap characters."""
        ops = []
        for a, mid, b in zip(self.seq_1_aligned, self.middle_part, self.seq_2_aligned):
            ops.append("=" if mid == "|" else "X" if mid == "*" else ("I" if a == "-" else "D"))
        out, k = [], 0
        while k < len(ops):
            q = k
            while q < len(ops) and ops[q] == ops[k]:
                q += 1
            out.append(f"{q - k}{ops[k]}")
            k = q
        return "".join(out)
