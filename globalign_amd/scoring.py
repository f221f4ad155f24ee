"""Argument validation, scoring/costing matrices and input readers.

Host-side mirror of the reference's settings layer
(iamgiddyaboutgit/globalign src/globalign/start.py), reimplemented so that
the same arguments produce the same matrices and the same exceptions:

  SimpleScoringSettings / SimpleCostingSettings   start.py:10-147
  validate_and_transform_args                     start.py:150-353
  check_seq_lengths                               start.py:361-376
  read_scoring_mat                                start.py:378-428
  create_scoring_mat / create_costing_mat         start.py:431-468
  validate_scoring_mat_keys                       start.py:471-485
  get_max_val                                     start.py:488-497
  scoring_mat_to_costing_mat                      start.py:500-557
  costing_mat_to_scoring_mat                      start.py:559-612
  read_seq_from_fasta / read_first_2_seqs_...     start.py:614-688
  check_symmetric / check_big_main_diag           start.py:883-940
"""
import json
import math
import os
from dataclasses import dataclass
from pathlib import Path

DATA_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "data")
MAX_SEQ_LEN_PROD = 20_000_000  # the reference's API cap (start.py:213); GlobalAligner can lift it


def _as_int(value, default, label):
    v = default if value is None else value
    try:
        return int(v)
    except (TypeError, ValueError):
        print(f"{label} must be convertible to an integer.")
        raise


@dataclass
class SimpleScoringSettings:
    """Scores for the simple (match / mismatch / gap) scheme; defaults 2, -3, -4, -2."""
    match_score: int = 2
    mismatch_score: int = -3
    gap_open_score: int = -4
    gap_extension_score: int = -2

    def __post_init__(self):
        ms = _as_int(self.match_score, 2, "match_score")
        mms = _as_int(self.mismatch_score, -3, "mismatch_score")
        gos = _as_int(self.gap_open_score, -4, "gap_open_score")
        ges = _as_int(self.gap_extension_score, -2, "gap_extension_score")
        if ms <= 0 or mms >= 0 or gos > 0 or ges >= 0:
            raise ValueError
        self.match_score, self.mismatch_score = ms, mms
        self.gap_open_score, self.gap_extension_score = gos, ges


@dataclass
class SimpleCostingSettings:
    """Costs for the simple scheme; defaults 5, 4, 3.

    As in the reference, the sign checks run on the values *before* integer
    conversion, so string arguments raise TypeError there (start.py:138-145)."""
    mismatch_cost: int = 5
    gap_open_cost: int = 4
    gap_extension_cost: int = 3

    def __post_init__(self):
        raw = [self.mismatch_cost if self.mismatch_cost is not None else 5,
               self.gap_open_cost if self.gap_open_cost is not None else 4,
               self.gap_extension_cost if self.gap_extension_cost is not None else 3]
        self.mismatch_cost = _as_int(raw[0], 5, "mismatch_cost")
        self.gap_open_cost = _as_int(raw[1], 4, "gap_open_cost")
        self.gap_extension_cost = _as_int(raw[2], 3, "gap_extension_cost")
        if raw[0] <= 0 or raw[1] < 0 or raw[2] <= 0:
            raise ValueError


def get_max_val(mat):
    """Largest entry of a nested-dict matrix (gap row/column included)."""
    best = -math.inf
    for row in mat.values():
        best = max(best, max(row.values()))
    return best


def _deltas(b):
    return math.floor(b / 2), math.ceil(b / 2)


def scoring_mat_to_costing_mat(scoring_mat, max_score, delta_d=None, delta_i=None):
    """Shift similarity scores to non-negative edit costs.

    Horizontal steps (gap row) get -s + delta_d, vertical steps (gap column)
    -s + delta_i, substitutions -s + delta_d + delta_i, with
    delta_d = floor(b/2), delta_i = ceil(b/2) (curiouscoding.nl score transform)."""
    dd, di = _deltas(max_score)
    dd = dd if delta_d is None else delta_d
    di = di if delta_i is None else delta_i
    out = {}
    for x, row in scoring_mat.items():
        out[x] = {}
        for y, s in row.items():
            if x == "-" and y != "-":
                out[x][y] = dd - s
            elif y == "-" and x != "-":
                out[x][y] = di - s
            else:
                out[x][y] = dd + di - s
    return out


def costing_mat_to_scoring_mat(costing_mat, max_score, delta_d=None, delta_i=None):
    """Inverse of scoring_mat_to_costing_mat for the same b."""
    dd, di = _deltas(max_score)
    dd = dd if delta_d is None else delta_d
    di = di if delta_i is None else delta_i
    out = {}
    for x, row in costing_mat.items():
        out[x] = {}
        for y, c in row.items():
            if x == "-" and y != "-":
                out[x][y] = dd - c
            elif y == "-" and x != "-":
                out[x][y] = di - c
            else:
                out[x][y] = dd + di - c
    return out


def _square(alphabet, diag, gap, off):
    keys = list(alphabet) + ["-"]
    return {x: {y: diag if x == y else (gap if (x == "-" or y == "-") else off) for y in keys} for x in keys}


def create_scoring_mat(common_alphabet, match_score, mismatch_score, gap_extension_score):
    common_alphabet.append("-")
    return _square(common_alphabet[:-1], match_score, gap_extension_score, mismatch_score)


def create_costing_mat(common_alphabet, mismatch_cost, gap_extension_cost):
    common_alphabet.append("-")
    return _square(common_alphabet[:-1], 0, gap_extension_cost, mismatch_cost)


def get_common_alphabet(seq_1, seq_2):
    return sorted(set(seq_1) | set(seq_2))


def check_seq_lengths(seq_1, seq_2, max_seq_len_prod):
    m, n = len(seq_1), len(seq_2)
    prod = m * n
    if max_seq_len_prod is not None and not prod < max_seq_len_prod:
        raise RuntimeError(f"Your sequences are too long.  The product of their lengths should be less than "
                           f"{max_seq_len_prod}.  They have lengths of {m} and {n}")
    if prod == 0:
        raise RuntimeError("Detected a sequence of length 0.")


def validate_scoring_mat_keys(scoring_mat_keys, common_alphabet):
    common_alphabet.append("-")
    missing = set(common_alphabet) - set(scoring_mat_keys)
    if missing:
        raise RuntimeError(f"common_alphabet contains values not in scoring_mat_keys, e.g. {missing}.  "
                           "Please check your sequences and your scoring matrix.")


def check_symmetric(mat):
    try:
        keys = list(mat.keys())
        for x in keys:
            for y in keys:
                try:
                    if mat[x][y] != mat[y][x]:
                        return False
                except KeyError:
                    return False
        return True
    except AttributeError:
        print("The check_symmetric function expected a nested dictionary.")
        raise


def check_big_main_diag(mat):
    ok = None
    for x in mat.keys():
        top = max(mat[x].values())
        try:
            ok = mat[x][x] == top
        except KeyError:
            raise RuntimeError("mat is not a proper nested dict representation of a matrix.")
        if not ok:
            return False
    return ok


def read_scoring_mat(scoring_mat_path):
    """Parse a whitespace-separated scoring matrix whose first line holds the column letters."""
    path = Path(scoring_mat_path)
    if not path.is_file():
        raise FileNotFoundError("scoring_mat_path does not point to a valid file.")
    with path.open() as fh:
        letters = fh.readline().upper().split()
        if any(len(x) != 1 for x in letters):
            raise RuntimeError("The header row did not have single letters spaced apart.")
        mat = dict.fromkeys(letters)
        for row_no, line in enumerate(fh):
            fields = line.split()
            head = fields[0]
            if head != letters[row_no]:
                raise RuntimeError("Row headers do not match column headers.")
            mat[head] = dict.fromkeys(letters)
            for col_no, col in enumerate(letters, start=1):
                mat[head][col.upper()] = int(fields[col_no])
    return mat


def load_named_matrix(name):
    """Packaged matrices (BLOSUM50, BLOSUM62, nucleotide), same values as the reference's data files."""
    path = os.path.join(DATA_DIR, f"{name}.json")
    if not os.path.isfile(path):
        raise FileNotFoundError("scoring_mat_path does not point to a valid file.")
    with open(path) as fh:
        d = json.load(fh)
    letters = list(d["letters"])
    return {x: {y: d["scores"][i][j] for j, y in enumerate(letters)} for i, x in enumerate(letters)}


def read_seq_from_fasta(fasta_path):
    """Yield (description, upper-cased sequence) records."""
    with Path(fasta_path).open() as fh:
        first = fh.readline().strip()
        if not first.startswith(">"):
            raise RuntimeError("Invalid FASTA format. Expected the first line to start with '>'.")
        desc, parts = first, []
        for line in fh:
            line = line.strip()
            if line.startswith(">"):
                seq = "".join(parts).upper()
                if not seq:
                    raise RuntimeError("Empty sequence detected in FASTA.")
                yield desc, seq
                desc, parts = line, []
            elif line:
                parts.append(line)
        seq = "".join(parts).upper()
        if not seq:
            raise RuntimeError("Empty sequence detected in FASTA.")
        yield desc, seq


def read_first_2_seqs_from_fasta(fasta_path):
    """The first two records (start.py:666-688).  Like the reference, a THIRD record is pulled from the
    reader before stopping, so a malformed (empty) third record still raises."""
    seqs = []
    for _, seq in read_seq_from_fasta(fasta_path):
        seqs.append(seq)
        if len(seqs) == 3:
            break
    if len(seqs) < 2:
        raise RuntimeError("Two sequences could not be read from the FASTA file.")
    return seqs[0], seqs[1]


def validate_and_transform_args(input_fasta=None, output=None, seq_1=None, seq_2=None, scoring_mat_name=None,
                                scoring_mat_path=None, match_score=None, mismatch_score=None, mismatch_cost=None,
                                gap_open_score=None, gap_open_cost=None, gap_extension_score=None,
                                gap_extension_cost=None, max_seq_len_prod=MAX_SEQ_LEN_PROD):
    """-> (seq_1, seq_2, scoring_mat, costing_mat, gap_open_score, gap_open_cost, output)"""
    # output (start.py:184-194)
    out_path = None
    if output is not None:
        out_path = Path(output)
        if out_path.is_file():
            raise RuntimeWarning(f"Overwriting {out_path}")
        if not out_path.parent.exists():
            raise FileNotFoundError("The parent directory of output does not exist.")
    # sequences (start.py:201-222)
    if input_fasta is not None and seq_1 is None and seq_2 is None:
        try:
            seq_1, seq_2 = read_first_2_seqs_from_fasta(Path(input_fasta))
        except FileNotFoundError:
            print("input_fasta does not point to a valid file.  Please make sure it is in the correct FASTA format.  "
                  "Note that reading from standard input is not supported at this time.")
            raise
    elif (input_fasta is None and seq_2 is None) or (input_fasta is not None and seq_1 is not None) or \
            (seq_1 is None and seq_2 is not None):
        raise RuntimeError("The combination of arguments for input_fasta, seq_1, and seq_2 does not make sense.")
    check_seq_lengths(seq_1, seq_2, max_seq_len_prod)
    if "-" in seq_1 or "-" in seq_2:
        raise RuntimeError("The current implementation does not allow for '-' characters in the sequences because "
                           "they are used internally for gaps.  Please replace this character in your sequences.")
    s1, s2 = seq_1.upper(), seq_2.upper()
    # option combinations (start.py:227-232)
    others = (match_score, mismatch_score, mismatch_cost, gap_extension_score, gap_extension_cost)
    if scoring_mat_name is not None and any(x is not None for x in (scoring_mat_path,) + others):
        raise RuntimeError("The scoring_mat_name should not be specified if any of the other options with scores or "
                           "costs are specified, except for the gap_open options.")
    if scoring_mat_path is not None and any(x is not None for x in (scoring_mat_name,) + others):
        raise RuntimeError("The scoring_mat_path should not be specified if any of the other options with scores or "
                           "costs are specified, except for the gap_open options.")
    score_opts = (match_score, mismatch_score, gap_open_score, gap_extension_score)
    cost_opts = (mismatch_cost, gap_open_cost, gap_extension_cost)
    if any(x is not None for x in score_opts) and any(x is not None for x in cost_opts):
        raise RuntimeError("Scoring and costing options should not both be set.")
    scores = SimpleScoringSettings(match_score, mismatch_score, gap_open_score, gap_extension_score)
    costs = SimpleCostingSettings(mismatch_cost, gap_open_cost, gap_extension_cost)
    # gap_open score and cost are opposites (start.py:251-262)
    if gap_open_score is not None:
        costs.gap_open_cost = -scores.gap_open_score
    else:
        scores.gap_open_score = -costs.gap_open_cost
    if scoring_mat_name is not None:
        smat = load_named_matrix(scoring_mat_name)
        validate_scoring_mat_keys(smat.keys(), get_common_alphabet(s1, s2))
        cmat = scoring_mat_to_costing_mat(smat, get_max_val(smat))
    elif scoring_mat_path is not None:
        smat = read_scoring_mat(Path(scoring_mat_path))
        if not check_symmetric(smat):
            raise RuntimeError("The scoring matrix is not symmetric.")
        if not check_big_main_diag(smat):
            raise RuntimeError("The scoring matrix does not make sense because the maximum for each row does not "
                               "occur on the main diagonal.")
        validate_scoring_mat_keys(smat.keys(), get_common_alphabet(s1, s2))
        cmat = scoring_mat_to_costing_mat(smat, get_max_val(smat))
    elif any(x is not None for x in cost_opts):
        cmat = create_costing_mat(get_common_alphabet(s1, s2), costs.mismatch_cost, costs.gap_extension_cost)
        smat = costing_mat_to_scoring_mat(cmat, scores.match_score)
    else:
        smat = create_scoring_mat(get_common_alphabet(s1, s2), scores.match_score, scores.mismatch_score,
                                  scores.gap_extension_score)
        cmat = scoring_mat_to_costing_mat(smat, scores.match_score)
    return s1, s2, smat, cmat, scores.gap_open_score, costs.gap_open_cost, out_path


def make_matrix(num_rows, num_cols, fill_val):
    """num_rows independent rows of num_cols copies of fill_val (start.py:869-876)."""
    return [[fill_val] * num_cols for _ in range(num_rows)]


def make_3d_array(dim_1, dim_2, dim_3, fill_val):
    """dim_1 x dim_2 x dim_3 nested lists of fill_val (start.py:878-881)."""
    return [[[fill_val] * dim_3 for _ in range(dim_2)] for _ in range(dim_1)]
