"""Synthetic sequence pairs with the reference's exact random-call sequence.

`draw_random_seq` / `draw_two_random_seqs` mirror globalign's start.py:690-867: same arguments, same
consumption of the process-global CPython ``random`` state (so a given seed yields the same strings),
same exceptions.  The reference edits a Python list in place (``insert``/``pop`` per edit, O(L) each);
here every edit position is drawn first -- the draws depend only on the running length, never on the
contents -- and the edits are then resolved with order-statistic (Fenwick) trees, so a 1M-letter pair
with a few 10^4 edits takes well under a second instead of minutes.  Host code only: the generated
strings go to the aligner like any other input.
"""
import math
import random

__all__ = ["draw_random_seq", "draw_two_random_seqs"]


def draw_random_seq(alphabet, min_len, max_len, seed=None):
    """start.py:690-721: reseed with `seed` (None = OS entropy), draw a length uniformly in
    [min_len, max_len], then that many letters with replacement, joined.

    Raises ValueError (min_len < 0 or min_len > max_len), IndexError (empty alphabet),
    TypeError (alphabet without len(), or non-str letters drawn)."""
    random.seed(seed)
    if min_len < 0:
        print("min_len must be a non-negative integer.")
        raise ValueError
    try:
        length = random.randint(a=min_len, b=max_len)
    except ValueError:
        print("min_len and max_len must be non-negative integers with max_len >= min_len.")
        raise
    try:
        letters = random.choices(population=alphabet, k=length)
    except (IndexError, TypeError):
        print("alphabet must be a non-empty list of strings")
        raise
    return "".join(letters)


class _Slots:
    """Fenwick tree over 0/1 slot flags: k-th set slot and clear, both O(log n)."""

    def __init__(self, n, full=True):
        self.n = n
        t = [0] * (n + 1)
        if full:
            for i in range(1, n + 1):
                t[i] += 1
                j = i + (i & -i)
                if j <= n:
                    t[j] += t[i]
        self.t = t
        self.top = 1 << max(0, n.bit_length() - 1) if n else 0

    def take(self, k):
        """Index (0-based) of the k-th (0-based) set slot; the slot is cleared."""
        t, pos, step, rem = self.t, 0, self.top, k + 1
        while step:
            nxt = pos + step
            if nxt <= self.n and t[nxt] < rem:
                pos = nxt
                rem -= t[nxt]
            step >>= 1
        i = pos + 1
        while i <= self.n:
            t[i] -= 1
            i += i & -i
        return pos


def _edit_index(length, threshold, left, right, mid_hi):
    """One edit position as the reference draws it (start.py:793-805, 821-833, 846-858)."""
    r = random.random()
    if r < threshold / 2:
        return left
    if r < threshold:
        return right
    lo = min(1, length - 1)
    return random.randint(a=lo, b=mid_hi(lo))


def draw_two_random_seqs(alphabet, min_len_seq_1, max_len_seq_1, min_len_seq_2, max_len_seq_2, divergence,
                         seed_1=None, seed_2=None):
    """start.py:724-867.  seq_1 is drawn with `seed_1`; seq_2 starts as a copy and receives, in order,
    max(0, L2-L1) + e insertions, max(0, L1-L2) + e deletions and e substitutions, e =
    ceil(divergence * L2 / 3), with L2 drawn after reseeding with `seed_2`.  Each edit goes to the left
    end, the right end or a uniform middle position; the ends get probability (1-divergence)^(1/count).
    Insertion letters come from a second draw reseeded with `seed_2`; substitution letters from a draw
    reseeded with None (OS entropy, as in the reference -- so seq_2 is reproducible only when there
    are no substitutions, or when the caller controls that reseed)."""
    seq_1 = draw_random_seq(alphabet=alphabet, min_len=min_len_seq_1, max_len=max_len_seq_1, seed=seed_1)
    len_1 = len(seq_1)
    random.seed(seed_2)
    len_2 = random.randint(a=min_len_seq_2, b=max_len_seq_2)
    extra = math.ceil(divergence * len_2 / 3)
    n_ins = max(0, len_2 - len_1) + extra
    n_del = max(0, len_1 - len_2) + extra
    n_sub = extra

    # insertions: positions in a list that grows by one per step (list.insert clamps to [0, len])
    length = len_1
    ins_letters, ins_pos = "", []
    if n_ins > 0:
        ins_letters = draw_random_seq(alphabet=alphabet, min_len=n_ins, max_len=n_ins, seed=seed_2)
        p = (1 - divergence) ** (1 / n_ins)
        for _ in range(n_ins):
            k = _edit_index(length, p, 0, length, lambda lo, L=length: max(1, L - 1))
            if k < 0:
                k += length
            ins_pos.append(min(max(k, 0), length))
            length += 1
    chars = [None] * length
    if n_ins:
        # the last insertion sits at its drawn index of the final list; peel insertions off backwards
        slots = _Slots(length)
        for k in range(n_ins - 1, -1, -1):
            chars[slots.take(ins_pos[k])] = ins_letters[k]
        it = iter(seq_1)
        chars = [c if c is not None else next(it) for c in chars]
    else:
        chars = list(seq_1)

    # deletions: each pops the k-th surviving letter
    if n_del > 0:
        p = (1 - divergence) ** (1 / n_del)
        alive = _Slots(length)
        keep = bytearray(b"\x01") * length
        for _ in range(n_del):
            if length == 0:
                raise IndexError("pop from empty list")
            k = _edit_index(length, p, 0, length - 1, lambda lo, L=length: max(lo, L - 2))
            keep[alive.take(k)] = 0
            length -= 1
        chars = [c for c, f in zip(chars, keep) if f]

    # substitutions: fixed length, applied in order
    if n_sub > 0:
        sub_letters = draw_random_seq(alphabet=alphabet, min_len=n_sub, max_len=n_sub)
        p = (1 - divergence) ** (1 / n_sub)
        for s in range(n_sub):
            k = _edit_index(length, p, 0, length - 1, lambda lo, L=length: max(lo, L - 2))
            chars[k] = sub_letters[s]
    return seq_1, "".join(chars)
