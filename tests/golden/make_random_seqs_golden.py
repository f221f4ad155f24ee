#!/usr/bin/env python3
"""Golden vectors for draw_two_random_seqs (reference start.py:724-867), made by running the REFERENCE
in the build container (/root/reference is never shipped):

    PYTHONDONTWRITEBYTECODE=1 python3 tests/golden/make_random_seqs_golden.py  ->  tests/golden/random_seqs.json

The reference reseeds with None (OS entropy) before drawing substitution letters (start.py:837-841);
to make those cases reproducible, random.seed(None) is mapped to random.seed(NONE_SEED) while a case
runs -- tests/test_random_seqs.py applies the same mapping to the build.  Long outputs are stored as
sha256 digests plus lengths."""
import hashlib
import json
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
NONE_SEED = 987654321

CASES = [
    # alphabet, min1, max1, min2, max2, divergence, seed_1, seed_2
    (["A", "C", "G", "T"], 3, 10, 6, 15, 0.5, 1, 2),
    (["A", "C", "G", "T"], 20, 20, 20, 20, 0.0, 7, 8),
    (["A", "C", "G", "T"], 50, 80, 10, 30, 0.2, 3, 4),
    (["A", "C", "G", "T"], 10, 30, 50, 90, 0.9, 5, 6),
    (["A", "C", "G", "T"], 0, 0, 0, 5, 0.3, 11, 12),
    (["A", "C", "G", "T"], 0, 0, 0, 0, 0.0, 13, 14),
    (["A", "C", "G", "T"], 1, 1, 1, 2, 1.0, 15, 16),
    (["A", "C", "G", "T"], 4, 4, 0, 0, 0.0, 17, 18),
    (["A", "C", "G", "T"], 4, 4, 0, 1, 1.0, 19, 20),
    (["the", "fat", "cat"], 5, 9, 5, 9, 0.4, 21, 22),
    (list("ARNDCQEGHILKMFPSTWYV"), 200, 400, 200, 400, 0.1, 23, 24),
    (["A", "C", "G", "T"], 2000, 3000, 1500, 3500, 0.05, 25, 26),
    (["A", "C", "G", "T"], 20000, 20000, 20000, 20000, 0.3, 27, 28),
    (["A", "C", "G", "T"], 100000, 100000, 90000, 110000, 0.02, 29, 30),
    (["A", "C"], 5, 3, 1, 2, 0.1, 31, 32),      # ValueError (min_len > max_len)
    ([], 1, 2, 1, 2, 0.1, 33, 34),              # IndexError (empty alphabet)
    ([1, 0], 3, 3, 1, 2, 0.1, 35, 36),          # TypeError (non-str letters)
    (["A", "C"], 3, 3, 4, 2, 0.1, 37, 38),      # ValueError from seq_2's length draw
]


def main():
    sys.path.insert(0, "/root/reference/src")
    from globalign import start  # noqa: E402
    orig = random.seed

    def seed(a=None, version=2):
        return orig(NONE_SEED if a is None else a, version)

    out = []
    random.seed = seed
    try:
        for alph, a1, b1, a2, b2, div, s1, s2 in CASES:
            rec = {"args": [alph, a1, b1, a2, b2, div, s1, s2]}
            try:
                x, y = start.draw_two_random_seqs(alph, a1, b1, a2, b2, div, s1, s2)
            except Exception as e:  # noqa: BLE001 -- the exception type is the expected output
                rec["error"] = type(e).__name__
            else:
                if len(x) + len(y) <= 400:
                    rec["seq_1"], rec["seq_2"] = x, y
                rec["len"] = [len(x), len(y)]
                rec["sha256"] = [hashlib.sha256(x.encode()).hexdigest(), hashlib.sha256(y.encode()).hexdigest()]
            rec["state_after"] = hashlib.sha256(repr(random.getstate()).encode()).hexdigest()
            out.append(rec)
    finally:
        random.seed = orig
    json.dump({"none_seed": NONE_SEED, "cases": out}, open(os.path.join(HERE, "random_seqs.json"), "w"), indent=1)
    print(len(out), "cases;", sum("error" in r for r in out), "raise")


if __name__ == "__main__":
    main()
