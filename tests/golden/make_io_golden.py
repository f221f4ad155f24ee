"""Reference-run fixtures for the input/output side of the path:

    python tests/golden/make_io_golden.py      ->  tests/golden/io.json

* printout: str(AlignmentResults) with default and custom descriptions / line widths, and the text
  write() puts in a file (conclude.py:19-151, prettify_mat :252-310);
* cli: stdout / output file / exception of the `globaligner` console script (globaligner.py:23-129);
* fasta: read_first_2_seqs_from_fasta on hand-made files (start.py:614-688), incl. an empty THIRD record;
* backward: dp_array_backward on dp_arrays whose cells were edited after the fill (globaligner.py:395-593
  walks the caller's cells).

Each case runs in a child interpreter that imports ONLY the reference (PYTHONPATH=/root/reference/src,
cwd a temp dir, no bytecode written); this script keeps inputs and outputs as data.  Test infrastructure.
"""
import json
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
REF = "/root/reference/src"

CHILD = r'''
import contextlib, hashlib, io, json, os, random, sys
from pathlib import Path
from globalign import globaligner, start
from globalign.globaligner import find_global_alignment, dp_array_backward, dp_array_forward, make_dp_array

def digest():
    return hashlib.sha256(",".join(str(w) for w in random.getstate()[1]).encode()).hexdigest()[:32]

def res_fields(r):
    return dict(seq_1_aligned=r.seq_1_aligned, middle_part=r.middle_part, seq_2_aligned=r.seq_2_aligned, cost=r.cost,
                score=r.score, scoring_mat=r.scoring_mat, costing_mat=r.costing_mat, gap_open_score=r.gap_open_score,
                gap_open_cost=r.gap_open_cost)

def err(e):
    return {"error": type(e).__name__, "message": str(e)}

case = json.loads(sys.stdin.read())
kind = case["kind"]
out = {}
if kind == "printout":
    random.seed(case["seed"])
    kw = dict(case["kwargs"])
    if case.get("output"):
        kw["output"] = "out.txt"
    r = find_global_alignment(**kw)
    out["fields"] = res_fields(r)
    out["str"] = str(r)
    out["str_custom"] = r.__str__(desc_1=">first", desc_2=">second", chars_per_line=case.get("cpl", 30))
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        r.write()
    out["write_stdout"] = buf.getvalue()
    if case.get("output"):
        out["write_file"] = Path("out.txt").read_text()
    r.write(file="other.txt", desc_1="x", desc_2="y", chars_per_line=50)
    out["write_other"] = Path("other.txt").read_text()
    out["state_after"] = digest()
elif kind == "cli":
    # the reference is not pip-installed here, so importlib.metadata has no 'globalign' version for
    # main()'s --version argument (globaligner.py:31-36); the harness supplies one
    globaligner.version = lambda name: "0.0.0+reference"
    for name, text in case.get("files", {}).items():
        Path(name).write_text(text)
    random.seed(case["seed"])
    sys.argv = ["globaligner"] + case["argv"]
    buf, ebuf = io.StringIO(), io.StringIO()
    try:
        with contextlib.redirect_stdout(buf), contextlib.redirect_stderr(ebuf):
            globaligner.main()
        out["exit"] = 0
    except SystemExit as e:
        out["exit"] = e.code
    except Exception as e:
        out.update(err(e))
    out["stdout"] = buf.getvalue()
    out["stderr_has"] = [s for s in case.get("stderr_probe", []) if s in ebuf.getvalue()]
    if case.get("outfile") and Path(case["outfile"]).exists():
        out["outfile_text"] = Path(case["outfile"]).read_text()
    out["state_after"] = digest()
elif kind == "fasta":
    Path("in.fa").write_text(case["text"])
    try:
        out["seqs"] = list(start.read_first_2_seqs_from_fasta(Path("in.fa")))
    except Exception as e:
        out.update(err(e))
    random.seed(case["seed"])
    buf = io.StringIO()
    try:
        with contextlib.redirect_stdout(buf):
            r = find_global_alignment(input_fasta="in.fa", **case.get("kwargs", {}))
        out["aligned"] = [r.seq_1_aligned, r.middle_part, r.seq_2_aligned, r.cost, r.score]
    except Exception as e:
        out["api"] = err(e)
    out["printed"] = buf.getvalue()
elif kind == "backward":
    C = case["costing_mat"]
    s1, s2, o = case["seq_1"], case["seq_2"], case["gap_open_cost"]
    mc = max(max(r.values()) for r in C.values())
    dp = make_dp_array(seq_1=s1, seq_2=s2, costing_mat=C, max_cost=mc, gap_open_cost=o)
    dp_array_forward(dp_array=dp, seq_1=s1, seq_2=s2, costing_mat=C, gap_open_cost=o)
    for i, j, v in case["edits"]:
        dp[i][j] = tuple(v)
    out["dp"] = [[list(c) for c in row] for row in dp]
    random.seed(case["seed"])
    try:
        out["result"] = list(dp_array_backward(dp_array=dp, seq_1=s1, seq_2=s2, costing_mat=C, gap_open_cost=o))
    except Exception as e:
        out.update(err(e))
    out["state_after"] = digest()
print(json.dumps(out))
'''

DNA = dict(match_score=2, mismatch_score=-3, gap_open_score=-5, gap_extension_score=-1)


def splitmix(length, seed, alphabet="ACGT"):
    M = (1 << 64) - 1
    st, out = seed, []
    for _ in range(length):
        st = (st + 0x9E3779B97F4A7C15) & M
        z = st
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M
        z ^= z >> 31
        out.append(alphabet[z >> 62] if len(alphabet) == 4 else alphabet[((z >> 32) * len(alphabet)) >> 32])
    return "".join(out)


PROT = "ARNDCQEGHILKMFPSTWYV"
MTX = "A C G T -\nA 5 -4 -4 -4 -2\nC -4 5 -4 -4 -2\nG -4 -4 5 -4 -2\nT -4 -4 -4 5 -2\n- -2 -2 -2 -2 -2\n"


def cases():
    pr = [
        dict(seed=1, kwargs=dict(seq_1="GATTACA", seq_2="GCATGCU")),
        dict(seed=2, kwargs=dict(seq_1=splitmix(150, 1), seq_2=splitmix(140, 2), **DNA), output=True),
        dict(seed=3, kwargs=dict(seq_1=splitmix(70, 3), seq_2=splitmix(70, 4), **DNA), cpl=70),
        dict(seed=4, kwargs=dict(seq_1="acgtacgtta", seq_2="ACGGTTA", mismatch_cost=6, gap_open_cost=3,
                                 gap_extension_cost=2)),
        dict(seed=5, kwargs=dict(seq_1=splitmix(90, 5, PROT), seq_2=splitmix(85, 6, PROT), scoring_mat_name="BLOSUM62")),
        dict(seed=6, kwargs=dict(seq_1=splitmix(40, 7, PROT), seq_2=splitmix(52, 8, PROT), scoring_mat_name="BLOSUM50",
                                 gap_open_score=-10)),
        dict(seed=7, kwargs=dict(seq_1="TTAGGC", seq_2="TAGC", match_score=3, mismatch_score=-4, gap_open_score=0,
                                 gap_extension_score=-2)),
        dict(seed=8, kwargs=dict(seq_1=splitmix(213, 9), seq_2=splitmix(71, 10), **DNA), cpl=7),
    ]
    for c in pr:
        yield dict(kind="printout", **c)
    fa2 = ">one desc\nacgtac\nGTTA\n\n>two\nACG\nTTAGC\n"
    cli = [
        dict(argv=["--seq_1", "GATTACA", "--seq_2", "GCATGCU"]),
        dict(argv=["--seq_1", splitmix(120, 11), "--seq_2", splitmix(100, 12), "--match_score", "2",
                   "--mismatch_score", "-3", "--gap_open_score", "-5", "--gap_extension_score", "-1"]),
        dict(argv=["--seq_1", splitmix(60, 13, PROT), "--seq_2", splitmix(66, 14, PROT), "--scoring_mat_name",
                   "BLOSUM62", "--gap_open_score", "-11"]),
        dict(argv=["-i", "pair.fa"], files={"pair.fa": fa2}),
        dict(argv=["-i", "pair.fa", "-o", "aln.txt"], files={"pair.fa": fa2}, outfile="aln.txt"),
        dict(argv=["--seq_1", "ACGT", "--seq_2", "AGT", "--scoring_mat_path", "m.mtx"], files={"m.mtx": MTX}),
        dict(argv=["--seq_1", "ACGT", "--seq_2", "AGT", "--mismatch_cost", "5"]),  # str costs: TypeError
        dict(argv=["--seq_1", "ACGT", "--seq_2", "AGT", "--scoring_mat_name", "BLOSUM45"],
             stderr_probe=["invalid choice: 'BLOSUM45'", "choose from 'BLOSUM50', 'BLOSUM62'",
                           "choose from BLOSUM50, BLOSUM62"]),
        dict(argv=["--seq_1", "ACGT", "--seq_2", "AG-T"]),
        dict(argv=["--seq_2", "ACGT"]),
    ]
    for k, c in enumerate(cli):
        yield dict(kind="cli", seed=100 + k, **c)
    fasta = [
        ">a\nACGT\n>b\nAGT\n",
        ">a\nacgt\nacg\n>b\n\nAGT\nT\n>c\nGGG\n",
        ">a\nACGT\n>b\nAGT\n>c\n",                 # empty third record
        ">a\nACGT\n>b\nAGT\n>c\n\n>d\nAC\n",       # empty third record, a fourth follows
        ">a\nACGT\n>b\n>c\nGG\n",                  # empty second record
        ">a\nACGT\n",                              # one record
        "ACGT\n>b\nAGT\n",                         # no header first
        "\n>a\nACGT\n>b\nAGT\n",                   # blank first line
        ">a\n  ACGT  \n>b\nAG T\n",                # inner blanks kept
        ">a\nACGT\n>b\nAGT\n>c\nTT\n>d\n",         # empty FOURTH record: never read
    ]
    for k, text in enumerate(fasta):
        yield dict(kind="fasta", seed=200 + k, text=text, kwargs=DNA)
    cm_dna = {"A": {"A": 0, "C": 5, "G": 5, "T": 5, "-": 2}, "C": {"A": 5, "C": 0, "G": 5, "T": 5, "-": 2},
              "G": {"A": 5, "C": 5, "G": 0, "T": 5, "-": 2}, "T": {"A": 5, "C": 5, "G": 5, "T": 0, "-": 2},
              "-": {"A": 2, "C": 2, "G": 2, "T": 2, "-": 2}}
    bw = [
        dict(seq_1="GATTACAGG", seq_2="GCATGCAT", edits=[]),
        dict(seq_1="GATTACAGG", seq_2="GCATGCAT", edits=[[9, 8, [1, 1, 1]]]),            # tie at the start
        dict(seq_1="GATTACAGG", seq_2="GCATGCAT", edits=[[8, 7, [0, 50, 50]], [5, 5, [3, 3, 9]]]),
        dict(seq_1="ACGTACGTAC", seq_2="ACGTTGCA", edits=[[k, k, [-5, 40, 40]] for k in range(1, 9)]),
        dict(seq_1="TTTTGGGG", seq_2="GGGGTTTT", edits=[[i, j, [7, 7, 7]] for i in range(1, 9) for j in range(1, 9)
                                                        if (i + j) % 3 == 0]),
        dict(seq_1=splitmix(12, 21), seq_2=splitmix(11, 22), edits=[[6, 6, [100, -2, 100]], [6, 5, [-3, 100, 100]]]),
    ]
    for k, c in enumerate(bw):
        yield dict(kind="backward", seed=300 + k, costing_mat=cm_dna, gap_open_cost=5, **c)


def run_case(case):
    env = {"PYTHONPATH": REF, "PYTHONDONTWRITEBYTECODE": "1", "PATH": os.environ.get("PATH", "/usr/bin"),
           "HOME": os.environ.get("HOME", "/tmp")}
    with tempfile.TemporaryDirectory() as d:
        p = subprocess.run([sys.executable, "-c", CHILD], input=json.dumps(case), capture_output=True, text=True,
                           cwd=d, env=env, timeout=300)
    if p.returncode != 0:
        raise RuntimeError(p.stderr[-2000:])
    return json.loads(p.stdout.strip().splitlines()[-1])


if __name__ == "__main__":
    out = []
    for case in cases():
        out.append(dict(case=case, expect=run_case(case)))
        print(case["kind"], {k: v for k, v in out[-1]["expect"].items() if k in ("error", "exit", "message")})
    json.dump(out, open(os.path.join(ROOT, "tests", "golden", "io.json"), "w"), indent=0)
