"""Input/output side of the path vs reference-run fixtures (tests/golden/io.json, make_io_golden.py).

CPU: the AlignmentResults printout / write() built from the reference's own result fields
(conclude.py:19-151, prettify_mat :252-310), the FASTA reader (start.py:614-688), the CLI's argparse
layer (globaligner.py:23-129), cigar().  GPU: the same cases end to end through the engine."""
import contextlib
import io
import json
import os
import random

import pytest

from tests.conftest import GOLDEN, state_digest

IO = json.load(open(os.path.join(GOLDEN, "io.json")))


def _cases(kind):
    return [r for r in IO if r["case"]["kind"] == kind]


def _result(fields, output=None):
    from globalign_amd.results import AlignmentResults
    return AlignmentResults(output=output, **fields)


# ------------------------------------------------------------------------------------------ CPU
@pytest.mark.parametrize("k", range(len(_cases("printout"))))
def test_printout_matches_reference(k, tmp_path):
    rec = _cases("printout")[k]
    ex, case = rec["expect"], rec["case"]
    out = tmp_path / "out.txt"
    r = _result(ex["fields"], output=out if case.get("output") else None)
    assert str(r) == ex["str"]
    assert r.__str__(desc_1=">first", desc_2=">second", chars_per_line=case.get("cpl", 30)) == ex["str_custom"]
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        r.write()  # to the result's output file when it has one, else stdout
    assert buf.getvalue() == ex["write_stdout"]
    if case.get("output"):
        assert out.read_text() == ex["write_file"]
    other = tmp_path / "other.txt"
    r.write(file=str(other), desc_1="x", desc_2="y", chars_per_line=50)
    assert other.read_text() == ex["write_other"]


@pytest.mark.parametrize("k", range(len(_cases("fasta"))))
def test_fasta_reader_matches_reference(k, tmp_path):
    from globalign_amd.scoring import read_first_2_seqs_from_fasta
    rec = _cases("fasta")[k]
    ex = rec["expect"]
    path = tmp_path / "in.fa"
    path.write_text(rec["case"]["text"])
    if "error" in ex:
        with pytest.raises(Exception) as ei:
            read_first_2_seqs_from_fasta(path)
        assert type(ei.value).__name__ == ex["error"] and str(ei.value) == ex["message"]
    else:
        assert list(read_first_2_seqs_from_fasta(path)) == ex["seqs"]


def test_cli_rejects_unknown_matrix_name(capsys):
    """argparse `choices` (globaligner.py:65-70): exit status 2 before any alignment."""
    from globalign_amd.globaligner import main
    rec = [r for r in _cases("cli") if "BLOSUM45" in r["case"]["argv"]][0]
    with pytest.raises(SystemExit) as ei:
        main(rec["case"]["argv"])
    assert ei.value.code == rec["expect"]["exit"] == 2
    err = capsys.readouterr().err
    assert "invalid choice: 'BLOSUM45'" in err and rec["expect"]["stderr_has"]


def test_cli_version(capsys):
    """--version prints version('globalign') (globaligner.py:31-36): the installed globalign's, else ours."""
    from importlib.metadata import PackageNotFoundError, version

    from globalign_amd import __version__
    from globalign_amd.globaligner import main
    with pytest.raises(SystemExit) as ei:
        main(["--version"])
    assert ei.value.code == 0
    try:
        want = version("globalign")
    except PackageNotFoundError:
        want = __version__
    assert capsys.readouterr().out.strip() == want


def test_cigar_matches_columns():
    """cigar() (no reference counterpart): run-length of =/X/I/D over the printout columns of every fixture."""
    for rec in _cases("printout"):
        f = rec["expect"]["fields"]
        r = _result(f)
        ops = []
        for a, mid, b in zip(f["seq_1_aligned"], f["middle_part"], f["seq_2_aligned"]):
            ops.append("=" if mid == "|" else "X" if mid == "*" else "I" if a == "-" else "D")
        expanded = []
        num = ""
        for ch in r.cigar():
            if ch.isdigit():
                num += ch
            else:
                expanded += [ch] * int(num)
                num = ""
        assert expanded == ops and num == ""
        # adjacent runs differ (maximal runs)
        letters = [ch for ch in r.cigar() if not ch.isdigit()]
        assert all(x != y for x, y in zip(letters, letters[1:]))


# ------------------------------------------------------------------------------------------ GPU
@pytest.mark.gpu
@pytest.mark.parametrize("k", range(len(_cases("printout"))))
def test_printout_end_to_end(k, tmp_path, monkeypatch):
    import globalign_amd
    rec = _cases("printout")[k]
    case, ex = rec["case"], rec["expect"]
    monkeypatch.chdir(tmp_path)
    kw = dict(case["kwargs"])
    if case.get("output"):
        kw["output"] = "out.txt"
    random.seed(case["seed"])
    r = globalign_amd.find_global_alignment(**kw)
    assert str(r) == ex["str"]
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        r.write()
    assert buf.getvalue() == ex["write_stdout"]
    if case.get("output"):
        assert (tmp_path / "out.txt").read_text() == ex["write_file"]
    assert state_digest() == ex["state_after"]


@pytest.mark.gpu
@pytest.mark.parametrize("k", range(len(_cases("cli"))))
def test_cli_end_to_end(k, tmp_path, monkeypatch):
    from globalign_amd.globaligner import main
    rec = _cases("cli")[k]
    case, ex = rec["case"], rec["expect"]
    monkeypatch.chdir(tmp_path)
    for name, text in case.get("files", {}).items():
        (tmp_path / name).write_text(text)
    monkeypatch.setattr("sys.argv", ["globaligner"] + case["argv"])
    random.seed(case["seed"])
    buf, ebuf = io.StringIO(), io.StringIO()
    got = {}
    try:
        with contextlib.redirect_stdout(buf), contextlib.redirect_stderr(ebuf):
            main()
        got["exit"] = 0
    except SystemExit as e:
        got["exit"] = e.code
    except Exception as e:
        got["error"], got["message"] = type(e).__name__, str(e)
    for key in ("exit", "error", "message"):
        assert got.get(key) == ex.get(key), (key, got, ex)
    assert buf.getvalue() == ex["stdout"]
    if "outfile_text" in ex:
        assert (tmp_path / case["outfile"]).read_text() == ex["outfile_text"]
    assert state_digest() == ex["state_after"]


@pytest.mark.gpu
@pytest.mark.parametrize("k", range(len(_cases("fasta"))))
def test_fasta_end_to_end(k, tmp_path, monkeypatch):
    import globalign_amd
    rec = _cases("fasta")[k]
    case, ex = rec["case"], rec["expect"]
    monkeypatch.chdir(tmp_path)
    (tmp_path / "in.fa").write_text(case["text"])
    random.seed(case["seed"])
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        try:
            r = globalign_amd.find_global_alignment(input_fasta="in.fa", **case.get("kwargs", {}))
            got = [r.seq_1_aligned, r.middle_part, r.seq_2_aligned, r.cost, r.score]
            assert got == ex["aligned"]
        except AssertionError:
            raise
        except Exception as e:
            assert {"error": type(e).__name__, "message": str(e)} == ex["api"]
    assert buf.getvalue() == ex["printed"]


@pytest.mark.gpu
@pytest.mark.parametrize("k", range(len(_cases("backward"))))
def test_dp_array_backward_walks_callers_cells(k):
    """dp_array_backward on dp_arrays edited after the fill: the walk follows the caller's cells."""
    import globalign_amd
    rec = _cases("backward")[k]
    case, ex = rec["case"], rec["expect"]
    dp = [[tuple(c) for c in row] for row in ex["dp"]]
    random.seed(case["seed"])
    if "error" in ex:
        with pytest.raises(Exception) as ei:
            globalign_amd.dp_array_backward(dp, case["seq_1"], case["seq_2"], case["costing_mat"],
                                            case["gap_open_cost"])
        assert type(ei.value).__name__ == ex["error"]
    else:
        got = globalign_amd.dp_array_backward(dp, case["seq_1"], case["seq_2"], case["costing_mat"],
                                              case["gap_open_cost"])
        assert list(got) == ex["result"]
    assert state_digest() == ex["state_after"]
