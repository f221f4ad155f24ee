"""bench.py's multi-rank launcher on CPU: ``--gpus N`` without a launcher starts N ranks itself.

The ranks run the real slab orchestration over gloo with the oracle-backed CPU engine
(tests/bench_cpu_engine.py); rank 0 prints ONE JSON line with n_gpus == N and the C1 cost
(2471, BASELINE.md golden results)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, **env):
    e = dict(os.environ, PYTHONPATH=ROOT, **env)
    e.pop("WORLD_SIZE", None)
    e.pop("RANK", None)
    e.pop("LOCAL_RANK", None)
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=e, capture_output=True,
                          text=True, timeout=600)


@pytest.mark.parametrize("n", [2, 3, 8])
def test_bench_spawns_ranks_gloo(n):
    """World sizes up to the driver's 8-GPU node: 8 ranks over gloo (C1's 1000 columns cut into slabs as narrow as
    one column: the orchestration's edge cases)."""
    r = _run(["--gpus", str(n), "--workload", "c1", "--steps", "2", "--warmup", "1"], GA_DIST_BACKEND="gloo",
             GA_BENCH_ENGINE="tests.bench_cpu_engine:make_engine")
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    line = json.loads(lines[0])
    assert line["n_gpus"] == n and line["steps"] == 2 and line["warmup"] == 1
    assert line["config"]["cost"] == 2471 and line["config"]["backend"] == "gloo"
    assert line["value"] > 0 and line["slab_fill_ms_max"] > 0
    assert sum(line["slab_columns"]) == 1000
    # the edge preflight: every boundary's transport in the line (CPU engines relay bands)
    pre = line["config"]["edge_links"]
    assert len(pre["boundaries"]) == n - 1 and not pre["ipc_agreed"]
    assert all(b["transport"].startswith("bands") for b in pre["boundaries"])


def test_bench_refuses_missing_gpus():
    """No silent single-rank run: with the RCCL backend and fewer GPUs than asked, exit non-zero."""
    r = _run(["--gpus", "2", "--workload", "c1"], GA_DIST_BACKEND="nccl", HIP_VISIBLE_DEVICES="")
    assert r.returncode != 0
    assert "needs 2 visible GPUs" in r.stderr


def test_bench_refuses_world_mismatch():
    e = dict(WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--workload", "c1"],
                       env=dict(os.environ, PYTHONPATH=ROOT, **e), capture_output=True, text=True, timeout=300)
    assert r.returncode == 2 and "launcher started 1 ranks" in r.stderr


def test_roofline_profiles_must_match_the_variant_that_ran():
    """bench.roofline divides the committed profile's SQ_INSTS_VALU per launch by the fill's measured time: only when
    the profile (and its VALU mix) are of the kernel variant that ran (columns per lane), else achieved stays null."""
    sys.path.insert(0, ROOT)
    import bench
    assert bench._variant_td("void ga::fill_lane_kernel<4, 2, 0, 16, false, false, true, true>(ga::FillArgs)") == 2
    assert bench._variant_td("_ZN2ga16fill_lane_kernelILi4ELi8ELi0ELi16ELb0ELb0ELb0ELb0EEEvNS_8FillArgsE") == 8
    assert bench._variant_td("fill_kernel") is None
    c3 = bench.WORKLOADS["c3"]
    ok = bench.roofline("c3", c3, 7.6, fill_kind=("rc", 4, 391, 4, 98))
    assert "profile_mismatch" not in ok and 0 < ok["frac"] < 1
    bad = bench.roofline("c3", c3, 6.8, fill_kind=("rc", 2, 782, 4, 196))
    assert bad["achieved"] is None and bad["frac"] is None and "profile_mismatch" in bad
