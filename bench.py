#!/usr/bin/env python3
"""Benchmark: DP cells/s of globalign's hot path (fill + traceback) on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload c3|c2|c4] [--no-cpu-baseline]

A step is one pass of the hot path over one synthetic pair already resident
in HBM: boundary + query profile + wavefront fill (with traceback words) +
tie-break table + traceback walk + alignment strings (the whole
find_global_alignment DP, globaligner.py:258-302).  Workloads (BASELINE.json
configs, SURVEY 8d SplitMix64 inputs):
  c3 (default): 100k x 100k DNA, match 2 / mismatch -3 / open -5 / ext -1, full traceback
  c2:           10k x 10k DNA, same scoring
  c4:           1M x 1M DNA, score only
With N > 1 (one process per GPU, torch.distributed over RCCL) the workload is
weak-scaled: the per-GPU cell count is fixed, the matrix grows as a square
(side x sqrt(N)) and is tiled into N column slabs whose left/right edges are
exchanged in row bands with RCCL send/recv (globalign_amd/distributed.py).
"""
import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

METRIC = "DP cells/s (matrix fill) + alignment score bit-exact vs ref"
HBM_PEAK_GBS = 8000.0
BYTES_PER_CELL_TB = 26  # 24 B/cell fill (M, Ix, Iy int32 written + read once) + 2 B traceback word
BYTES_PER_CELL = 24

WORKLOADS = {
    "c2": dict(m=10_000, n=10_000, traceback=True,
               desc="C2: 10k x 10k DNA (SplitMix64 seeds 1,2), match 2 / mismatch -3 / open -5 / ext -1"),
    "c3": dict(m=100_000, n=100_000, traceback=True,
               desc="C3: 100k x 100k DNA (SplitMix64 seeds 1,2), match 2 / mismatch -3 / open -5 / ext -1, "
                    "full traceback"),
    "c4": dict(m=1_000_000, n=1_000_000, traceback=False,
               desc="C4: 1M x 1M DNA (SplitMix64 seeds 1,2), match 2 / mismatch -3 / open -5 / ext -1, score only"),
}
SCORING = dict(match_score=2, mismatch_score=-3, gap_open_score=-5, gap_extension_score=-1)


def splitmix(length, seed, alphabet="dna"):
    """SplitMix64 synthetic sequence; vectorised."""
    with np.errstate(over="ignore"):
        k = np.arange(1, length + 1, dtype=np.uint64)
        z = np.uint64(seed) + k * np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    if alphabet == "dna":
        return np.frombuffer(b"ACGT", dtype=np.uint8)[(z >> np.uint64(62)).astype(np.int64)].tobytes().decode()
    idx = (((z >> np.uint64(32)) * np.uint64(20)) >> np.uint64(32)).astype(np.int64)
    return np.frombuffer(b"ARNDCQEGHILKMFPSTWYV", dtype=np.uint8)[idx].tobytes().decode()


def problem_tables(seq_1, seq_2):
    from globalign_amd import _native
    from globalign_amd.scoring import validate_and_transform_args
    # validation on short prefixes (same alphabet); the API cap does not apply to the engine
    good = validate_and_transform_args(None, None, seq_1[:64], seq_2[:64], **SCORING)
    _, _, smat, cmat, _, goc, _ = good
    return _native.CostTables(cmat, goc), smat


def cpu_baseline(sample=5000):
    """The reference-equivalent pure-Python loop (oracle/pyport.py), 1 core, on a bounded sample."""
    import random
    from oracle import pyport
    s1, s2 = splitmix(sample, 1), splitmix(sample, 2)
    tables, _ = problem_tables(s1, s2)
    C = {x: {y: int(tables.sub[tables.code[x] * tables.K + tables.code[y]]) for y in tables.keys} for x in tables.keys}
    random.seed(0)
    t0 = time.perf_counter()
    T = pyport.fill(s1, s2, C, tables.gap_open, tables.max_cost)
    pyport.traceback(T, s1, s2, C, tables.gap_open)
    dt = time.perf_counter() - t0
    return {"value": sample * sample / dt, "unit": "cells/s", "cores": 1, "kind": "port",
            "sample": f"{sample}x{sample} DNA (SplitMix64 seeds 1,2), fill + traceback, pure-Python port of the "
                      f"reference loop (oracle/pyport.py), {dt:.1f} s"}


def load_traffic(kernel_prefix="fill_kernel"):
    """Measured HBM bytes per fill launch from the committed PMC summary (profiles/), if present."""
    path = os.path.join(ROOT, "profiles", "traffic.json")
    if not os.path.exists(path):
        return None
    try:
        d = json.load(open(path))
        return d.get("fill_kernel_hbm_bytes_per_launch")
    except Exception:
        return None


def run_single(args, wl):
    import random
    from globalign_amd import _native
    m, n = wl["m"], wl["n"]
    s1, s2 = splitmix(m, 1), splitmix(n, 2)
    tables, smat = problem_tables(s1, s2)
    eng = _native.Engine(0)
    eng.load(tables.codes(s1), tables.codes(s2), tables)
    random.seed(0)
    mt0 = np.array(random.getstate()[1], dtype=np.uint32)
    import torch
    fill_ms, walk_ms, rng_ms = [], [], []
    result = None

    def step():
        if wl["traceback"]:
            return eng.align(mt0, s1, s2)
        return eng.fill(traceback=False)

    for _ in range(args.warmup):
        result = step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        result = step()
        tm = eng.timings()
        fill_ms.append(tm["fill_ms"])
        walk_ms.append(tm["walk_ms"])
        rng_ms.append(tm["rng_ms"])
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    cost = result[0]
    if wl["traceback"]:
        _, (a, mid, b), status, _ = result
        assert status == 0 and a.replace("-", "") == s1 and b.replace("-", "") == s2
    return elapsed, cost, fill_ms, walk_ms, rng_ms


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--workload", default="c3", choices=sorted(WORKLOADS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample", type=int, default=5000)
    args = ap.parse_args()
    wl = WORKLOADS[args.workload]
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if args.gpus > 1 or world > 1:
        from globalign_amd import distributed
        return distributed.bench_main(args, wl, WORKLOADS, SCORING)
    elapsed, cost, fill_ms, walk_ms, rng_ms = run_single(args, wl)
    m, n, K = wl["m"], wl["n"], args.steps
    cells = m * n
    value = cells * K / elapsed
    f_avg = float(np.mean(fill_ms))
    bpc = BYTES_PER_CELL_TB if wl["traceback"] else BYTES_PER_CELL
    achieved = bpc * cells / (f_avg * 1e-3) / 1e9
    traffic = load_traffic() if wl is WORKLOADS["c3"] else None
    line = {
        "metric": METRIC,
        "value": value,
        "unit": "cells/s",
        "n_gpus": 1,
        "steps": K,
        "warmup": args.warmup,
        "ms_per_step": elapsed * 1e3 / K,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "int32",
        "data": "synthetic (SplitMix64 DNA, SURVEY 8d)",
        "config": {"workload": wl["desc"], "m": m, "n": n, "traceback": wl["traceback"], "parallelism": "single GPU",
                   "cost": cost},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                     "kernel": "fill_kernel", "bytes_per_cell": bpc, "kernel_ms": f_avg,
                     "measured_hbm_GBps": (traffic / (f_avg * 1e-3) / 1e9) if traffic else None},
        "fill_cells_per_s": cells / (f_avg * 1e-3),
        "walk_ms": float(np.mean(walk_ms)),
        "host_tiebreak_ms": float(np.mean(rng_ms)),
    }
    if not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline(args.cpu_sample)
    print(json.dumps(line))


if __name__ == "__main__":
    main()
