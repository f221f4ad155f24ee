#!/usr/bin/env python3
"""Benchmark: DP cells/s of globalign's hot path on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload c4|c3|c5|c2] [--no-cpu-baseline]
                    [--no-headline]

Workloads (BASELINE.json configs, SURVEY 8d SplitMix64 inputs, resident in HBM):
  c4 (default): 1M x 1M DNA, match 2 / mismatch -3 / open -5 / ext -1, score only.  BASELINE's
                1/2/4/8-GPU scaling config: the SAME pair for every N (strong scaling), cut into
                N column slabs whose edges stream between GPUs in row bands over RCCL
                (globalign_amd/distributed.py).  A step = boundary + fill + score.
  c3:           100k x 100k DNA, same scoring, full traceback: a step is the whole
                find_global_alignment DP (fill + tie-break table + walk + strings,
                globaligner.py:258-302).  At N=1 the default run also measures this headline
                config and reports it as "headline_c3".
  c4tb:         C4 with full traceback on one GPU: 10^12 traceback bytes do not fit in HBM, so the
                traceback runs in row bands (a checkpointing score pass, then band refills + walk).
  c5:           20k x 20k protein (seeds 3, 4), BLOSUM62, gap_open_score -10, full traceback.
  c2:           10k x 10k DNA, full traceback.
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
SCORING = dict(match_score=2, mismatch_score=-3, gap_open_score=-5, gap_extension_score=-1)
PROTEIN_SCORING = dict(scoring_mat_name="BLOSUM62", gap_open_score=-10)

WORKLOADS = {
    "c2": dict(m=10_000, n=10_000, traceback=True, alphabet="dna", seeds=(1, 2), scoring=SCORING,
               desc="C2: 10k x 10k DNA (SplitMix64 seeds 1,2), match 2 / mismatch -3 / open -5 / ext -1, full traceback"),
    "c3": dict(m=100_000, n=100_000, traceback=True, alphabet="dna", seeds=(1, 2), scoring=SCORING,
               desc="C3: 100k x 100k DNA (SplitMix64 seeds 1,2), match 2 / mismatch -3 / open -5 / ext -1, "
                    "full traceback"),
    "c4": dict(m=1_000_000, n=1_000_000, traceback=False, alphabet="dna", seeds=(1, 2), scoring=SCORING,
               desc="C4: 1M x 1M DNA (SplitMix64 seeds 1,2), match 2 / mismatch -3 / open -5 / ext -1, score only"),
    "c4tb": dict(m=1_000_000, n=1_000_000, traceback=True, alphabet="dna", seeds=(1, 2), scoring=SCORING, golden="c4",
                 desc="C4 with full traceback: 1M x 1M DNA (SplitMix64 seeds 1,2), match 2 / mismatch -3 / open -5 / "
                      "ext -1; banded traceback (checkpointed score pass + band refills, DESIGN.md 5.5)"),
    "c5": dict(m=20_000, n=20_000, traceback=True, alphabet="protein", seeds=(3, 4), scoring=PROTEIN_SCORING,
               desc="C5: 20k x 20k protein (SplitMix64 seeds 3,4), BLOSUM62, gap_open_score -10, full traceback"),
}
DEFAULT_WORKLOAD = "c4"


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


def problem_tables(seq_1, seq_2, scoring=None):
    from globalign_amd import _native
    from globalign_amd.scoring import validate_and_transform_args
    # validation on short prefixes (same alphabet); the API cap does not apply to the engine
    good = validate_and_transform_args(None, None, seq_1[:64], seq_2[:64], **(scoring or SCORING))
    _, _, smat, cmat, _, goc, _ = good
    return _native.CostTables(cmat, goc), smat


def cpu_baseline(sample=5000, traceback=False):
    """The reference-equivalent pure-Python loop (oracle/pyport.py), 1 core, on a bounded sample of the
    workload's kind (DNA, same scoring; fill only for score-only workloads, fill + traceback otherwise)."""
    import random
    from oracle import pyport
    s1, s2 = splitmix(sample, 1), splitmix(sample, 2)
    tables, _ = problem_tables(s1, s2)
    C = {x: {y: int(tables.sub[tables.code[x] * tables.K + tables.code[y]]) for y in tables.keys} for x in tables.keys}
    random.seed(0)
    t0 = time.perf_counter()
    T = pyport.fill(s1, s2, C, tables.gap_open, tables.max_cost)
    if traceback:
        pyport.traceback(T, s1, s2, C, tables.gap_open)
    dt = time.perf_counter() - t0
    what = "fill + traceback" if traceback else "fill + score (dp_array_forward, min of the last cell)"
    return {"value": sample * sample / dt, "unit": "cells/s", "cores": 1, "kind": "port",
            "sample": f"{sample}x{sample} DNA (SplitMix64 seeds 1,2), {what}, pure-Python port of the "
                      f"reference loop (oracle/pyport.py), {dt:.1f} s"}


def load_traffic(name="traffic.json"):
    """Measured HBM bytes per fill launch from a committed PMC summary (profiles/), if present."""
    path = os.path.join(ROOT, "profiles", name)
    if not os.path.exists(path):
        return None
    try:
        return json.load(open(path)).get("fill_kernel_hbm_bytes_per_launch")
    except Exception:
        return None


def golden_cost(workload):
    """The oracle-pinned cost of a workload (tests/golden/<workload>_cost.json), if committed."""
    path = os.path.join(ROOT, "tests", "golden", f"{workload}_cost.json")
    if not os.path.exists(path):
        return None
    return json.load(open(path)).get("cost")


def workload_pair(wl):
    return splitmix(wl["m"], wl["seeds"][0], wl["alphabet"]), splitmix(wl["n"], wl["seeds"][1], wl["alphabet"])


def measure_single(wl, steps, warmup):
    """Time `steps` passes of the hot path over one resident pair on cuda:0."""
    import random
    import torch
    from globalign_amd import _native
    s1, s2 = workload_pair(wl)
    tables, _ = problem_tables(s1, s2, wl["scoring"])
    eng = _native.Engine(0)
    eng.load(tables.codes(s1), tables.codes(s2), tables)
    random.seed(0)
    mt0 = np.array(random.getstate()[1], dtype=np.uint32)
    fill_ms, walk_ms, rng_ms = [], [], []
    result = None

    def step():
        if wl["traceback"]:
            return eng.align(mt0, s1, s2)
        return eng.fill(traceback=False)

    for _ in range(warmup):
        result = step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        result = step()
        tm = eng.timings()
        fill_ms.append(tm["fill_ms"])
        walk_ms.append(tm["walk_ms"] if wl["traceback"] else 0.0)
        rng_ms.append(tm["rng_ms"] if wl["traceback"] else 0.0)
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    cost = result[0]
    if wl["traceback"]:
        _, (a, mid, b), status, _ = result
        assert status == 0 and a.replace("-", "") == s1 and b.replace("-", "") == s2
    cells = wl["m"] * wl["n"]
    f_avg = float(np.mean(fill_ms))
    return dict(elapsed=elapsed, cost=int(cost), cells=cells, value=cells * steps / elapsed,
                ms_per_step=elapsed * 1e3 / steps, fill_ms=f_avg, walk_ms=float(np.mean(walk_ms)),
                rng_ms=float(np.mean(rng_ms)))


# VALU issue peak of MI355X: 256 CUs x 4 SIMDs x 2.4 GHz, one wave64 instruction per 4 cycles per SIMD at the
# single rate of v_min_i32 / DPP / VOP3 (tools/micro/valu_rate.hip; adds and logic ops dual-issue at 2 per 4)
VALU_PEAK_INSTS = 256 * 4 * 2.4e9 / 4


def load_valu(name):
    """Measured fill-kernel wave-instructions per launch from a committed SQ counter summary (profiles/)."""
    path = os.path.join(ROOT, "profiles", name)
    if not os.path.exists(path):
        return None
    try:
        return json.load(open(path)).get("sq_insts_valu_per_launch")
    except Exception:
        return None


def roofline(wl, fill_ms, traffic, valu_insts=None):
    """The HBM roofline of SURVEY 8(d) (algorithmic bytes per cell) plus what actually bounds the kernel:
    it moves ~1 B/cell or less (traffic, PMC) and is VALU-issue bound, so the VALU issue rate is reported
    against the single-rate wave-instruction peak beside it."""
    bpc = BYTES_PER_CELL_TB if wl["traceback"] else BYTES_PER_CELL
    cells = wl["m"] * wl["n"]
    achieved = bpc * cells / (fill_ms * 1e-3) / 1e9
    out = {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
           "traffic": traffic, "kernel": "fill_kernel", "bytes_per_cell": bpc,
           "units_per_launch": f"{cells} cells (m*n)", "kernel_ms": fill_ms,
           "measured_hbm_GBps": (traffic / (fill_ms * 1e-3) / 1e9) if traffic else None}
    if valu_insts:
        rate = valu_insts / (fill_ms * 1e-3)
        out["valu"] = {"insts_per_launch": valu_insts, "insts_per_cell": valu_insts / cells,
                       "issue_rate": rate, "peak_single_rate": VALU_PEAK_INSTS, "frac": rate / VALU_PEAK_INSTS,
                       "unit": "wave64 instructions/s", "source": "SQ_INSTS_VALU (profiles/valu_<workload>.json)"}
    return out


TRAFFIC_FILES = {"c3": "traffic.json", "c4": "traffic_c4.json"}
VALU_FILES = {"c3": "valu_c3.json", "c4": "valu_c4.json"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--workload", default=DEFAULT_WORKLOAD, choices=sorted(WORKLOADS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-headline", action="store_true", help="skip the C3 headline measurement at N=1")
    ap.add_argument("--cpu-sample", type=int, default=5000)
    args = ap.parse_args()
    wl = WORKLOADS[args.workload]
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if args.gpus > 1 or world > 1:
        from globalign_amd import distributed
        return distributed.bench_main(args, wl, args.workload)
    r = measure_single(wl, args.steps, args.warmup)
    gold = golden_cost(wl.get("golden", args.workload))
    line = {
        "metric": METRIC,
        "value": r["value"],
        "unit": "cells/s",
        "n_gpus": 1,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": r["ms_per_step"],
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "int32",
        "data": "synthetic (SplitMix64, SURVEY 8d)",
        "config": {"workload": wl["desc"], "m": wl["m"], "n": wl["n"], "traceback": wl["traceback"],
                   "parallelism": "single GPU", "cost": r["cost"], "oracle_cost": gold,
                   "cost_matches_oracle": (r["cost"] == gold) if gold is not None else None},
        "roofline": roofline(wl, r["fill_ms"], load_traffic(TRAFFIC_FILES.get(args.workload, "none.json")),
                             load_valu(VALU_FILES.get(args.workload, "none.json"))),
        "fill_cells_per_s": r["cells"] / (r["fill_ms"] * 1e-3),
    }
    if wl["traceback"]:
        line["walk_ms"] = r["walk_ms"]
        line["host_tiebreak_ms"] = r["rng_ms"]
    if args.workload == DEFAULT_WORKLOAD and not args.no_headline:
        # the north-star 1-GPU config: 100k x 100k with full traceback (BASELINE configs[2])
        w3 = WORKLOADS["c3"]
        h = measure_single(w3, max(3, min(args.steps, 5)), 1)
        line["headline_c3"] = {"workload": w3["desc"], "value": h["value"], "unit": "cells/s",
                               "ms_per_step": h["ms_per_step"], "cost": h["cost"], "fill_ms": h["fill_ms"],
                               "walk_ms": h["walk_ms"], "host_tiebreak_ms": h["rng_ms"],
                               "roofline": roofline(w3, h["fill_ms"], load_traffic("traffic.json"),
                                                    load_valu("valu_c3.json"))}
    if not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline(args.cpu_sample, traceback=wl["traceback"])
    print(json.dumps(line))


if __name__ == "__main__":
    main()
