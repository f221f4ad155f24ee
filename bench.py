#!/usr/bin/env python3
"""Benchmark: DP cells/s of globalign's hot path on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload c3|c4|c4tb|c5|c2|c1]
                    [--no-cpu-baseline] [--no-extra]

Workloads (BASELINE.json configs, SURVEY 8d SplitMix64 inputs, resident in HBM):
  c3 (default at N=1): 100k x 100k DNA, match 2 / mismatch -3 / open -5 / ext -1, full traceback --
                the config BASELINE's roofline target is quoted on.  A step is ONE whole
                find_global_alignment DP call (fill + tie-break table + walk + strings,
                globaligner.py:258-302), steps run one after another with nothing overlapped; the
                repeated-pair pipeline is reported beside it as an extra key.  The N=1 line also carries "c4": one GPU's point of
                the C4 scaling curve.
  c4 (default at N>1): 1M x 1M DNA, same scoring, score only.  BASELINE's 1/2/4/8-GPU scaling
                config: the SAME pair for every N (strong scaling), cut into N column slabs, each fill
                storing its right edge into the next GPU's memory over xGMI (RCCL row bands as the
                fallback; globalign_amd/distributed.py).
  c4tb:         C4 with full traceback on one GPU (10^12 traceback bytes do not fit in HBM: the recompute
                walk, a checkpointing score fill, then blocks recomputed beside the walk).
  c5:           20k x 20k protein (seeds 3, 4), BLOSUM62, gap_open_score -10, full traceback.
  c2:           10k x 10k DNA, full traceback.
  c1:           1k x 1k DNA (BASELINE configs[0], the reference's CPU-runnable case).
  c4r:          1M x 16k DNA score only: a multi-rank rehearsal shape for ranks sharing one GPU.

--gpus N > 1 without a torch.distributed launcher environment starts N rank processes itself
(torch.distributed.run, 127.0.0.1) and exits with their status; it fails if fewer than N GPUs
are visible (GA_DIST_BACKEND=gloo rehearses the ranks without that check).
"""
import argparse
import json
import os
import re
import socket
import subprocess
import sys
import time

# The repeated-alignment pipeline runs four fill streams beside the walk stream, all at the greatest
# priority, whose pool holds GPU_MAX_HW_QUEUES hardware queues per process (HIP's default 4; two streams on
# one in-order queue serialise).  Set before anything initialises the HIP runtime.
os.environ.setdefault("GPU_MAX_HW_QUEUES", "8")  # a caller's own setting is kept

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

METRIC = "DP cells/s (matrix fill) + alignment score bit-exact vs ref"
HBM_PEAK_GBS = 8000.0
BYTES_PER_CELL_TB = 26  # 24 B/cell fill (M, Ix, Iy int32 written + read once) + 2 B traceback word
BYTES_PER_CELL = 24
SCORING = dict(match_score=2, mismatch_score=-3, gap_open_score=-5, gap_extension_score=-1)
PROTEIN_SCORING = dict(scoring_mat_name="BLOSUM62", gap_open_score=-10)
DNA_SCORING_DESC = "match 2 / mismatch -3 / open -5 / ext -1"

WORKLOADS = {
    "c1": dict(m=1_000, n=1_000, traceback=True, alphabet="dna", seeds=(1, 2), scoring=SCORING,
               desc=f"C1: 1k x 1k DNA (SplitMix64 seeds 1,2), {DNA_SCORING_DESC}, full traceback"),
    "c2": dict(m=10_000, n=10_000, traceback=True, alphabet="dna", seeds=(1, 2), scoring=SCORING,
               desc=f"C2: 10k x 10k DNA (SplitMix64 seeds 1,2), {DNA_SCORING_DESC}, full traceback"),
    "c3": dict(m=100_000, n=100_000, traceback=True, alphabet="dna", seeds=(1, 2), scoring=SCORING,
               desc=f"C3: 100k x 100k DNA (SplitMix64 seeds 1,2), {DNA_SCORING_DESC}, full traceback"),
    "c4": dict(m=1_000_000, n=1_000_000, traceback=False, alphabet="dna", seeds=(1, 2), scoring=SCORING,
               desc=f"C4: 1M x 1M DNA (SplitMix64 seeds 1,2), {DNA_SCORING_DESC}, score only"),
    "c4tb": dict(m=1_000_000, n=1_000_000, traceback=True, alphabet="dna", seeds=(1, 2), scoring=SCORING, golden="c4",
                 desc=f"C4 with full traceback: 1M x 1M DNA (SplitMix64 seeds 1,2), {DNA_SCORING_DESC}; recompute "
                      "walk (checkpointing score fill, blocks recomputed beside the walk, DESIGN.md 5.8)"),
    # multi-rank rehearsal on ONE GPU only (tools/dist_rehearsal.sh): C4's rows, 16k columns, score only, so
    # that every rank's lane-kernel slab is resident beside the others' (not a BASELINE config)
    "c4r": dict(m=1_000_000, n=16_384, traceback=False, alphabet="dna", seeds=(1, 2), scoring=SCORING,
                desc=f"C4 rows x 16k columns DNA (SplitMix64 seeds 1,2), {DNA_SCORING_DESC}, score only "
                     "(multi-rank rehearsal on one GPU)"),
    "c5": dict(m=20_000, n=20_000, traceback=True, alphabet="protein", seeds=(3, 4), scoring=PROTEIN_SCORING,
               desc="C5: 20k x 20k protein (SplitMix64 seeds 3,4), BLOSUM62, gap_open_score -10, full traceback"),
}
SINGLE_GPU_DEFAULT = "c3"
MULTI_GPU_DEFAULT = "c4"

# committed profiles the roofline block is built from: PMC bytes and VALU
# instructions per fill launch, the fill kernel's static VALU mix, the VALU issue microbenchmark
# (C3: the pipeline's lane-skewed traceback fill, fill_lane_kernel<4,4,1,8>; C4: the lane-skewed
# score fill fill_lane_kernel<4,8,0,16>)
# (round 5, tools/profile_r05.sh on the round-5 fills: C3 / C5 / C2 the recompute walk's checkpointing lane fill
# fill_lane_kernel<4,4,0,16,...,RC,LATE>, C4 the score-only lane fill fill_lane_kernel<4,8,0,16>; the mixes from
# tools/lane_variant_asm.sh + tools/valu_mix.py --asm-block-with v_min3_i32)
TRAFFIC_FILES = {w: f"r06/traffic_{w}.json" for w in ("c3", "c4", "c5", "c2")}
VALU_FILES = {w: f"r06/valu_{w}.json" for w in ("c3", "c4", "c5", "c2")}
VALU_MIX_FILES = {w: f"r06/valu_mix_{w}.json" for w in ("c3", "c4", "c5", "c2")}
VALU_RATE_FILE = "r02/valu_rate.txt"


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


def workload_pair(wl):
    return splitmix(wl["m"], wl["seeds"][0], wl["alphabet"]), splitmix(wl["n"], wl["seeds"][1], wl["alphabet"])


# ----------------------------------------------------------------------------- CPU baselines
def host_cores():
    """CPU threads this process may use (the box sets OMP_NUM_THREADS to its CPU share)."""
    try:
        avail = len(os.sched_getaffinity(0))
    except AttributeError:
        avail = os.cpu_count() or 1
    share = os.environ.get("OMP_NUM_THREADS")
    return max(1, min(avail, int(share))) if share and share.isdigit() else avail


def cpu_baseline(py_sample=3000, c_sample=40_000, par_sample=100_000):
    """The reference's CPU path timed on this host (rank 0, N = 1), three legs (BASELINE.md plan):
    (1) the reference-equivalent pure-Python loop (oracle/pyport.py: nested lists of tuples, one keyword
        call per cell as globaligner.py:317-392), 1 core -- the reported `value`;
    (2) the C restatement (oracle/ga_oracle.c, int64 cells), 1 core;
    (3) the same C cells as a column-slab x row-band wavefront over every host thread."""
    import random
    from oracle import core, pyport
    s1, s2 = splitmix(py_sample, 1), splitmix(py_sample, 2)
    tables, _ = problem_tables(s1, s2)
    C = {x: {y: int(tables.sub[tables.code[x] * tables.K + tables.code[y]]) for y in tables.keys} for x in tables.keys}
    random.seed(0)
    t0 = time.perf_counter()
    T = pyport.fill(s1, s2, C, tables.gap_open, tables.max_cost)
    pyport.traceback(T, s1, s2, C, tables.gap_open)
    dt_py = time.perf_counter() - t0
    del T

    def c_leg(L, threads):
        a_s, b_s = splitmix(L, 1), splitmix(L, 2)
        tab = core.Tables(C)
        a, b = tab.codes(a_s), tab.codes(b_s)
        row0, col0 = core.boundary(tab, a, b, tables.gap_open, (tab.max_cost + 1) * L)
        t = time.perf_counter()
        if threads == 1:
            last = core.fill_score(tab, a, b, tables.gap_open, row0, col0)
        else:
            last = core.fill_score_parallel(tab, a, b, tables.gap_open, row0, col0, threads)
        return L * L / (time.perf_counter() - t), int(min(last))

    cores = host_cores()
    c1_rate, _ = c_leg(c_sample, 1)
    cp_rate, cp_cost = c_leg(par_sample, cores)
    return {"value": py_sample * py_sample / dt_py, "unit": "cells/s", "cores": 1, "kind": "port",
            "sample": f"{py_sample}x{py_sample} DNA (SplitMix64 seeds 1,2), fill + traceback, pure-Python port of the "
                      f"reference loop (oracle/pyport.py, keyword call per cell as globaligner.py:317-392), "
                      f"{dt_py:.1f} s",
            "host_nproc": os.cpu_count(), "host_threads_available": cores,
            "c_scalar_1core": {"value": c1_rate, "unit": "cells/s", "cores": 1,
                               "sample": f"{c_sample}x{c_sample} DNA fill + score, oracle/ga_oracle.c"},
            "c_threads_all_cores": {"value": cp_rate, "unit": "cells/s", "cores": cores,
                                    "sample": f"{par_sample}x{par_sample} DNA (= C3 cells) fill + score, "
                                              f"oracle/ga_oracle.c column-slab wavefront on {cores} threads",
                                    "cost": cp_cost}}


# ----------------------------------------------------------------------------- profiles / roofline
def _profile(name, key=None):
    path = os.path.join(ROOT, "profiles", name)
    if not name or not os.path.exists(path):
        return None
    try:
        d = json.load(open(path))
    except Exception:
        return None
    return d.get(key) if key else d


def golden_cost(workload):
    """The oracle-pinned cost of a workload (tests/golden/<workload>_cost.json), if committed."""
    path = os.path.join(ROOT, "tests", "golden", f"{workload}_cost.json")
    if not os.path.exists(path):
        return None
    return json.load(open(path)).get("cost")


def _variant_td(name):
    """Columns per lane (the second template argument) of a fill_lane_kernel name or mangled symbol, else None."""
    if not name:
        return None
    m = re.search(r"fill_lane_kernel<\s*\d+\s*,\s*(\d+)", name) or re.search(r"fill_lane_kernelILi\d+ELi(\d+)E", name)
    return int(m.group(1)) if m else None


def roofline(workload, wl, fill_ms, per_step_ms=None, profile_cells=None, fill_kind=None):
    """What bounds the fill, from the committed profiles.

    The row-scan fill keeps M/X/Y in registers and LDS: it moves ~1 B/cell (PMC FETCH+WRITE), not the
    24-26 B/cell of SURVEY 8(d)'s streaming model, and is VALU-issue bound.  So the bound is the VALU
    issue rate: SQ_INSTS_VALU per launch / kernel time (HIP events on the launch stream) against the
    chip's issue peak for the kernel's own op mix (tools/valu_mix.py over the hot loop, each form
    priced by the measured microbenchmark profiles/r02/valu_rate.txt).  The HBM model is kept as a
    secondary block."""
    cells = wl["m"] * wl["n"]
    bpc = BYTES_PER_CELL_TB if wl["traceback"] else BYTES_PER_CELL
    traffic = _profile(TRAFFIC_FILES.get(workload, ""), "fill_kernel_hbm_bytes_per_launch")
    insts = _profile(VALU_FILES.get(workload, ""), "sq_insts_valu_per_launch")
    if insts and profile_cells:
        # a slab of a multi-GPU step: the 1-GPU launch's instructions per cell times the slab's cells
        insts = insts * cells / profile_cells
        traffic = traffic * cells / profile_cells if traffic else traffic
    mix = _profile(VALU_MIX_FILES.get(workload, ""))
    kernel = (_profile(VALU_FILES.get(workload, ""), "kernel") or "fill").split("(")[0].replace("void ga::", "")
    secs = fill_ms * 1e-3
    hbm_alg = bpc * cells / secs / 1e9
    out = {"bound": "valu", "achieved": None, "peak": None, "unit": "wave64 VALU instructions/s", "frac": None,
           "traffic": traffic, "kernel": kernel, "kernel_ms": fill_ms, "units_per_launch": f"{cells} cells (m*n)",
           "hbm": {"bytes_per_cell_algorithmic": bpc, "achieved_GBps": hbm_alg, "peak_GBps": HBM_PEAK_GBS,
                   "frac": hbm_alg / HBM_PEAK_GBS,
                   "measured_GBps": traffic / secs / 1e9 if traffic else None,
                   "measured_bytes_per_cell": traffic / cells if traffic else None}}
    # the committed profiles must be of the kernel variant that ran (columns per lane): a default that changed after
    # the last profile run would otherwise divide one variant's instructions by another's time
    run_td = fill_kind[1] if fill_kind and fill_kind[0] in ("lane", "rc") else None
    prof_tds = {_variant_td(_profile(VALU_FILES.get(workload, ""), "kernel")), _variant_td((mix or {}).get("symbol"))}
    if run_td is not None and prof_tds != {run_td}:
        out["profile_mismatch"] = (f"the committed profiles are of {sorted(t for t in prof_tds if t)} columns per lane, "
                                   f"this fill ran {run_td}: achieved left null until tools/profile_r06.sh is re-run")
        insts = None
    if insts and mix:
        peak = mix["peak_valu_insts_per_s"]
        rate = insts / secs
        if per_step_ms:
            # pipelined steps: fill launches overlap (two at a time), so one launch's duration is not the
            # time the chip spends on it; the bound is the chip's VALU issue rate over the timed steps
            out["per_launch"] = {"achieved": rate, "frac": rate / peak, "kernel_ms": fill_ms,
                                 "note": "several fill launches run at once (ga_problem_align_many: four "
                                         "lane-kernel fills for C3-shaped problems, three row-scan fills otherwise)"}
            rate = insts / (per_step_ms * 1e-3)
            out["basis"] = "chip-wide: SQ_INSTS_VALU per alignment x alignments per second of the timed region"
        else:
            out["basis"] = "per launch: SQ_INSTS_VALU per launch / launch duration (HIP events)"
        out.update(achieved=rate, peak=peak, frac=rate / peak, insts_per_launch=insts, insts_per_cell=insts / cells,
                   peak_model=f"1024 SIMDs x 2.4 GHz / {mix['mean_simd_cycles_per_op']:.3f} SIMD cycles per op "
                              f"(hot-loop mix, profiles/{VALU_MIX_FILES[workload]}; rates {VALU_RATE_FILE})",
                   sources=f"profiles/{VALU_FILES[workload]} (rocprofv3 SQ_INSTS_VALU), "
                           f"profiles/{TRAFFIC_FILES[workload]} (FETCH_SIZE x2 + WRITE_SIZE)")
    return out


# ----------------------------------------------------------------------------- single GPU
def measure_single(wl, steps, warmup, pipelined=True):
    """Time `steps` passes of the hot path over one resident pair on cuda:0.

    Traceback workloads: the `steps` alignments are consecutive find_global_alignment-equivalent calls
    (each starts from the random state the previous left, from random.seed(0)), run through
    ga_problem_align_many: the walk of alignment k overlaps the fill of alignment k+1 on the GPU.  The
    single-alignment latency (fill + table + walk + strings, nothing overlapped) is measured separately."""
    import random
    import torch
    from globalign_amd import _native
    s1, s2 = workload_pair(wl)
    tables, _ = problem_tables(s1, s2, wl["scoring"])
    eng = _native.Engine(0)
    eng.load(tables.codes(s1), tables.codes(s2), tables)
    random.seed(0)
    mt0 = np.array(random.getstate()[1], dtype=np.uint32)
    out = {}
    if wl["traceback"] and pipelined:
        if warmup:
            eng.align_many(mt0, s1, s2, warmup)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        runs, mt_after = eng.align_many(mt0, s1, s2, steps)
        torch.cuda.synchronize()
        elapsed = time.perf_counter() - t0
        tm = eng.timings()
        fill_ms, walk_ms, rng_ms = tm["fill_ms"], tm["walk_ms"], tm["rng_ms"]
        cost, (a, mid, b), status = runs[0]
        for c_k, (a_k, _, b_k), st_k in runs:
            assert st_k == 0 and c_k == cost and a_k.replace("-", "") == s1 and b_k.replace("-", "") == s2
        out["aln"] = (a, mid, b)
        # the state after the FIRST alignment (the pin is for one call from random.seed(0))
        _, _, _, out["mt_after"] = eng.align(mt0, s1, s2)
        lat = []
        for _ in range(2):
            t1 = time.perf_counter()
            eng.align(mt0, s1, s2)
            lat.append((time.perf_counter() - t1) * 1e3)
        out["latency_ms"] = float(min(lat))
        out["mode"] = "pipelined: walk k beside fill k+1 (ga_problem_align_many)"
    else:
        fill_l, walk_l, rng_l = [], [], []
        result = None

        def step():
            if wl["traceback"]:
                return eng.align(mt0, s1, s2)
            return eng.fill(traceback=False)

        for _ in range(warmup):
            result = step()
        first = result
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            result = step()
            if wl["traceback"] and first is not None:
                # every call starts from the same random state: the same alignment (checked, untimed cost ~us)
                assert result[0] == first[0] and result[1] == first[1] and np.array_equal(result[3], first[3])
            tm = eng.timings()
            fill_l.append(tm["fill_ms"])
            walk_l.append(tm["walk_ms"] if wl["traceback"] else 0.0)
            rng_l.append(tm["rng_ms"] if wl["traceback"] else 0.0)
        torch.cuda.synchronize()
        elapsed = time.perf_counter() - t0
        fill_ms, walk_ms, rng_ms = float(np.mean(fill_l)), float(np.mean(walk_l)), float(np.mean(rng_l))
        cost = result[0]
        if wl["traceback"]:
            _, (a, mid, b), status, mt_after = result
            assert status == 0 and a.replace("-", "") == s1 and b.replace("-", "") == s2
            out["aln"] = (a, mid, b)
            out["mt_after"] = mt_after
            out["latency_ms"] = elapsed * 1e3 / steps
        out["mode"] = "one call per step"
    out["fill_kind"] = eng.fill_kind()
    if wl["traceback"]:
        out["walk_kind"] = eng.walk_kind()
    eng.close()
    cells = wl["m"] * wl["n"]
    out.update(elapsed=elapsed, cost=int(cost), cells=cells, value=cells * steps / elapsed,
               ms_per_step=elapsed * 1e3 / steps, fill_ms=float(fill_ms), walk_ms=float(walk_ms),
               rng_ms=float(rng_ms))
    return out


def traceback_pin(workload, r):
    """Alignment-string and random-state digests vs the oracle's (tests/golden/<workload>_aln.json)."""
    path = os.path.join(ROOT, "tests", "golden", f"{workload}_aln.json")
    if "aln" not in r or not os.path.exists(path):
        return None
    import hashlib
    g = json.load(open(path))
    a, mid, b = r["aln"]
    dig = hashlib.sha256("\n".join([a, mid, b]).encode()).hexdigest()[:16]
    st = hashlib.sha256(",".join(str(int(w)) for w in r["mt_after"]).encode()).hexdigest()[:32]
    return {"aln_len": len(mid), "aln_sha16": dig, "state_sha32": st,
            "matches_oracle": dig == g["aln_sha16"] and len(mid) == g["aln_len"] and st == g["state_sha32"]}


def single_line(args, workload, wl):
    # the headline: consecutive single find_global_alignment-equivalent calls (ga_problem_align), nothing
    # overlapped across steps (for C3-sized problems the recompute walk)
    r = measure_single(wl, args.steps, args.warmup, pipelined=False)
    gold = golden_cost(wl.get("golden", workload))
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
        "roofline": roofline(workload, wl, r["fill_ms"], fill_kind=r.get("fill_kind")),
        "fill_ms": r["fill_ms"],
        "fill_cells_per_s": r["cells"] / (r["fill_ms"] * 1e-3),
    }
    if wl["traceback"]:
        line["walk_ms"] = r["walk_ms"]
        line["walk_ns_per_step"] = r["walk_ms"] * 1e6 / max(len(r["aln"][1]), 1)
        line["host_tiebreak_ms"] = r["rng_ms"]
        line["latency_ms_per_alignment"] = r["latency_ms"]
        line["step_mode"] = r["mode"]
        line["fill_kind"] = r.get("fill_kind")
        line["walk_kind"] = r.get("walk_kind")  # 'jump': the tie-to-tie walk
        line["config"]["traceback_pin"] = traceback_pin(workload, r)
        if not args.no_extra:
            # the repeated-pair throughput mode (ga_problem_align_many: walk k beside fill k+1, stored words)
            q = measure_single(wl, max(4, args.steps), 2, pipelined=True)
            line["pipelined_repeated_pair"] = {
                "value": q["value"], "unit": "cells/s", "ms_per_step": q["ms_per_step"], "steps": max(4, args.steps),
                "cost_matches_oracle": (q["cost"] == gold) if gold is not None else None,
                "traceback_pin": traceback_pin(workload, q),
                "note": "consecutive alignments of the SAME pair with fills in flight beside the walks; not the "
                        "headline (a single call cannot overlap)"}
    if workload == SINGLE_GPU_DEFAULT and not args.no_extra:
        # one GPU's point of BASELINE's C4 scaling curve (the same pair bench.py --gpus N slabs)
        w4 = WORKLOADS["c4"]
        h = measure_single(w4, max(2, min(args.steps, 5)), 1)
        g4 = golden_cost("c4")
        line["c4"] = {"workload": w4["desc"], "value": h["value"], "unit": "cells/s", "n_gpus": 1,
                      "ms_per_step": h["ms_per_step"], "cost": h["cost"], "cost_matches_oracle": h["cost"] == g4,
                      "fill_ms": h["fill_ms"], "roofline": roofline("c4", w4, h["fill_ms"], fill_kind=h.get("fill_kind"))}
    if not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline()
    print(json.dumps(line), flush=True)


# ----------------------------------------------------------------------------- launcher
def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(args):
    """bench.py --gpus N run without a launcher: start the N ranks (one process per GPU) and wait."""
    backend = os.environ.get("GA_DIST_BACKEND", "nccl")
    if backend == "nccl":
        import torch
        ndev = torch.cuda.device_count()  # does not initialise the GPU (ROCm image)
        if ndev < args.gpus:
            print(f"bench.py: --gpus {args.gpus} needs {args.gpus} visible GPUs, found {ndev}", file=sys.stderr)
            return 2
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    return subprocess.call(cmd, env=env)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--workload", default=None, choices=sorted(WORKLOADS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extra", action="store_true", help="skip the C4 point of the N=1 line")
    ap.add_argument("--opt", action="append", default=[], metavar="GA_NAME=VALUE",
                    help="a context option (ga_ctx_create_opts: kernel variants for experiments); repeatable")
    args = ap.parse_args()
    if args.opt:
        from globalign_amd import _native
        for kv in args.opt:
            k, _, v = kv.partition("=")
            _native.OPTIONS[k] = v
    if args.gpus < 1:
        ap.error("--gpus must be >= 1")
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return launch_ranks(args)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but the launcher started {world} ranks", file=sys.stderr)
        return 2
    workload = args.workload or (SINGLE_GPU_DEFAULT if args.gpus == 1 else MULTI_GPU_DEFAULT)
    wl = WORKLOADS[workload]
    if world > 1:
        from globalign_amd import distributed
        return distributed.bench_main(args, wl, workload)
    single_line(args, workload, wl)
    return 0


if __name__ == "__main__":
    sys.exit(main())
