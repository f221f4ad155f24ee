"""Diagnostic: per-stripe timestamps of one lane-skewed fill (fill_lane_kernel DBG variant).

    GA_FILL_MODE=lane python tools/lane_stamps.py [m] [n]

Prints one JSON line: the fill time, the chain's start lags (intra- and cross-workgroup), stripe
durations, and the cycles each stripe waited for its left edge / the profile / ring space, grouped by
the SIMD the wave ran on (HW_ID bits 5:4) -- a chain runs at its slowest stripe's pace, and that
stripe is the one that never waits for its left neighbour.  Every stripe is resident from the kernel's start, so its
edge wait includes the ramp (stripe s first waits about s lags for its left neighbour to reach row SUB):
"steady_state" splits that first wait off.""" 
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from globalign_amd import _native  # noqa: E402

m = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
n = int(sys.argv[2]) if len(sys.argv) > 2 else 125_000
# optional third argument: a bench workload whose alphabet, seeds and scoring to use (e.g. c5)
wl = bench.WORKLOADS[sys.argv[3]] if len(sys.argv) > 3 else None
if wl:
    s1, s2 = bench.splitmix(m, wl["seeds"][0], wl["alphabet"]), bench.splitmix(n, wl["seeds"][1], wl["alphabet"])
    tables, _ = bench.problem_tables(s1, s2, wl["scoring"])
else:
    s1, s2 = bench.splitmix(m, 1), bench.splitmix(n, 2)
    tables, _ = bench.problem_tables(s1, s2)
# context options for experiments (GA_OPTIONS="GA_NAME=VALUE;..."; the library reads only its shipped knobs from
# the environment)
for kv in filter(None, os.environ.get("GA_OPTIONS", "").split(";")):
    _native.OPTIONS[kv.partition("=")[0]] = kv.partition("=")[2]
eng = _native.Engine(0)
eng.load(tables.codes(s1), tables.codes(s2), tables)
L = _native.load_library()
L.ga_debug_stamps.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_int64]
eng.fill(traceback=False)
plain_ms = eng.kernel_ms()[0]
L.ga_debug_stamps(eng._h, 1, None, 0)
cost, _ = eng.fill(traceback=False)
kind, T, ns, nwc, nslabs = eng.fill_kind()
W = 20  # LK_DBG_WORDS (ga_lane.h)
buf = np.zeros(W * ns, dtype=np.uint64)
L.ga_debug_stamps(eng._h, 0, buf.ctypes.data, buf.size)
L.ga_debug_stamps(eng._h, 0, None, 0)
st = buf.reshape(ns, W).astype(np.int64)
t0 = st[:, 0].min()
start, end = (st[:, 0] - t0) / 100.0, (st[:, 1] - t0) / 100.0  # microseconds (100 MHz)
dur = end - start
tot = np.maximum(st[:, 5], 1)
simd = (st[:, 6] >> 4) & 3
wave_in_wg = np.arange(ns) % nwc
lag = np.diff(start)
# every stripe runs the same rows at the same busy pace once its left edge arrives, so consecutive
# stripes' END times differ by the hand-over lag between them (the start stamps are the kernel's start)
elag = np.diff(end)
cross = np.array([(k + 1) % nwc == 0 for k in range(ns - 1)], dtype=bool)
by_simd = {}
for sd in range(4):
    sel = simd == sd
    if sel.any():
        by_simd[int(sd)] = {"stripes": int(sel.sum()), "dur_us_median": float(np.median(dur[sel])),
                            "wait_edge_frac": float(np.median(st[sel, 2] / tot[sel])),
                            "wait_prof_frac": float(np.median(st[sel, 3] / tot[sel])),
                            "wait_space_frac": float(np.median(st[sel, 4] / tot[sel])),
                            "cyc_per_step_busy": float(np.median((tot[sel] - st[sel, 2] - st[sel, 3] - st[sel, 4]) /
                                                                 (m + 63)))}
# the first edge wait (word 12) is the ramp: stripe s waits for its left neighbour to reach row SUB, about s lags after
# the kernel's start; everything after it (words 2 - 12) is the steady state's waiting
first_w = st[:, 12]
steady_w = st[:, 2] - first_w
t_first = (st[:, 13] - t0) / 100.0
steady_ns = (end - t_first) * 1e3 / (m + 63)
dec = np.array_split(np.arange(ns), 10)
steady = {"wait_edge_first_frac_median": float(np.median(first_w / tot)),
          "wait_edge_steady_frac_median": float(np.median(steady_w / tot)),
          "wait_edge_steady_frac_p90": float(np.percentile(steady_w / tot, 90)),
          "wait_edge_steady_frac_by_decile": [float(np.median(steady_w[d] / tot[d])) for d in dec],
          "first_edge_us_by_decile": [float(np.median(t_first[d])) for d in dec],
          "ns_per_step_after_first_edge_median": float(np.median(steady_ns)),
          "ns_per_step_after_first_edge_by_decile": [float(np.median(steady_ns[d])) for d in dec],
          "cyc_per_step_after_first_edge_median": float(np.median((tot - first_w) / (m + 63)))}
# the first 64 steps (the ramp's masked sub-chunks, or the lean ones with lean0) against the next 64 (words 18, 19)
if (st[:, 18] > 0).all() and (st[:, 19] > 0).all():
    steady["ns_per_step_first64_median"] = float(np.median((st[:, 18] - st[:, 13]) * 10.0 / 64))
    steady["ns_per_step_next64_median"] = float(np.median((st[:, 19] - st[:, 18]) * 10.0 / 64))
# the lag between consecutive stripes at rows 256 / 1024 / 4096 / 16384 (words 14..17), intra- and cross-workgroup
# links apart: a link's lag is set where it first grows (a consumer never catches up), DESIGN.md 5.6.2
lag_by_row = {}
for k, row in enumerate((256, 1024, 4096, 16384)):
    tr = st[:, 14 + k]
    if row < m and (tr > 0).all():
        lr = np.diff((tr - t0) / 100.0)
        lag_by_row[str(row)] = {"intra_median_us": float(np.median(lr[~cross])) if (~cross).any() else None,
                                "cross_median_us": float(np.median(lr[cross])) if cross.any() else None,
                                "cross_p90_us": float(np.percentile(lr[cross], 90)) if cross.any() else None}
lag_by_row["end"] = {"intra_median_us": float(np.median(elag[~cross])) if (~cross).any() else None,
                     "cross_median_us": float(np.median(elag[cross])) if cross.any() else None,
                     "cross_p90_us": float(np.percentile(elag[cross], 90)) if cross.any() else None}
by_wave = {int(w): {"wait_edge_frac": float(np.median(st[wave_in_wg == w, 2] / tot[wave_in_wg == w])),
                    "simd_mode": int(np.bincount(simd[wave_in_wg == w]).argmax())} for w in range(min(nwc, ns))}
if os.environ.get("LANE_STAMPS_DUMP"):
    # the raw per-stripe stamps: start, end (s_memrealtime), wait cycles (edges, profile, ring space), total cycles,
    # HW_ID, XCC_ID
    np.save(os.environ["LANE_STAMPS_DUMP"], st)
xcc = st[:, 7] & 0xF
xcross = xcc[1:] != xcc[:-1]
pct = {f"p{q}": float(np.percentile(elag, q)) for q in (10, 50, 90, 99)} if len(elag) else {}
top = np.argsort(elag)[::-1][:12] if len(elag) else []
dist = {"end_lag_pct_us": pct, "end_lag_max_us": float(elag.max()) if len(elag) else None,
        "end_lag_sum_ms": {"intra": float(elag[~cross].sum() / 1e3), "cross_same_xcd": float(elag[cross & ~xcross].sum() / 1e3),
                           "cross_other_xcd": float(elag[cross & xcross].sum() / 1e3)},
        "cross_wg_links": {"same_xcd": int((cross & ~xcross).sum()), "other_xcd": int((cross & xcross).sum())},
        "end_lag_top": [{"stripe": int(i + 1), "lag_us": float(elag[i]), "wave": int((i + 1) % nwc),
                         "cross": bool(cross[i]), "xcd": [int(xcc[i]), int(xcc[i + 1])]} for i in top]}
# the row-m/2 probe: per link s -> s+1, from the producer's publish of row m/2 to the consumer's
# knowing it landed; cross-workgroup links through the out-path's store and the IO wave's landing in ring 0
probe = {}
if (st[:, 8] > 0).all() and (st[:, 9] > 0).all():
    pub, avail = (st[:, 9] - t0) / 100.0, (st[:, 8] - t0) / 100.0
    link = avail[1:] - pub[:-1]
    probe["pub_to_avail_us"] = {"intra": float(np.median(link[~cross])) if (~cross).any() else None,
                                "cross": float(np.median(link[cross])) if cross.any() else None}
    ci = np.nonzero(cross)[0]
    if len(ci) and (st[ci, 11] > 0).all() and (st[ci + 1, 10] > 0).all():
        stored, landed = (st[ci, 11] - t0) / 100.0, (st[ci + 1, 10] - t0) / 100.0
        probe["cross_parts_us"] = {"pub_to_stored": float(np.median(stored - pub[ci])),
                                   "stored_to_landed": float(np.median(landed - stored)),
                                   "landed_to_avail": float(np.median(avail[ci + 1] - landed))}
        probe["cross_parts_mean_us"] = {"pub_to_stored": float(np.mean(stored - pub[ci])),
                                        "stored_to_landed": float(np.mean(landed - stored)),
                                        "landed_to_avail": float(np.mean(avail[ci + 1] - landed))}
    # the consumer's own publish of row m/2 after it knew its edge row landed (the stripe's skew + batching)
    own = pub - avail
    probe["avail_to_own_pub_us"] = float(np.median(own))
print(json.dumps({
    "probe_m2": probe,
    "m": m, "n": n, "cost": int(cost), "kind": kind, "TD": T, "nstripes": ns, "nwc": nwc, "nslabs": nslabs,
    "fill_ms_plain": plain_ms, "fill_ms_dbg": eng.kernel_ms()[0],
    "last_end_us": float(end.max()), "last_start_us": float(start.max()),
    "lag_intra_wg_us": float(np.mean(lag[~cross])) if (~cross).any() else None,
    "lag_cross_wg_us": float(np.mean(lag[cross])) if cross.any() else None,
    "end_lag_intra_wg_us": float(np.median(elag[~cross])) if (~cross).any() else None,
    "end_lag_cross_wg_us": float(np.median(elag[cross])) if cross.any() else None,
    "end_lag_mean_us": float(np.mean(elag)) if len(elag) else None,
    "end_lag_by_wave_us": {int(w): float(np.median(elag[(np.arange(ns - 1) % nwc) == w])) for w in range(min(nwc, ns - 1))},
    "stripe_dur_us_median": float(np.median(dur)), "stripe_dur_us_max": float(dur.max()),
    "ns_per_step_median": float(np.median(dur) * 1e3 / (m + 63)),
    "cycles_per_step_median": float(np.median(tot / (m + 63))),
    "by_simd": by_simd, "by_wave": by_wave, "lag_distribution": dist, "steady_state": steady, "lag_by_row": lag_by_row,
}), flush=True)
