set -o pipefail
# round 4: IO / profile wave priority -- lane stamps (C3 and C5 shapes) and bench lines at GA_LANE_IOPRIO 0 / 3
mkdir -p gpurun_out/r4_prio
O=gpurun_out/r4_prio
for pr in 0 3; do
  GA_LANE_IOPRIO=$pr GA_FILL_MODE=lane timeout -k 10 120 python -u tools/lane_stamps.py 100000 100000 > $O/stamps_c3_p$pr.json 2> $O/stamps_c3_p$pr.err || { tail -5 $O/stamps_c3_p$pr.err; exit 1; }
  GA_LANE_IOPRIO=$pr GA_FILL_MODE=lane timeout -k 10 120 python -u tools/lane_stamps.py 20000 20000 c5 > $O/stamps_c5_p$pr.json 2> $O/stamps_c5_p$pr.err || { tail -5 $O/stamps_c5_p$pr.err; exit 1; }
  GA_LANE_IOPRIO=$pr timeout -k 10 150 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extra > $O/c3_p$pr.json 2> $O/c3_p$pr.err || { tail -5 $O/c3_p$pr.err; exit 1; }
  GA_LANE_IOPRIO=$pr GA_RC=1 timeout -k 10 120 python -u bench.py --workload c5 --steps 20 --warmup 5 --no-cpu-baseline --no-extra > $O/c5rc_p$pr.json 2> $O/c5rc_p$pr.err || { tail -5 $O/c5rc_p$pr.err; exit 1; }
done
python3 - <<'PY'
import json
O = "gpurun_out/r4_prio"
for pr in (0, 3):
    for w in ("c3", "c5"):
        d = json.loads(open(f"{O}/stamps_{w}_p{pr}.json").read().strip().splitlines()[-1])
        print(f"prio {pr} stamps {w}: fill {d['fill_ms_dbg']:.2f} intra {d['end_lag_intra_wg_us']:.2f} cross {d['end_lag_cross_wg_us']:.2f} mean {d['end_lag_mean_us']:.2f} cyc/step {d['cycles_per_step_median']:.1f} busy {[round(v['cyc_per_step_busy'],1) for v in d['by_simd'].values()]} wait_prof {[round(v['wait_prof_frac'],3) for v in d['by_simd'].values()]}")
    for w in ("c3", "c5rc"):
        d = json.loads(open(f"{O}/{w}_p{pr}.json").read().strip().splitlines()[-1])
        print(f"prio {pr} bench {w}: call {d['ms_per_step']:.3f} fill {d['fill_ms']:.3f} walk {d['walk_ms']:.3f} pin {d['config']['traceback_pin']['matches_oracle']}")
PY
