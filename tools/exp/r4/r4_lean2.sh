set -o pipefail
# round 4: the lean sub-chunk with the last compute wave's direct hand-off (GA_LANE_DIRECT=1: rows from lanes 48..63
# straight to HBM after each sub-chunk, the IO wave only frees ring slots) and with the IO / profile waves at
# priority 3 -- lane stamps (C3 and the N = 8 slab shape) and the C3 bench line
mkdir -p gpurun_out/r4_lean2
O=gpurun_out/r4_lean2
for v in base direct prio3 directprio3; do
  case $v in
    base) E="";; direct) E="GA_LANE_DIRECT=1";; prio3) E="GA_LANE_IOPRIO=3";; directprio3) E="GA_LANE_DIRECT=1 GA_LANE_IOPRIO=3";;
  esac
  env $E GA_FILL_MODE=lane timeout -k 10 120 python -u tools/lane_stamps.py 100000 100000 > $O/stamps_c3_$v.json 2> $O/stamps_c3_$v.err || { tail -5 $O/stamps_c3_$v.err; exit 1; }
  env $E GA_FILL_MODE=lane timeout -k 10 120 python -u tools/lane_stamps.py 1000000 125000 > $O/stamps_slab_$v.json 2> $O/stamps_slab_$v.err || { tail -5 $O/stamps_slab_$v.err; exit 1; }
  env $E timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extra > $O/c3_$v.json 2> $O/c3_$v.err || { tail -5 $O/c3_$v.err; exit 1; }
done
python3 - <<'PY'
import json
O = "gpurun_out/r4_lean2"
for v in ("base", "direct", "prio3", "directprio3"):
    for w in ("c3", "slab"):
        d = json.loads(open(f"{O}/stamps_{w}_{v}.json").read().strip().splitlines()[-1])
        print(f"{v} stamps {w}: dbg {d['fill_ms_dbg']:.2f} intra {d['end_lag_intra_wg_us']:.2f} cross {d['end_lag_cross_wg_us']:.2f} mean {d['end_lag_mean_us']:.2f} busy {[round(x['cyc_per_step_busy'],1) for x in d['by_simd'].values()]} wait_edge {[round(x['wait_edge_frac'],3) for x in d['by_simd'].values()]}")
    d = json.loads(open(f"{O}/c3_{v}.json").read().strip().splitlines()[-1])
    print(f"{v} bench c3: call {d['ms_per_step']:.3f} fill {d['fill_ms']:.3f} walk {d['walk_ms']:.3f} pin {d['config']['traceback_pin']['matches_oracle']}")
PY
