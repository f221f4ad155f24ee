set -o pipefail
# round 4: the lean sub-chunk alone in the kernel (round-3 asm path removed): lane / rc / slab / parity tests, lane
# stamps with the lag distribution (XCD of every stripe) with and without the direct hand-off, the C3 bench line
mkdir -p gpurun_out/r4_lean4
O=gpurun_out/r4_lean4
timeout -k 10 600 python -u -m pytest tests/test_gpu_rc.py tests/test_gpu_lane.py tests/test_distributed_gpu.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for v in base direct; do
  case $v in base) E="";; direct) E="GA_LANE_DIRECT=1";; esac
  env $E GA_FILL_MODE=lane timeout -k 10 120 python -u tools/lane_stamps.py 100000 100000 > $O/stamps_c3_$v.json 2> $O/stamps_c3_$v.err || { tail -5 $O/stamps_c3_$v.err; exit 1; }
  env $E GA_FILL_MODE=lane timeout -k 10 120 python -u tools/lane_stamps.py 1000000 125000 > $O/stamps_slab_$v.json 2> $O/stamps_slab_$v.err || { tail -5 $O/stamps_slab_$v.err; exit 1; }
  env $E timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/c3_$v.json 2> $O/c3_$v.err || { tail -5 $O/c3_$v.err; exit 1; }
done
python3 - <<'PY'
import json
O = "gpurun_out/r4_lean4"
for v in ("base", "direct"):
    for w in ("c3", "slab"):
        d = json.loads(open(f"{O}/stamps_{w}_{v}.json").read().strip().splitlines()[-1])
        ld = d["lag_distribution"]
        print(f"{v} stamps {w}: dbg {d['fill_ms_dbg']:.2f} intra {d['end_lag_intra_wg_us']:.2f} cross {d['end_lag_cross_wg_us']:.2f} mean {d['end_lag_mean_us']:.2f} busy {[round(x['cyc_per_step_busy'],1) for x in d['by_simd'].values()]}")
        print(f"    pct {ld['end_lag_pct_us']} max {ld['end_lag_max_us']:.1f} sum {ld['end_lag_sum_ms']} links {ld['cross_wg_links']}")
        print(f"    top {[(t['stripe'], round(t['lag_us'],1), t['wave'], t['cross'], t['xcd']) for t in ld['end_lag_top'][:8]]}")
    d = json.loads(open(f"{O}/c3_{v}.json").read().strip().splitlines()[-1])
    print(f"{v} bench c3: call {d['ms_per_step']:.3f} fill {d['fill_ms']:.3f} walk {d['walk_ms']:.3f} pin {d['config']['traceback_pin']['matches_oracle']} C4 {d['c4']['fill_ms']:.2f} ok {d['c4']['cost_matches_oracle']} pipe {d['pipelined_repeated_pair']['ms_per_step']:.3f}")
PY
