set -o pipefail
# round 4: the lean asm sub-chunk (GA_LANE_ASM=1, default) against the round-3 asm steps (GA_LANE_ASM=2): lane / rc /
# slab parity, then lane stamps (C3 and the N = 8 slab shape) and bench lines
mkdir -p gpurun_out/r4_lean
O=gpurun_out/r4_lean
timeout -k 10 600 python -u -m pytest tests/test_gpu_rc.py tests/test_gpu_lane.py tests/test_distributed_gpu.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for a in 1 2; do
  GA_LANE_ASM=$a GA_FILL_MODE=lane timeout -k 10 120 python -u tools/lane_stamps.py 100000 100000 > $O/stamps_c3_a$a.json 2> $O/stamps_c3_a$a.err || { tail -5 $O/stamps_c3_a$a.err; exit 1; }
  GA_LANE_ASM=$a GA_FILL_MODE=lane timeout -k 10 120 python -u tools/lane_stamps.py 1000000 125000 > $O/stamps_slab_a$a.json 2> $O/stamps_slab_a$a.err || { tail -5 $O/stamps_slab_a$a.err; exit 1; }
  GA_LANE_ASM=$a timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/c3_a$a.json 2> $O/c3_a$a.err || { tail -5 $O/c3_a$a.err; exit 1; }
done
python3 - <<'PY'
import json
O = "gpurun_out/r4_lean"
for a in (1, 2):
    for w in ("c3", "slab"):
        d = json.loads(open(f"{O}/stamps_{w}_a{a}.json").read().strip().splitlines()[-1])
        print(f"asm {a} stamps {w}: plain {d['fill_ms_plain']:.2f} dbg {d['fill_ms_dbg']:.2f} intra {d['end_lag_intra_wg_us']:.2f} cross {d['end_lag_cross_wg_us']:.2f} mean {d['end_lag_mean_us']:.2f} cyc/step {d['cycles_per_step_median']:.1f} busy {[round(v['cyc_per_step_busy'],1) for v in d['by_simd'].values()]}")
    d = json.loads(open(f"{O}/c3_a{a}.json").read().strip().splitlines()[-1])
    print(f"asm {a} bench c3: call {d['ms_per_step']:.3f} fill {d['fill_ms']:.3f} walk {d['walk_ms']:.3f} pin {d['config']['traceback_pin']['matches_oracle']} C4 {d['c4']['fill_ms']:.2f} ok {d['c4']['cost_matches_oracle']} pipe {d['pipelined_repeated_pair']['ms_per_step']:.3f}")
PY
