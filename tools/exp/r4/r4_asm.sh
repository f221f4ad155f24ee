set -o pipefail
# round 4: the hand-scheduled lane step + the profile wave -- GPU suite, then A/B bench lines
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r4_suite_asm.log 2>&1 || { tail -60 gpurun_out/r4_suite_asm.log; exit 1; }
tail -3 gpurun_out/r4_suite_asm.log
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r4_bench_asm.json 2> gpurun_out/r4_bench_asm.err || { tail -20 gpurun_out/r4_bench_asm.err; exit 1; }
GA_LANE_ASM=0 timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r4_bench_noasm.json 2> gpurun_out/r4_bench_noasm.err || { tail -20 gpurun_out/r4_bench_noasm.err; exit 1; }
timeout -k 10 120 python -u bench.py --workload c5 --steps 20 --warmup 5 --no-cpu-baseline --no-extra > gpurun_out/r4_c5.json 2> gpurun_out/r4_c5.err || { tail -20 gpurun_out/r4_c5.err; exit 1; }
GA_RC=1 timeout -k 10 120 python -u bench.py --workload c5 --steps 20 --warmup 5 --no-cpu-baseline --no-extra > gpurun_out/r4_c5_rc.json 2> gpurun_out/r4_c5_rc.err || { tail -20 gpurun_out/r4_c5_rc.err; exit 1; }
python3 - <<'PY'
import json
for f in ("gpurun_out/r4_bench_asm.json", "gpurun_out/r4_bench_noasm.json", "gpurun_out/r4_c5.json", "gpurun_out/r4_c5_rc.json"):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    s = f"{f}: call {d['ms_per_step']:.3f} fill {d['fill_ms']:.3f} walk {d.get('walk_ms', 0):.3f} kind {d.get('fill_kind')} pin {d['config'].get('traceback_pin', {}).get('matches_oracle')}"
    if "c4" in d:
        s += f" C4 {d['c4']['fill_ms']:.2f} ok {d['c4']['cost_matches_oracle']}"
    if "pipelined_repeated_pair" in d:
        s += f" pipe {d['pipelined_repeated_pair']['ms_per_step']:.3f}"
    print(s)
PY
