# round 2: hand-formed one-byte traceback code in the lane kernel: parity, then the C3 bench (twice)
set -o pipefail
mkdir -p gpurun_out/exp
timeout -k 10 400 python -u -m pytest tests/test_gpu_lane.py tests/test_gpu_many.py -x -q --timeout 240 --timeout-method thread > gpurun_out/exp/code.log 2>&1 || { tail -30 gpurun_out/exp/code.log; exit 1; }
tail -1 gpurun_out/exp/code.log
for r in 1 2; do
  rm -f gpurun_out/exp/trace_c3_code$r.jsonl
  GA_PIPE_TRACE=gpurun_out/exp/trace_c3_code$r.jsonl timeout -k 10 200 python -u bench.py --workload c3 --no-cpu-baseline --no-extra > gpurun_out/exp/code_c3_$r.json 2> gpurun_out/exp/code_c3_$r.err || { tail -20 gpurun_out/exp/code_c3_$r.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/exp/code_c3_$r.json'));print('c3', round(d['ms_per_step'],3), 'fill', round(d['fill_ms'],2), 'walk', round(d['walk_ms'],2), d['config']['traceback_pin']['matches_oracle'])"
done
