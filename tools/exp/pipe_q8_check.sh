# round 2: four lane fills with eight hardware queues as the bench default: pipeline parity, default bench
set -o pipefail
mkdir -p gpurun_out/exp
GPU_MAX_HW_QUEUES=8 timeout -k 10 400 python -u -m pytest tests/test_gpu_many.py -x -q --timeout 240 --timeout-method thread > gpurun_out/exp/q8many.log 2>&1 || { tail -30 gpurun_out/exp/q8many.log; exit 1; }
tail -1 gpurun_out/exp/q8many.log
for r in 1 2; do
  rm -f gpurun_out/exp/trace_c3_q8d$r.jsonl
  GA_PIPE_TRACE=gpurun_out/exp/trace_c3_q8d$r.jsonl timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/exp/q8d$r.json 2> gpurun_out/exp/q8d$r.err || { tail -20 gpurun_out/exp/q8d$r.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/exp/q8d$r.json'));print('c3', round(d['ms_per_step'],3), 'fill', round(d['fill_ms'],2), 'walk', round(d['walk_ms'],2), d['config']['traceback_pin']['matches_oracle'], 'c4', round(d['c4']['ms_per_step'],1))"
done
