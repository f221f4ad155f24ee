# round 2: pipelined concurrent fills -- parity tests, then C3/C5/C2 bench lines
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_many.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_many.log 2>&1 || { tail -30 gpurun_out/gpu_many.log; exit 1; }
tail -2 gpurun_out/gpu_many.log
for W in c3 c5 c2; do
  timeout -k 10 300 python -u bench.py --workload $W --steps 20 --warmup 5 --no-cpu-baseline --no-extra > gpurun_out/bench_$W.json 2> gpurun_out/bench_$W.err || { tail -20 gpurun_out/bench_$W.err; exit 1; }
done
