# round 2: pipeline with the walk chain decoupled from host decoding
set -o pipefail
mkdir -p gpurun_out/exp
timeout -k 10 300 python -u -m pytest tests/test_gpu_many.py -x -q --timeout 300 --timeout-method thread > gpurun_out/exp/many.log 2>&1 || { tail -30 gpurun_out/exp/many.log; exit 1; }
tail -1 gpurun_out/exp/many.log
for W in c3 c5 c2; do
  timeout -k 10 300 python -u bench.py --workload $W --steps 20 --warmup 5 --no-cpu-baseline --no-extra > gpurun_out/exp/bench_$W.json 2> gpurun_out/exp/bench_$W.err || { tail -20 gpurun_out/exp/bench_$W.err; exit 1; }
done
