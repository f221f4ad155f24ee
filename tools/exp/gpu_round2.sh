set -o pipefail
cd /root/repo
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 300 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
timeout -k 10 400 python -u bench.py --workload c4tb --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench_c4tb.json 2> gpurun_out/bench_c4tb.err || exit 1
