set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_banded.py tests/test_gpu_parity.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/t31.log 2>&1 || { tail -40 gpurun_out/t31.log; exit 1; }
tail -2 gpurun_out/t31.log
timeout -k 10 400 python -u bench.py --workload c4tb --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench_c4tb.json 2> gpurun_out/bench_c4tb.err || { tail -20 gpurun_out/bench_c4tb.err; exit 1; }
