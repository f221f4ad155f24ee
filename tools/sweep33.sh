set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_banded.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/t36.log 2>&1 || { tail -40 gpurun_out/t36.log; exit 1; }
tail -1 gpurun_out/t36.log
for k in 1 2; do timeout -k 10 300 python -u bench.py --workload c5 --no-cpu-baseline > gpurun_out/b36_c5_$k.json 2>/dev/null || exit 1; done
timeout -k 10 300 python -u bench.py --workload c3 --no-cpu-baseline > gpurun_out/b36_c3.json 2>/dev/null || exit 1
