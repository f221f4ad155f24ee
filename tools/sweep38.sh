set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_blocked.py tests/test_distributed_gpu.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/t38.log 2>&1 || { tail -40 gpurun_out/t38.log; exit 1; }
tail -1 gpurun_out/t38.log
timeout -k 10 200 python -u tools/fill_stamps.py 100000 100000 --tb > gpurun_out/s38_c3.json || exit 1
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/b38.json 2>/dev/null || exit 1
