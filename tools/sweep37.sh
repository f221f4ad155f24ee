set -o pipefail
# workgroup hand-off by polling the rows (sentinel) instead of a progress word
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/t37.log 2>&1 || { tail -40 gpurun_out/t37.log; exit 1; }
tail -1 gpurun_out/t37.log
timeout -k 10 200 python -u tools/fill_stamps.py 100000 100000 --tb > gpurun_out/s37_c3.json || exit 1
timeout -k 10 200 python -u tools/fill_stamps.py 1000000 125000 > gpurun_out/s37_n8.json || exit 1
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/b37.json 2>/dev/null || exit 1
