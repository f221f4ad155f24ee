set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/t30.log 2>&1 || { tail -40 gpurun_out/t30.log; exit 1; }
tail -2 gpurun_out/t30.log
echo "auto $(timeout -k 10 120 python -u tools/fill_sweep.py 1000000 125000 3 0)" > gpurun_out/sweep30.txt || exit 1
echo "auto $(timeout -k 10 120 python -u tools/fill_sweep.py 1000000 124928 3 0)" >> gpurun_out/sweep30.txt || exit 1
