set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/t47.log 2>&1 || { tail -40 gpurun_out/t47.log; exit 1; }
tail -1 gpurun_out/t47.log
echo "c4 $(timeout -k 10 120 python -u tools/fill_sweep.py 1000000 1000000 3 0)" >> gpurun_out/sweep47.txt || exit 1
echo "n8row $(GA_FILL_MODE=row timeout -k 10 120 python -u tools/fill_sweep.py 1000000 125000 3 0)" >> gpurun_out/sweep47.txt || exit 1
echo "n4row $(GA_FILL_MODE=row timeout -k 10 120 python -u tools/fill_sweep.py 1000000 250000 3 0)" >> gpurun_out/sweep47.txt || exit 1
echo "n2row $(GA_FILL_MODE=row timeout -k 10 120 python -u tools/fill_sweep.py 1000000 500000 3 0)" >> gpurun_out/sweep47.txt || exit 1
