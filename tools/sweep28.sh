set -o pipefail
# anti-diagonal fill after the partial-stripe fix: parity, then the slab shapes by width
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_diag.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t28.log 2>&1 || { tail -30 gpurun_out/t28.log; exit 1; }
tail -1 gpurun_out/t28.log
for n in 125000 250000 500000; do for td in 1 2 4; do
  echo "diag td=$td $(GA_FILL_MODE=diag GA_DIAG_COLS_PER_LANE=$td timeout -k 10 120 python -u tools/fill_sweep.py 1000000 $n 3 0)" >> gpurun_out/sweep28.txt || exit 1
done; done
for td in 1 2 4; do
  echo "diag td=$td $(GA_FILL_MODE=diag GA_DIAG_COLS_PER_LANE=$td timeout -k 10 120 python -u tools/fill_sweep.py 100000 100000 3 0)" >> gpurun_out/sweep28.txt || exit 1
done
echo "row $(timeout -k 10 120 python -u tools/fill_sweep.py 100000 100000 3 0)" >> gpurun_out/sweep28.txt || exit 1
