set -o pipefail
# anti-diagonal fill with TD columns per lane: parity at TD = 1, 2, 4, then the slab shapes
mkdir -p gpurun_out
for td in 1 2 4; do
  GA_FILL_MODE=diag GA_DIAG_COLS_PER_LANE=$td timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_blocked.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t22_$td.log 2>&1 || { tail -30 gpurun_out/t22_$td.log; exit 1; }
  echo "td=$td $(tail -1 gpurun_out/t22_$td.log)"
done
for n in 125000 250000 500000 1000000; do for td in 2 4; do
  echo "diag td=$td $(GA_FILL_MODE=diag GA_DIAG_COLS_PER_LANE=$td timeout -k 10 120 python -u tools/fill_sweep.py 1000000 $n 3 0)" >> gpurun_out/sweep22.txt || exit 1
done; done
for td in 2 4; do
GA_FILL_MODE=diag GA_DIAG_COLS_PER_LANE=$td timeout -k 10 120 python -u tools/fill_stamps.py 1000000 125000 > gpurun_out/s22_diag_n8_$td.json || exit 1
GA_FILL_MODE=diag GA_DIAG_COLS_PER_LANE=$td timeout -k 10 120 python -u tools/fill_stamps.py 100000 100000 > gpurun_out/s22_diag_c3_$td.json || exit 1
done
