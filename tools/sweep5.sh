set -o pipefail
GA_COLS_PER_LANE=8 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/parity_T8.log 2>&1 || { tail -30 gpurun_out/parity_T8.log; exit 1; }
tail -1 gpurun_out/parity_T8.log
for T in 8 4; do
  GA_COLS_PER_LANE=$T timeout -k 5 120 python -u tools/fill_stamps.py 100000 1000000 >> gpurun_out/stamps5.txt || exit 1
  GA_COLS_PER_LANE=$T timeout -k 5 120 python -u tools/fill_sweep.py 1000000 1000000 2 0 >> gpurun_out/sweep5.txt || exit 1
done
