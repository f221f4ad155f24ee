# parity of the blocked fill (forced T) on the GPU parity suite, then a timing sweep
set -o pipefail
for T in 4 2; do
  GA_COLS_PER_LANE=$T timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/parity_T$T.log 2>&1 || { echo "parity T=$T failed"; tail -30 gpurun_out/parity_T$T.log; exit 1; }
  tail -2 gpurun_out/parity_T$T.log
done
for T in 1 2 4; do
  for f in "" 0; do
    if [ -z "$f" ]; then unset GA_FILL_LDS_FLOOR; else export GA_FILL_LDS_FLOOR=$f; fi
    GA_COLS_PER_LANE=$T timeout -k 5 120 python -u tools/fill_sweep.py 250000 1000000 4 0 >> gpurun_out/sweep2.txt || exit 1
    GA_COLS_PER_LANE=$T timeout -k 5 120 python -u tools/fill_sweep.py 100000 100000 4 1 >> gpurun_out/sweep2.txt || exit 1
  done
done
