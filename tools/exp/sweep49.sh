set -o pipefail
# anti-diagonal TD=1 fast path through the hand-scheduled 4-step blocks
mkdir -p gpurun_out
GA_FILL_MODE=diag GA_DIAG_COLS_PER_LANE=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_blocked.py tests/test_gpu_diag.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t49.log 2>&1 || { tail -30 gpurun_out/t49.log; exit 1; }
tail -1 gpurun_out/t49.log
timeout -k 10 300 python -u -m pytest tests/test_distributed_gpu.py tests/test_gpu_diag.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/t49b.log 2>&1 || { tail -30 gpurun_out/t49b.log; exit 1; }
tail -1 gpurun_out/t49b.log
for n in 2048 125000; do
  echo "diag1 $(GA_FILL_MODE=diag GA_DIAG_COLS_PER_LANE=1 timeout -k 10 120 python -u tools/fill_sweep.py 1000000 $n 3 0)" >> gpurun_out/sweep49.txt || exit 1
done
echo "diag1 $(GA_FILL_MODE=diag GA_DIAG_COLS_PER_LANE=1 timeout -k 10 120 python -u tools/fill_sweep.py 100000 100000 3 0)" >> gpurun_out/sweep49.txt || exit 1
