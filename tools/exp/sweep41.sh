set -o pipefail
# anti-diagonal fill with 8-step sub-chunks: parity, then pace at the slab shapes
mkdir -p gpurun_out
for td in 1 2 4; do
  GA_FILL_MODE=diag GA_DIAG_COLS_PER_LANE=$td timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_blocked.py tests/test_gpu_diag.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t41_$td.log 2>&1 || { tail -30 gpurun_out/t41_$td.log; exit 1; }
  echo "td=$td $(tail -1 gpurun_out/t41_$td.log)"
done
timeout -k 10 300 python -u -m pytest tests/test_distributed_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/t41_d.log 2>&1 || { tail -30 gpurun_out/t41_d.log; exit 1; }
tail -1 gpurun_out/t41_d.log
for n in 125000 250000 1000000; do for td in 1 2; do
  echo "diag td=$td $(GA_FILL_MODE=diag GA_DIAG_COLS_PER_LANE=$td timeout -k 10 120 python -u tools/fill_sweep.py 1000000 $n 3 0)" >> gpurun_out/sweep41.txt || exit 1
done; done
GA_FILL_MODE=diag GA_DIAG_COLS_PER_LANE=1 timeout -k 10 120 python -u tools/fill_stamps.py 1000000 125000 > gpurun_out/s41_n8.json || exit 1
GA_FILL_MODE=diag GA_DIAG_COLS_PER_LANE=1 timeout -k 10 120 python -u tools/fill_stamps.py 1000000 2048 > gpurun_out/s41_chain.json || exit 1
