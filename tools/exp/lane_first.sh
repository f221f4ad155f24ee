# lane-skewed fill: GPU parity, then fill times at the C4 / slab shapes against the row scan
set -o pipefail
mkdir -p gpurun_out/exp
timeout -k 10 300 python -u -m pytest tests/test_gpu_lane.py -x -q --timeout 120 --timeout-method thread > gpurun_out/exp/lane_tests.log 2>&1 || { tail -30 gpurun_out/exp/lane_tests.log; exit 1; }
tail -2 gpurun_out/exp/lane_tests.log
for shape in "1000000 125000" "1000000 250000" "1000000 500000" "1000000 1000000" "100000 100000"; do
  set -- $shape
  for mode in row lane; do
    GA_FILL_MODE=$mode timeout -k 10 120 python -u tools/fill_sweep.py $1 $2 3 0 >> gpurun_out/exp/lane_times.jsonl || exit 1
  done
done
for td in 1 2 4; do
  GA_FILL_MODE=lane GA_LANE_COLS_PER_LANE=$td timeout -k 10 120 python -u tools/fill_sweep.py 1000000 125000 3 0 >> gpurun_out/exp/lane_times.jsonl || exit 1
done
cat gpurun_out/exp/lane_times.jsonl
