set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_lane.py -x -q --timeout 120 --timeout-method thread > gpurun_out/exp/lane_tests.log 2>&1 || { tail -30 gpurun_out/exp/lane_tests.log; exit 1; }
tail -1 gpurun_out/exp/lane_tests.log
for shape in "1000000 128" "1000000 125000" "1000000 1000000"; do
  set -- $shape
  GA_FILL_MODE=lane timeout -k 10 120 python -u tools/lane_stamps.py $1 $2 || exit 1
done
