# Round 3: the lane kernel's per-stripe hand-over lag at C3 (end-time differences of consecutive stripes)
set -o pipefail
mkdir -p gpurun_out
for td in 2 4; do
  GA_FILL_MODE=lane GA_LANE_COLS_PER_LANE=$td timeout -k 10 120 python -u tools/lane_stamps.py 100000 100000 > gpurun_out/r3_lanelag_td$td.json 2>&1 || exit 1
done
GA_FILL_MODE=lane GA_LANE_COLS_PER_LANE=2 timeout -k 10 120 python -u tools/lane_stamps.py 1000000 125000 > gpurun_out/r3_lanelag_c4s.json 2>&1 || exit 1
