# Round 3: where the lane kernel's time goes at C3 size (score only): per-stripe stamps at TD 1 / 2 / 4
set -o pipefail
mkdir -p gpurun_out
for td in 1 2 4; do
  GA_FILL_MODE=lane GA_LANE_COLS_PER_LANE=$td timeout -k 10 120 python -u tools/lane_stamps.py 100000 100000 > gpurun_out/r3_lanec3_td$td.json 2>&1 || exit 1
done
GA_FILL_MODE=lane GA_LANE_COLS_PER_LANE=2 GA_FILL_NWC=8 timeout -k 10 120 python -u tools/lane_stamps.py 100000 100000 > gpurun_out/r3_lanec3_td2n8.json 2>&1 || exit 1
timeout -k 10 300 python -u tools/exp/r3_single.py c3 c5 c2 > gpurun_out/r3_single.txt 2>&1
