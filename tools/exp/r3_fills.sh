# Round 3: score-only C3 fills by kernel and geometry (steady state), and the group-step microbenchmark
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/r3_fills.txt
: > $O
timeout -k 10 120 tools/micro/group_bench > gpurun_out/group_bench2.txt 2>&1 || exit 1
for cfg in "GA_FILL_MODE=row" "GA_FILL_MODE=row GA_COLS_PER_LANE=2 GA_FILL_NWC=4" "GA_FILL_MODE=row GA_COLS_PER_LANE=2 GA_FILL_NWC=8" \
           "GA_FILL_MODE=row GA_COLS_PER_LANE=4 GA_FILL_NWC=4" "GA_FILL_MODE=lane GA_LANE_COLS_PER_LANE=2" \
           "GA_FILL_MODE=lane GA_LANE_COLS_PER_LANE=4" "GA_FILL_MODE=lane GA_LANE_COLS_PER_LANE=2 GA_LANE_SUB=8"; do
  env $cfg timeout -k 10 120 python -u tools/exp/r3_fills.py 100000 100000 4 >> $O 2>&1 || exit 1
done
