# Round 3 (second session): the C3 recompute-walk call with the lane fill's direct hand-off (GA_LANE_DIRECT)
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/r3b_direct.txt
: > $O
for cfg in "GA_LANE_DIRECT=0" "GA_LANE_DIRECT=1" "GA_LANE_DIRECT=0" "GA_LANE_DIRECT=1"; do
  echo "== $cfg" >> $O
  env $cfg timeout -k 10 120 python -u tools/exp/r3_rc_diag.py 100000 96:48:1 >> $O 2>&1 || exit 1
done
timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-extra --steps 10 --warmup 3 >> $O 2>&1 || exit 1
