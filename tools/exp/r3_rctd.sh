# Round 3: the recompute walk's fill at C3 by lane width (TD 2 is lane_geometry's choice)
set -eo pipefail
for td in 2 4 1 8; do
  GA_LANE_COLS_PER_LANE=$td timeout -k 10 200 python -u tools/exp/r3_rc_diag.py 100000 96:48:1 | grep -v amdgpu.ids | cut -c1-140
done
