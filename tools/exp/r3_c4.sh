# Round 3: C4 score-only fill (rounds of lane workgroups) by hand-off mode; C3 rc fill by hand-off mode
set -eo pipefail
for d in 1 0; do
  GA_LANE_DIRECT=$d timeout -k 10 120 python -u tools/exp/r3_fills.py 1000000 1000000 3 | grep -v amdgpu.ids
  GA_LANE_DIRECT=$d timeout -k 10 120 python -u tools/exp/r3_fills.py 1000000 125000 3 | grep -v amdgpu.ids
  GA_LANE_DIRECT=$d timeout -k 10 120 python -u tools/exp/r3_rc_diag.py 100000 96:48:1 | grep -v amdgpu.ids | cut -c1-120
done
