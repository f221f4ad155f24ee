# Round 3: recompute walk by loader count (12 / 13 leave the walker's SIMD to the walker and the helper)
set -eo pipefail
for nl in 14 13 12; do
  GA_RC_LOADERS=$nl timeout -k 10 200 python -u tools/exp/r3_rc_diag.py 100000 96:48:1 | grep -v amdgpu.ids | cut -c1-200
done
