#!/bin/bash
# The assembly of ONE fill_lane_kernel variant (seconds instead of `make asm`'s minutes), for tools/valu_mix.py and
# for reading the lean loop's glue (round 5):
#   tools/lane_variant_asm.sh "4, 4, 0, 16, false, false, true, true" out.s
# (the recompute fill of the single calls; C4's score-only fill is "4, 8, 0, 16, false, false, false, false")
set -e
ARGS=${1:?template arguments}
OUT=${2:?output .s}
HERE=$(cd "$(dirname "$0")/.." && pwd)
T=$(mktemp -d)
cat > $T/v.hip <<HIP
#define GA_LANE_KERNEL_ONLY
#include "ga_lane.hip"
namespace ga {
template __global__ void fill_lane_kernel<$ARGS>(FillArgs p);
}
HIP
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -I$HERE/globalign_amd/csrc --offload-device-only -S -o "$OUT" $T/v.hip
rm -rf $T
