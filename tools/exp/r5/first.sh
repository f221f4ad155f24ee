set -o pipefail
# round 5, first GPU call: the tie-to-tie trip micro-benchmark, then the XCD-order A/B (xcd.sh)
mkdir -p gpurun_out/r5_xcd
timeout -k 10 60 tools/micro/jump_trip > gpurun_out/r5_xcd/jump_trip.txt 2>&1 && cat gpurun_out/r5_xcd/jump_trip.txt && bash tools/exp/r5/xcd.sh
