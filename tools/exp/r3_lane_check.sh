# Round 3: lane-kernel change check: GPU parity of the lane / rc / slab paths, then fill timings
set -eo pipefail
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_lane.py tests/test_gpu_rc.py tests/test_gpu_parity.py tests/test_distributed_gpu.py > gpurun_out/r3_lane_tests.log 2>&1
tail -3 gpurun_out/r3_lane_tests.log
timeout -k 10 120 python -u tools/exp/r3_fills.py 1000000 1000000 3 | grep -v amdgpu.ids
timeout -k 10 120 python -u tools/exp/r3_fills.py 1000000 125000 3 | grep -v amdgpu.ids
timeout -k 10 120 python -u tools/exp/r3_rc_diag.py 100000 96:48:1 | grep -v amdgpu.ids
