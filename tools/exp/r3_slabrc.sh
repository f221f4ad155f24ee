# Round 3: slab traceback through the recompute walk (gloo ranks sharing one GPU) + the r03 profiles
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_distributed_gpu.py -x -v --timeout 240 --timeout-method thread > gpurun_out/r3_slabrc.txt 2>&1 || { tail -40 gpurun_out/r3_slabrc.txt; exit 1; }
tail -4 gpurun_out/r3_slabrc.txt
timeout -k 10 300 python -u -m pytest tests/test_gpu_rc.py tests/test_gpu_lane.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r3_late.txt 2>&1 || { tail -40 gpurun_out/r3_late.txt; exit 1; }
tail -2 gpurun_out/r3_late.txt
timeout -k 10 120 python -u tools/exp/r3_fills.py 1000000 1000000 2 | grep -v amdgpu.ids
bash tools/profile_r03.sh
