# round-end evidence: full GPU suite, the default bench line (C3 pipelined + C4 point + CPU legs), rocprofv3
# kernel stats of it, and the C4 fill's FETCH/WRITE/SQ passes (each its own run)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/gpu_check.log 2>&1 || { tail -40 gpurun_out/gpu_check.log; exit 1; }
tail -1 gpurun_out/gpu_check.log
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/check_bench.json 2> gpurun_out/check_bench.err || { tail -20 gpurun_out/check_bench.err; exit 1; }
bash tools/profile_lane.sh
