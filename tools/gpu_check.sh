set -o pipefail
# full GPU suite + the default bench line (C3 pipelined, with the C4 point and the CPU baseline)
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/gpu_check.log 2>&1 || { tail -40 gpurun_out/gpu_check.log; exit 1; }
tail -2 gpurun_out/gpu_check.log
timeout -k 10 400 python -u bench.py > gpurun_out/check_bench.json 2> gpurun_out/check_bench.err || { tail -20 gpurun_out/check_bench.err; exit 1; }
cat gpurun_out/check_bench.json
