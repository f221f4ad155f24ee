set -o pipefail
mkdir -p gpurun_out
timeout -k 10 60 ./tools/micro/lane_step2 > gpurun_out/r4_lane_step2.txt 2>&1 || exit 1
cat gpurun_out/r4_lane_step2.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r4_suite.log 2>&1 || { tail -60 gpurun_out/r4_suite.log; exit 1; }
tail -3 gpurun_out/r4_suite.log
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r4_bench.json 2> gpurun_out/r4_bench.err || { tail -20 gpurun_out/r4_bench.err; exit 1; }
cat gpurun_out/r4_bench.json
