# full GPU check: parity suite, default bench, rocprof kernel stats of the default bench
set -o pipefail
cd /root/repo
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -3 gpurun_out/gpu_tests.log
timeout -k 10 300 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_default -o run -- python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/prof_default.log 2>&1 || { tail -20 gpurun_out/prof_default.log; exit 1; }
find gpurun_out/prof_default -name "*kernel_stats.csv" | head -3
