# round 2: GPU suite, the default bench line, then the round-2 profiles
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 400 python -u bench.py > gpurun_out/bench_n1.json 2> gpurun_out/bench_n1.err || { tail -20 gpurun_out/bench_n1.err; exit 1; }
bash tools/exp/profile_r02.sh
