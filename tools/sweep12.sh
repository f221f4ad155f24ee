set -o pipefail
GA_COLS_PER_LANE=4 timeout -k 10 300 python -u -m pytest tests/test_gpu_blocked.py -x -q --timeout 120 --timeout-method thread > gpurun_out/blocked_T4.log 2>&1 || { tail -30 gpurun_out/blocked_T4.log; exit 1; }
tail -1 gpurun_out/blocked_T4.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_banded.py -x -q --timeout 200 --timeout-method thread > gpurun_out/banded.log 2>&1 || { tail -30 gpurun_out/banded.log; exit 1; }
tail -1 gpurun_out/banded.log
for T in 4 2; do
GA_COLS_PER_LANE=$T timeout -k 5 120 python -u tools/fill_sweep.py 65536 1000000 3 1 >> gpurun_out/sweep12.txt || exit 1
done
timeout -k 10 400 python -u bench.py --workload c4tb --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench_c4tb.json 2> gpurun_out/bench_c4tb.err || exit 1
