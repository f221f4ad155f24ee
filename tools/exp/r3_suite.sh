# Round 3: new recompute-walk tests, then the whole GPU suite, smoke, and the default bench line
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_rc.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r3_rc_tests.txt 2>&1 || { tail -40 gpurun_out/r3_rc_tests.txt; exit 1; }
tail -3 gpurun_out/r3_rc_tests.txt
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/r3_suite.txt 2>&1 || { tail -40 gpurun_out/r3_suite.txt; exit 1; }
tail -3 gpurun_out/r3_suite.txt
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3_smoke.txt 2>&1 || { tail -20 gpurun_out/r3_smoke.txt; exit 1; }
tail -1 gpurun_out/r3_smoke.txt
timeout -k 10 400 python -u bench.py > gpurun_out/r3_bench.json 2> gpurun_out/r3_bench.err || { tail -20 gpurun_out/r3_bench.err; exit 1; }
cat gpurun_out/r3_bench.json
