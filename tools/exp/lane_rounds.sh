set -o pipefail
mkdir -p gpurun_out/exp
timeout -k 10 600 python -u -m pytest tests/test_gpu_lane.py -x -q --timeout 120 --timeout-method thread > gpurun_out/exp/lane_tests.log 2>&1 || { tail -30 gpurun_out/exp/lane_tests.log; exit 1; }
tail -1 gpurun_out/exp/lane_tests.log
for shape in "1000000 1000000" "1000000 500000" "1000000 250000" "1000000 125000" "1000000 16384"; do
  set -- $shape
  timeout -k 10 120 python -u tools/fill_sweep.py $1 $2 3 0 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['m'], d['n'], d['kind'], [round(x,2) for x in d['fill_ms']], d['cost'])" || exit 1
done
