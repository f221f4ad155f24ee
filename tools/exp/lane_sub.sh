# lane kernel: 8- vs 16-step sub-chunks (GA_LANE_SUB) at the slab and lone-stripe shapes; parity first
set -o pipefail
mkdir -p gpurun_out/exp
timeout -k 10 600 python -u -m pytest tests/test_gpu_lane.py -x -q --timeout 120 --timeout-method thread > gpurun_out/exp/lane_tests.log 2>&1 || { tail -30 gpurun_out/exp/lane_tests.log; exit 1; }
tail -1 gpurun_out/exp/lane_tests.log
GA_LANE_SUB=8 timeout -k 10 600 python -u -m pytest tests/test_gpu_lane.py -x -q --timeout 120 --timeout-method thread -k "cost or workgroups or protein_blosum or custom or sentinel" > gpurun_out/exp/lane_tests8.log 2>&1 || { tail -30 gpurun_out/exp/lane_tests8.log; exit 1; }
tail -1 gpurun_out/exp/lane_tests8.log
for sub in 8 16; do
  for shape in "1000000 512" "1000000 125000" "1000000 250000" "1000000 500000" "1000000 1000000"; do
    set -- $shape
    GA_LANE_SUB=$sub timeout -k 10 120 python -u tools/fill_sweep.py $1 $2 3 0 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('sub=$sub', d['m'], d['n'], d['kind'], [round(x,2) for x in d['fill_ms']], d['cost'])" || exit 1
  done
done
