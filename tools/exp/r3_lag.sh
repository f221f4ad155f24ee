# Round 3: lane fill hand-over changes (late edge reads, direct hand-off stores): parity + C3 / C4-slab timing
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_lane.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r3_lag_tests.txt 2>&1 || { tail -30 gpurun_out/r3_lag_tests.txt; exit 1; }
tail -2 gpurun_out/r3_lag_tests.txt
timeout -k 10 120 python -u tools/exp/r3_rc_check.py quick > gpurun_out/r3_lag_rc.txt 2>&1 || exit 1
grep ALL gpurun_out/r3_lag_rc.txt
for td in 2 4; do
  GA_FILL_MODE=lane GA_LANE_COLS_PER_LANE=$td timeout -k 10 120 python -u tools/lane_stamps.py 100000 100000 > gpurun_out/r3_lag_td$td.json 2>&1 || exit 1
  tail -1 gpurun_out/r3_lag_td$td.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: d[k] for k in d if k.startswith('end_lag') or k in ('TD','fill_ms_dbg','fill_ms_plain')})"
done
GA_FILL_MODE=lane GA_LANE_COLS_PER_LANE=2 timeout -k 10 120 python -u tools/lane_stamps.py 1000000 125000 > gpurun_out/r3_lag_c4s.json 2>&1 || exit 1
tail -1 gpurun_out/r3_lag_c4s.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: d[k] for k in d if k.startswith('end_lag') or k in ('TD','fill_ms_dbg','fill_ms_plain')})"
GA_FILL_MODE=lane GA_LANE_COLS_PER_LANE=2 timeout -k 10 120 python -u tools/exp/r3_fills.py 100000 100000 4 | grep -v amdgpu.ids
timeout -k 10 120 python -u tools/exp/r3_rc_diag.py 100000 96:48:1 | grep -v amdgpu.ids
