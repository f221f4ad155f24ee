set -o pipefail
# round 5: a workgroup's first wave reads its edges early (GA_LANE_XEARLY=1) against the late read everywhere: rc/lane
# GPU tests with it on, lane stamps of the C3-shape fill, the C3 / C5 / C2 single calls
O=gpurun_out/r5_xearly
mkdir -p $O
GA_LANE_XEARLY=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_lane.py tests/test_gpu_rc.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
for x in 0 1 0 1; do
  GA_LANE_XEARLY=$x GA_FILL_MODE=lane GA_LANE_COLS_PER_LANE=4 timeout -k 10 120 python -u tools/lane_stamps.py 100000 100000 > $O/stamps_$x.json 2> $O/stamps_$x.err || { tail -5 $O/stamps_$x.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('$O/stamps_$x.json').read().strip().splitlines()[-1])
print('xearly $x', 'plain', round(d['fill_ms_plain'],3), 'dbg', round(d['fill_ms_dbg'],3), 'intra', round(d['end_lag_intra_wg_us'],2), 'cross', round(d['end_lag_cross_wg_us'],2), 'busy', round(d['cycles_per_step_median'],1))
"
done
for x in 0 1; do
for w in c3 c5 c2; do
  GA_LANE_XEARLY=$x timeout -k 10 300 python -u bench.py --workload $w --steps 20 --warmup 5 --no-cpu-baseline --no-extra > $O/bench_${w}_$x.json 2> $O/bench_${w}_$x.err || { tail -20 $O/bench_${w}_$x.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('$O/bench_${w}_$x.json').read().strip().splitlines()[-1])
print('xearly $x $w', 'ms/step', round(d['ms_per_step'],3), 'fill', round(d.get('fill_ms',0),3), 'walk', round(d.get('walk_ms',0),3), 'pin', (d['config'].get('traceback_pin') or {}).get('matches_oracle'))
"
done
done
