set -o pipefail
# round 4: the lean path's ring-space test in an SGPR and its checkpoint store as one asm dwordx2 (no exec changes):
# lane / rc tests, C3-shape stamps at TD 4, the C3 / C5 / C2 single calls
O=gpurun_out/r4_glue2
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_lane.py tests/test_gpu_rc.py -m gpu > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
GA_LANE_COLS_PER_LANE=4 GA_FILL_MODE=lane timeout -k 10 120 python -u tools/lane_stamps.py 100000 100000 > $O/stamps_c3_td4.json 2> $O/stamps_c3_td4.err || { tail -5 $O/stamps_c3_td4.err; exit 1; }
python3 -c "
import json
d=json.loads(open('$O/stamps_c3_td4.json').read().strip().splitlines()[-1])
print('td4 c3', 'dbg', round(d['fill_ms_dbg'],2), 'mean lag', round(d['end_lag_mean_us'],2), 'busy', [round(x['cyc_per_step_busy'],1) for x in d['by_simd'].values()])
"
for w in c3 c5 c2; do
  timeout -k 10 200 python -u bench.py --workload $w --steps 20 --warmup 5 --no-cpu-baseline --no-extra > $O/$w.json 2> $O/$w.err || { tail -5 $O/$w.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('$O/$w.json').read().strip().splitlines()[-1])
print('$w call', round(d['ms_per_step'],3), 'fill', round(d['fill_ms'],3), 'walk', round(d['walk_ms'],3), d.get('fill_kind'), 'pin', d['config']['traceback_pin']['matches_oracle'])
"
done
