set -o pipefail
# round 5: the lean statement reading the next edges after step 8 instead of 12 (more time for the reads to land before
# the statement's closing wait; the stripe trails its producer by 4 more steps): a library built with -DGA_LANE_RS=8
# (globalign_amd/_lib/rs8, GA_LIB_PATH) against the default -- lane / rc GPU tests with it, C3-shape lane stamps, and
# the C3 / C5 / C2 single calls
O=gpurun_out/r5_rs8
mkdir -p $O
RS8=$GRAFT_REPO_ROOT/globalign_amd/_lib/rs8/libglobalign_amd.so
GA_LIB_PATH=$RS8 timeout -k 10 600 python -u -m pytest tests/test_gpu_lane.py tests/test_gpu_rc.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
for k in 1 2; do
for v in def rs8; do
  if [ $v = rs8 ]; then export GA_LIB_PATH=$RS8; else unset GA_LIB_PATH; fi
  GA_FILL_MODE=lane GA_LANE_COLS_PER_LANE=4 timeout -k 10 120 python -u tools/lane_stamps.py 100000 100000 > $O/stamps_${v}_$k.json 2> $O/stamps_${v}_$k.err || { tail -5 $O/stamps_${v}_$k.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('$O/stamps_${v}_$k.json').read().strip().splitlines()[-1])
print('$v', 'plain', round(d['fill_ms_plain'],3), 'intra', round(d['end_lag_intra_wg_us'],2), 'cross', round(d['end_lag_cross_wg_us'],2), 'busy', round(d['by_simd']['0']['cyc_per_step_busy'],1))
"
  for w in c3 c5 c2; do
    timeout -k 10 300 python -u bench.py --workload $w --steps 20 --warmup 5 --no-cpu-baseline --no-extra > $O/bench_${w}_${v}_$k.json 2> $O/bench_${w}_${v}_$k.err || { tail -20 $O/bench_${w}_${v}_$k.err; exit 1; }
    python3 -c "
import json
d=json.loads(open('$O/bench_${w}_${v}_$k.json').read().strip().splitlines()[-1])
print('$v $w', 'ms/step', round(d['ms_per_step'],3), 'fill', round(d.get('fill_ms',0),3), 'walk', round(d.get('walk_ms',0),3), 'pin', (d['config'].get('traceback_pin') or {}).get('matches_oracle'))
"
  done
done
done
