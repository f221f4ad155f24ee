set -o pipefail
# round 5: lean sub-chunk addresses from loop-invariant per-lane parts -- lane / rc / parity GPU tests, then the single
# calls (C3 twice, C5, C2), the score-only C3-shape fill and C4
O=gpurun_out/r5_glue
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_lane.py tests/test_gpu_rc.py tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
GA_FILL_MODE=lane GA_LANE_COLS_PER_LANE=4 timeout -k 10 120 python -u tools/fill_score.py 100000 100000 5 || exit 1
for w in c3 c5 c2 c3; do
  timeout -k 10 300 python -u bench.py --workload $w --steps 20 --warmup 5 --no-cpu-baseline --no-extra > $O/bench_$w.json 2> $O/bench_$w.err || { tail -20 $O/bench_$w.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('$O/bench_$w.json').read().strip().splitlines()[-1])
print('$w', 'ms/step', round(d['ms_per_step'],3), 'fill', round(d.get('fill_ms',0),3), 'walk', round(d.get('walk_ms',0),3), 'pin', (d['config'].get('traceback_pin') or {}).get('matches_oracle'), 'cost', d['config'].get('cost_matches_oracle'))
"
done
timeout -k 10 200 python -u bench.py --workload c4 --steps 3 --warmup 1 --no-cpu-baseline --no-extra > $O/bench_c4.json 2> $O/bench_c4.err || { tail -20 $O/bench_c4.err; exit 1; }
python3 -c "
import json
d=json.loads(open('$O/bench_c4.json').read().strip().splitlines()[-1])
print('c4 fill', round(d['fill_ms'],2), 'cost', d['config'].get('cost_matches_oracle'))
"
