set -o pipefail
# round 5: the recompute (checkpointing) fill against the plain score-only lane fill at the same geometry (C3, TD 4),
# same box; then the C3 / C2 single calls; rc GPU tests first (checkpoint spacing as a power of two)
O=gpurun_out/r5_rcvl
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_rc.py tests/test_gpu_lane.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
for k in 1 2; do
  GA_FILL_MODE=lane GA_LANE_COLS_PER_LANE=4 timeout -k 10 120 python -u tools/fill_score.py 100000 100000 5 || exit 1
  for w in c3 c2; do
    timeout -k 10 300 python -u bench.py --workload $w --steps 20 --warmup 5 --no-cpu-baseline --no-extra > $O/bench_${w}_$k.json 2> $O/bench_${w}_$k.err || { tail -20 $O/bench_${w}_$k.err; exit 1; }
    python3 -c "
import json
d=json.loads(open('$O/bench_${w}_$k.json').read().strip().splitlines()[-1])
print('$w', 'ms/step', round(d['ms_per_step'],3), 'fill', round(d.get('fill_ms',0),3), 'walk', round(d.get('walk_ms',0),3), 'tb', round(d.get('host_tiebreak_ms',0),3), 'pin', (d['config'].get('traceback_pin') or {}).get('matches_oracle'))
"
  done
done
