set -o pipefail
# round 5: the single C3 call's stripe width after the lean-loop changes: 2 against 4 columns per lane (fill and walk)
O=gpurun_out/r5_td
mkdir -p $O
for k in 1 2; do
for td in 4 2; do
  GA_LANE_COLS_PER_LANE=$td timeout -k 10 300 python -u bench.py --workload c3 --steps 20 --warmup 5 --no-cpu-baseline --no-extra > $O/bench_c3_td${td}_$k.json 2> $O/bench_c3_td${td}_$k.err || { tail -20 $O/bench_c3_td${td}_$k.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('$O/bench_c3_td${td}_$k.json').read().strip().splitlines()[-1])
print('td $td', 'ms/step', round(d['ms_per_step'],3), 'fill', round(d.get('fill_ms',0),3), 'walk', round(d.get('walk_ms',0),3), 'kind', d.get('fill_kind'), 'pin', (d['config'].get('traceback_pin') or {}).get('matches_oracle'))
"
done
done
