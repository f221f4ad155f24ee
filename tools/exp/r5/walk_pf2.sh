set -o pipefail
# round 5: the walker entries loaded two groups ahead, after the widening wait -- full GPU suite, then
# the C3 / C5 / C2 single calls twice
O=gpurun_out/r5_wpf2
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
for k in 1 2; do
for w in c3 c5 c2; do
  timeout -k 10 300 python -u bench.py --workload $w --steps 20 --warmup 5 --no-cpu-baseline --no-extra > $O/bench_${w}_$k.json 2> $O/bench_${w}_$k.err || { tail -20 $O/bench_${w}_$k.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('$O/bench_${w}_$k.json').read().strip().splitlines()[-1])
print('$w', 'ms/step', round(d['ms_per_step'],3), 'fill', round(d.get('fill_ms',0),3), 'walk', round(d.get('walk_ms',0),3), 'ns/step', round(d.get('walk_ns_per_step',0),2), 'pin', (d['config'].get('traceback_pin') or {}).get('matches_oracle'))
"
done
done
