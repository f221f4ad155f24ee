set -o pipefail
# round 5: C3 recompute fill time against the staircase checkpoint spacing (GA_RC_EVERY), to price the checkpoint
# stores; the walk's recompute blocks grow with the spacing, so only fill_ms is read here
O=gpurun_out/r5_every
mkdir -p $O
for e in 64 128 256 512 1024; do
  GA_RC_EVERY=$e timeout -k 10 300 python -u bench.py --workload c3 --steps 10 --warmup 3 --no-cpu-baseline --no-extra > $O/bench_$e.json 2> $O/bench_$e.err || { tail -20 $O/bench_$e.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('$O/bench_$e.json').read().strip().splitlines()[-1])
print('every $e', 'ms/step', round(d['ms_per_step'],3), 'fill', round(d.get('fill_ms',0),3), 'walk', round(d.get('walk_ms',0),3), 'pin', (d['config'].get('traceback_pin') or {}).get('matches_oracle'))
"
done
