set -o pipefail
# round 4: the out wave on / off for the final C3 single call (4-column recompute fill), and C5 / C2
O=gpurun_out/r4_outw4
mkdir -p $O
for v in 1 0; do
  for w in c3 c5 c2; do
    GA_LANE_OUTWAVE=$v timeout -k 10 200 python -u bench.py --workload $w --steps 20 --warmup 5 --no-cpu-baseline --no-extra > $O/${w}_$v.json 2> $O/${w}_$v.err || { tail -5 $O/${w}_$v.err; exit 1; }
    python3 -c "
import json
d=json.loads(open('$O/${w}_$v.json').read().strip().splitlines()[-1])
print('outwave $v $w call', round(d['ms_per_step'],3), 'fill', round(d['fill_ms'],3), 'walk', round(d['walk_ms'],3), 'pin', d['config']['traceback_pin']['matches_oracle'])
"
  done
done
