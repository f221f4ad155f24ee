set -o pipefail
# round 5: C4 on one GPU (TD 8, two rounds of 4-wave workgroups) under the round-4 lane changes:
# out wave on / off, lean asm on / off, poll window adaptive (0) / 64 / 192; C4 fill ms and the cost pin per variant
O=gpurun_out/r5_c4ab
mkdir -p $O
run() {
  name=$1; shift
  env "$@" timeout -k 10 150 python -u bench.py --workload c4 --steps 3 --warmup 1 --no-cpu-baseline > $O/$name.json 2> $O/$name.err || { tail -5 $O/$name.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('$O/$name.json').read().strip().splitlines()[-1])
print('$name', 'fill', round(d['fill_ms'],2), 'ms/step', round(d['ms_per_step'],2), 'cost_ok', d['config'].get('cost_matches_oracle'), 'kind', d.get('fill_kind'))
"
}
run default GA_X=0
run outwave0 GA_LANE_OUTWAVE=0
run asm0 GA_LANE_ASM=0
run poll192 GA_LANE_POLLWIN=192
run poll64 GA_LANE_POLLWIN=64
run default2 GA_X=0
