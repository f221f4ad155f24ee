set -o pipefail
# round 4: columns per lane of the recompute fill for the single calls of C3, C5, C2 (GA_RC=1 forces the recompute
# walk for the smaller problems)
O=gpurun_out/r4_td
mkdir -p $O
run() {
  local w=$1 tag=$2; shift 2
  env "$@" timeout -k 10 200 python -u bench.py --workload $w --steps 20 --warmup 5 --no-cpu-baseline --no-extra > $O/${w}_$tag.json 2> $O/${w}_$tag.err || { tail -5 $O/${w}_$tag.err; return 1; }
  python3 -c "
import json
d=json.loads(open('$O/${w}_$tag.json').read().strip().splitlines()[-1])
print('$w $tag', 'call', round(d['ms_per_step'],3), 'fill', round(d['fill_ms'],3), 'walk', round(d['walk_ms'],3), d.get('fill_kind'), 'pin', d['config']['traceback_pin']['matches_oracle'], 'cost', d['config'].get('cost_matches_oracle'))
"
}
run c3 td4 GA_LANE_COLS_PER_LANE=4 || exit 1
run c3 td2 GA_LANE_COLS_PER_LANE=2 || exit 1
run c5 rc8 GA_RC=1 GA_LANE_COLS_PER_LANE=8 || exit 1
run c5 rc4 GA_RC=1 GA_LANE_COLS_PER_LANE=4 || exit 1
run c2 default GA_X=0 || exit 1
run c2 rc2 GA_RC=1 GA_LANE_COLS_PER_LANE=2 || exit 1
run c2 rc4 GA_RC=1 GA_LANE_COLS_PER_LANE=4 || exit 1
