set -o pipefail
# round 6: the colck offset as one v_add (no 64-bit mad per sub-chunk); C3 at 2 columns per lane with the lean ramp
# (782 stripes: a shorter step, twice the lags; the walk's blocks narrower), with 64 and 96 recompute workers
export TMPDIR=/tmp
O=gpurun_out/r6_check5
mkdir -p $O
b() {
  name=$1; w=$2; shift 2
  env "$@" timeout -k 10 200 python -u bench.py --workload $w --steps 20 --warmup 5 --no-cpu-baseline --no-extra > $O/bench_$name.json 2> $O/bench_$name.err || { tail -20 $O/bench_$name.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('$O/bench_$name.json').read().strip().splitlines()[-1])
print('$name', round(d['ms_per_step'],3), 'fill', round(d['fill_ms'],3), 'walk', round(d['walk_ms'],3), 'tiebreak', round(d.get('host_tiebreak_ms',0),3), d.get('fill_kind'), (d['config'].get('traceback_pin') or {}).get('matches_oracle'), 'frac', d['roofline'].get('frac'))
"
}
b c3 c3 X=1
b c3td2 c3 GA_LANE_COLS_PER_LANE=2
b c3td2s96 c3 GA_LANE_COLS_PER_LANE=2 GA_RC_SERVERS=96
b c3b c3 X=1
b c5 c5 X=1
b c2 c2 X=1
b c2td2 c2 GA_LANE_COLS_PER_LANE=2
