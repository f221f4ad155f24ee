set -o pipefail
# round 6: Python-side call trims; C5 / C2 at 2 columns per lane against 4 (with the lean ramp); the 8-rank rehearsal
# with the preflight's relink fix
export TMPDIR=/tmp
O=gpurun_out/r6_check4
mkdir -p $O
b() {
  name=$1; w=$2; shift 2
  env "$@" timeout -k 10 200 python -u bench.py --workload $w --steps 20 --warmup 5 --no-cpu-baseline --no-extra > $O/bench_$name.json 2> $O/bench_$name.err || { tail -20 $O/bench_$name.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('$O/bench_$name.json').read().strip().splitlines()[-1])
print('$name', round(d['ms_per_step'],3), 'fill', round(d['fill_ms'],3), 'walk', round(d['walk_ms'],3), 'tiebreak', round(d.get('host_tiebreak_ms',0),3), d.get('fill_kind'), (d['config'].get('traceback_pin') or {}).get('matches_oracle'))
"
}
b c3 c3 X=1
b c5 c5 X=1
b c5td2 c5 GA_LANE_COLS_PER_LANE=2
b c2 c2 X=1
b c2td2 c2 GA_LANE_COLS_PER_LANE=2
bash tools/exp/r6/dist8.sh || exit 1
