set -o pipefail
# round 6: the recompute window's cone at 2 and 4 columns per lane (C3 accounting), and C5 / C2 calls with it
export TMPDIR=/tmp
O=gpurun_out/r6_check6
mkdir -p $O
timeout -k 10 300 python -u tools/exp/r6/rc_diag.py 100000 GA_LANE_COLS_PER_LANE=2,GA_RC_CONE=2 GA_LANE_COLS_PER_LANE=2,GA_RC_CONE=3 GA_LANE_COLS_PER_LANE=2,GA_RC_CONE=4 GA_LANE_COLS_PER_LANE=4,GA_RC_CONE=2 GA_LANE_COLS_PER_LANE=4,GA_RC_CONE=3 GA_LANE_COLS_PER_LANE=2,GA_RC_CONE=2,GA_RC_SERVERS=80 > $O/rc_diag_cone.txt 2>&1 || { tail -5 $O/rc_diag_cone.txt; exit 1; }
b() {
  name=$1; w=$2; shift 2
  timeout -k 10 200 python -u bench.py --workload $w --steps 20 --warmup 5 --no-cpu-baseline --no-extra "$@" > $O/bench_$name.json 2> $O/bench_$name.err || { tail -20 $O/bench_$name.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('$O/bench_$name.json').read().strip().splitlines()[-1])
print('$name', round(d['ms_per_step'],3), 'fill', round(d['fill_ms'],3), 'walk', round(d['walk_ms'],3), 'tiebreak', round(d.get('host_tiebreak_ms',0),3), d.get('fill_kind'), (d['config'].get('traceback_pin') or {}).get('matches_oracle'))
"
}
b c5 c5
b c5cone2 c5 --opt GA_RC_CONE=2
b c5td2cone2 c5 --opt GA_RC_CONE=2 --opt GA_LANE_COLS_PER_LANE=2
b c2td2cone2 c2 --opt GA_RC_CONE=2 --opt GA_LANE_COLS_PER_LANE=2
b c2cone2 c2 --opt GA_RC_CONE=2
b c3td2cone2 c3 --opt GA_RC_CONE=2 --opt GA_LANE_COLS_PER_LANE=2
