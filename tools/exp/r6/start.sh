set -o pipefail
# round 6, first look: lane stamps with the first edge wait (the ramp) split from the steady state's waits, at the C3
# shape (TD 4, the recompute fill's geometry) and the C5 shape (TD 4 / TD 2); the C5 single call at TD 4 / TD 2;
# the default line
export TMPDIR=/tmp
O=gpurun_out/r6_start
mkdir -p $O
st() {
  name=$1; shift
  env GA_FILL_MODE=lane "$@" timeout -k 10 120 python -u tools/lane_stamps.py $SHAPE > $O/stamps_$name.json 2> $O/stamps_$name.err || { tail -5 $O/stamps_$name.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('$O/stamps_$name.json').read().strip().splitlines()[-1])
s=d['steady_state']
print('$name', 'plain', round(d['fill_ms_plain'],3), 'intra', round(d['end_lag_intra_wg_us'],2), 'cross', round(d['end_lag_cross_wg_us'],2), 'cyc/step', round(d['cycles_per_step_median'],1), 'after-first', round(s['cyc_per_step_after_first_edge_median'],1), 'steady wait', round(s['wait_edge_steady_frac_median'],4), 'first', round(s['wait_edge_first_frac_median'],4))
print('   steady wait by decile', [round(x,4) for x in s['wait_edge_steady_frac_by_decile']])
print('   ns/step after first edge by decile', [round(x,1) for x in s['ns_per_step_after_first_edge_by_decile']])
"
}
SHAPE="100000 100000" st c3td4 GA_LANE_COLS_PER_LANE=4
SHAPE="20000 20000 c5" st c5td4 GA_LANE_COLS_PER_LANE=4
SHAPE="20000 20000 c5" st c5td2 GA_LANE_COLS_PER_LANE=2
for td in 4 2; do
  GA_LANE_COLS_PER_LANE=$td timeout -k 10 200 python -u bench.py --workload c5 --steps 20 --warmup 5 --no-cpu-baseline --no-extra > $O/bench_c5_td$td.json 2> $O/bench_c5_td$td.err || { tail -20 $O/bench_c5_td$td.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('$O/bench_c5_td$td.json').read().strip().splitlines()[-1])
print('c5 td$td', round(d['ms_per_step'],3), 'fill', round(d['fill_ms'],3), 'walk', round(d['walk_ms'],3), d['fill_kind'], d['config'].get('traceback_pin',{}).get('matches_oracle'))
"
done
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
python3 -c "
import json
d=json.loads(open('$O/bench_default.json').read().strip().splitlines()[-1])
print('c3', round(d['ms_per_step'],3), 'fill', round(d['fill_ms'],3), 'walk', round(d['walk_ms'],3), 'tiebreak', round(d['host_tiebreak_ms'],3), d['config']['traceback_pin']['matches_oracle'], 'c4', round(d['c4']['fill_ms'],2))
"
