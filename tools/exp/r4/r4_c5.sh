set -o pipefail
# round 4: C5's single call through the lane fill (stored words / recompute walk) at 1 and 2 columns per lane, against
# the default row scan; lane stamps of the C5 shape
O=gpurun_out/r4_c5
mkdir -p $O
run() {
  local tag=$1; shift
  env "$@" timeout -k 10 200 python -u bench.py --workload c5 --steps 20 --warmup 5 --no-cpu-baseline > $O/c5_$tag.json 2> $O/c5_$tag.err || { tail -5 $O/c5_$tag.err; return 1; }
  python3 -c "
import json
d=json.loads(open('$O/c5_$tag.json').read().strip().splitlines()[-1])
print('$tag', 'call', round(d['ms_per_step'],3), 'fill', round(d['fill_ms'],3), 'walk', round(d['walk_ms'],3), d.get('fill_kind'), 'pin', d['config']['traceback_pin']['matches_oracle'], 'cost', d['config'].get('cost_matches_oracle'))
"
}
run default GA_X=0 || exit 1
run lane1 GA_FILL_MODE=lane GA_LANE_COLS_PER_LANE=1 || exit 1
run lane2 GA_FILL_MODE=lane GA_LANE_COLS_PER_LANE=2 || exit 1
run rc2 GA_RC=1 GA_LANE_COLS_PER_LANE=2 || exit 1
run rc4 GA_RC=1 GA_LANE_COLS_PER_LANE=4 || exit 1
for td in 1 2 4; do
  GA_LANE_COLS_PER_LANE=$td GA_FILL_MODE=lane timeout -k 10 120 python -u tools/lane_stamps.py 20000 20000 c5 > $O/stamps_td$td.json 2> $O/stamps_td$td.err || { tail -5 $O/stamps_td$td.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('$O/stamps_td$td.json').read().strip().splitlines()[-1])
print('td$td', 'stripes', d['nstripes'], 'plain', round(d['fill_ms_plain'],2), 'dbg', round(d['fill_ms_dbg'],2), 'intra', d['end_lag_intra_wg_us'], 'cross', d['end_lag_cross_wg_us'], 'mean', round(d['end_lag_mean_us'],2), 'busy', [round(x['cyc_per_step_busy'],1) for x in d['by_simd'].values()][0], 'waits', [round(x['wait_prof_frac'],3) for x in d['by_simd'].values()][0])
"
done
