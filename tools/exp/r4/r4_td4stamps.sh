set -o pipefail
# round 4: lane stamps of the C3-shape fill at 4 columns per lane (the recompute fill's width since round 4)
O=gpurun_out/r4_td4
mkdir -p $O
GA_LANE_COLS_PER_LANE=4 GA_FILL_MODE=lane timeout -k 10 120 python -u tools/lane_stamps.py 100000 100000 > $O/stamps_c3_td4.json 2> $O/stamps_c3_td4.err || { tail -5 $O/stamps_c3_td4.err; exit 1; }
python3 -c "
import json
d=json.loads(open('$O/stamps_c3_td4.json').read().strip().splitlines()[-1])
ld=d['lag_distribution']
print('td4 c3', 'plain', round(d['fill_ms_plain'],2), 'dbg', round(d['fill_ms_dbg'],2), 'intra', d['end_lag_intra_wg_us'], 'cross', d['end_lag_cross_wg_us'], 'mean', round(d['end_lag_mean_us'],2), 'sum', {k: round(x,2) for k,x in ld['end_lag_sum_ms'].items()}, 'busy', [round(x['cyc_per_step_busy'],1) for x in d['by_simd'].values()], 'probe', json.dumps(d['probe_m2']))
"
