set -o pipefail
# round 4: hand-off poll window (GA_LANE_POLLWIN: 0 adaptive 16 / 192, else fixed): lane stamps (C3 shape, 1M x 125k)
# and the C3 bench line
O=gpurun_out/r4_poll
mkdir -p $O
for v in 0 64 192; do
  GA_LANE_POLLWIN=$v GA_FILL_MODE=lane timeout -k 10 120 python -u tools/lane_stamps.py 100000 100000 > $O/stamps_c3_$v.json 2> $O/stamps_c3_$v.err || { tail -5 $O/stamps_c3_$v.err; exit 1; }
  GA_LANE_POLLWIN=$v GA_FILL_MODE=lane timeout -k 10 120 python -u tools/lane_stamps.py 1000000 125000 > $O/stamps_slab_$v.json 2> $O/stamps_slab_$v.err || { tail -5 $O/stamps_slab_$v.err; exit 1; }
  for w in c3 slab; do python3 -c "
import json
d=json.loads(open('$O/stamps_${w}_$v.json').read().strip().splitlines()[-1])
ld=d['lag_distribution']
print('$v $w', 'plain', round(d['fill_ms_plain'],2), 'dbg', round(d['fill_ms_dbg'],2), 'intra', d['end_lag_intra_wg_us'], 'cross', d['end_lag_cross_wg_us'], 'mean', round(d['end_lag_mean_us'],2), 'sum', {k: round(x,2) for k,x in ld['end_lag_sum_ms'].items()}, 'busy', [round(x['cyc_per_step_busy'],1) for x in d['by_simd'].values()][0], 'probe', json.dumps(d['probe_m2'].get('cross_parts_mean_us')))
"; done
  GA_LANE_POLLWIN=$v timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extra > $O/c3_$v.json 2> $O/c3_$v.err || { tail -5 $O/c3_$v.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('$O/c3_$v.json').read().strip().splitlines()[-1])
print('$v c3 call', round(d['ms_per_step'],3), 'fill', round(d['fill_ms'],3), 'walk', round(d['walk_ms'],3), 'pin', d['config']['traceback_pin']['matches_oracle'])
"
done
