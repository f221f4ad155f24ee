set -o pipefail
# round 5: chain neighbours on one XCD (GA_LANE_XCD=1, ga_lane.hip lane_slab) against ticket order (0): lane stamps
# of the C3-shape score fill and the 1M x 125k slab, and the C3 bench line (recompute fill) for both
O=gpurun_out/r5_xcd
mkdir -p $O
for v in 1 0; do
  GA_LANE_XCD=$v GA_FILL_MODE=lane timeout -k 10 120 python -u tools/lane_stamps.py 100000 100000 > $O/stamps_c3_$v.json 2> $O/stamps_c3_$v.err || { tail -5 $O/stamps_c3_$v.err; exit 1; }
  GA_LANE_XCD=$v GA_FILL_MODE=lane timeout -k 10 120 python -u tools/lane_stamps.py 1000000 125000 > $O/stamps_slab_$v.json 2> $O/stamps_slab_$v.err || { tail -5 $O/stamps_slab_$v.err; exit 1; }
  for w in c3 slab; do python3 -c "
import json
d=json.loads(open('$O/stamps_${w}_$v.json').read().strip().splitlines()[-1])
ld=d['lag_distribution']
print('$v $w', 'plain', round(d['fill_ms_plain'],2), 'dbg', round(d['fill_ms_dbg'],2), 'intra', d['end_lag_intra_wg_us'], 'cross', d['end_lag_cross_wg_us'], 'mean', round(d['end_lag_mean_us'],2), 'sum', {k: round(x,2) for k,x in ld['end_lag_sum_ms'].items()}, 'links', ld['cross_wg_links'], 'busy', [round(x['cyc_per_step_busy'],1) for x in d['by_simd'].values()])
"; done
  GA_LANE_XCD=$v timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/c3_$v.json 2> $O/c3_$v.err || { tail -5 $O/c3_$v.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('$O/c3_$v.json').read().strip().splitlines()[-1])
print('$v c3 call', round(d['ms_per_step'],3), 'fill', round(d['fill_ms'],3), 'walk', round(d['walk_ms'],3), 'pin', d['config']['traceback_pin']['matches_oracle'], 'C4', round(d['c4']['fill_ms'],2), d['c4']['cost_matches_oracle'])
"
done
