set -o pipefail
# round 5: where C5's single call goes -- lane stamps of the C5-shape score fill (protein, TD 4) against the same shape
# in DNA, and the recompute walk's accounting at C5
O=gpurun_out/r5_c5
mkdir -p $O
export GA_FILL_MODE=lane GA_LANE_COLS_PER_LANE=4
timeout -k 10 120 python -u tools/lane_stamps.py 20000 20000 c5 > $O/stamps_c5.json 2> $O/stamps_c5.err || { tail -5 $O/stamps_c5.err; exit 1; }
timeout -k 10 120 python -u tools/lane_stamps.py 20000 20000 > $O/stamps_dna20k.json 2> $O/stamps_dna20k.err || { tail -5 $O/stamps_dna20k.err; exit 1; }
for w in c5 dna20k; do python3 -c "
import json
d=json.loads(open('$O/stamps_$w.json').read().strip().splitlines()[-1])
ld=d['lag_distribution']
print('$w', 'plain', round(d['fill_ms_plain'],3), 'dbg', round(d['fill_ms_dbg'],3), 'intra', d['end_lag_intra_wg_us'], 'cross', d['end_lag_cross_wg_us'], 'sum', {k: round(x,3) for k,x in ld['end_lag_sum_ms'].items()}, 'busy', [round(x['cyc_per_step_busy'],1) for x in d['by_simd'].values()], 'waits', [(round(x['wait_edge_frac'],3), round(x['wait_prof_frac'],3)) for x in d['by_simd'].values()])
"; done
unset GA_FILL_MODE GA_LANE_COLS_PER_LANE
RC_WL=c5 timeout -k 10 200 python -u tools/exp/r5/rc_diag.py 20000 64:64 96:64 128:64 > $O/rc_diag_c5.txt 2>&1 || { tail -5 $O/rc_diag_c5.txt; exit 1; }
cat $O/rc_diag_c5.txt
