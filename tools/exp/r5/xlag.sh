set -o pipefail
# round 5: what sets the C3-shape (TD 4) fill's cross-workgroup lag (17 us median against 6.6 at 1M x 125k, TD 2):
# the hand-off poll window, the out wave, the late edge read -- lane stamps per variant
O=gpurun_out/r5_xlag
mkdir -p $O
run() {
  name=$1; shift
  env GA_FILL_MODE=lane GA_LANE_COLS_PER_LANE=4 "$@" timeout -k 10 120 python -u tools/lane_stamps.py 100000 100000 > $O/stamps_$name.json 2> $O/stamps_$name.err || { tail -5 $O/stamps_$name.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('$O/stamps_$name.json').read().strip().splitlines()[-1])
print('$name', 'plain', round(d['fill_ms_plain'],3), 'dbg', round(d['fill_ms_dbg'],3), 'intra', round(d['end_lag_intra_wg_us'],2), 'cross', round(d['end_lag_cross_wg_us'],2), 'busy', round(d['cycles_per_step_median'],1), d['probe_m2']['cross_parts_us'])
"
}
run base
run pollwin16 GA_LANE_POLLWIN=16
run pollwin64 GA_LANE_POLLWIN=64
run pollwin192 GA_LANE_POLLWIN=192
run outwave0 GA_LANE_OUTWAVE=0
run late0 GA_LANE_LATE=0
run td2 GA_LANE_COLS_PER_LANE=2
