set -o pipefail
# round 4: the row-m/2 probe of the lane stamps (publish -> out-path store -> IO wave landing -> consumer), C3 shape
# and the 1M x 125k slab, out wave on / off
O=gpurun_out/r4_probe
mkdir -p $O
for v in 1 0; do
  GA_LANE_OUTWAVE=$v GA_FILL_MODE=lane timeout -k 10 120 python -u tools/lane_stamps.py 100000 100000 > $O/stamps_c3_$v.json 2> $O/stamps_c3_$v.err || { tail -5 $O/stamps_c3_$v.err; exit 1; }
  GA_LANE_OUTWAVE=$v GA_FILL_MODE=lane timeout -k 10 120 python -u tools/lane_stamps.py 1000000 125000 > $O/stamps_slab_$v.json 2> $O/stamps_slab_$v.err || { tail -5 $O/stamps_slab_$v.err; exit 1; }
done
for f in $O/stamps_*.json; do echo $f; python3 -c "
import json,sys
d=json.loads(open('$f').read().strip().splitlines()[-1])
print(d['fill_ms_dbg'], d['end_lag_intra_wg_us'], d['end_lag_cross_wg_us'], json.dumps(d['probe_m2']))
"; done
