set -o pipefail
# round 4: the sub-chunk machinery micro (one / two waves per SIMD) and the C3 fill at TD 1 with 8 waves per
# workgroup (two compute waves per SIMD) against the default TD 2 / 4 waves
mkdir -p gpurun_out/r4_td1
O=gpurun_out/r4_td1
timeout -k 10 120 ./tools/micro/lane_parts > $O/lane_parts.txt 2>&1 || { cat $O/lane_parts.txt; exit 1; }
for cfg in "2 4" "1 8" "1 4"; do
  set -- $cfg
  GA_LANE_COLS_PER_LANE=$1 GA_FILL_NWC=$2 GA_FILL_MODE=lane timeout -k 10 120 python -u tools/lane_stamps.py 100000 100000 > $O/stamps_td$1_n$2.json 2> $O/stamps_td$1_n$2.err || { tail -5 $O/stamps_td$1_n$2.err; exit 1; }
done
python3 - <<'PY'
import json
O = "gpurun_out/r4_td1"
print(open(f"{O}/lane_parts.txt").read())
for cfg in ("2_n4", "1_n8", "1_n4"):
    d = json.loads(open(f"{O}/stamps_td{cfg}.json").read().strip().splitlines()[-1])
    print(f"td{cfg} stamps c3: kind {d['kind']} TD {d['TD']} nwc {d['nwc']} slabs {d['nslabs']} plain {d['fill_ms_plain']:.2f} dbg {d['fill_ms_dbg']:.2f} intra {d['end_lag_intra_wg_us']:.2f} cross {d['end_lag_cross_wg_us']:.2f} mean {d['end_lag_mean_us']:.2f} cyc/step {d['cycles_per_step_median']:.1f} busy {[round(v['cyc_per_step_busy'],1) for v in d['by_simd'].values()]}")
PY
