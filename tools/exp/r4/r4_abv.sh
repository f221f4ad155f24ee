set -o pipefail
# round 4: lane-fill build variants (GA_LIB_PATH) A/B: lane stamps busy cycles (C3 shape) and the C3 bench line
O=gpurun_out/r4_abv
mkdir -p $O
for v in cur nocons nocons_oldck; do
  GA_LIB_PATH=$PWD/_ab/$v.so GA_FILL_MODE=lane timeout -k 10 120 python -u tools/lane_stamps.py 100000 100000 > $O/stamps_c3_$v.json 2> $O/stamps_c3_$v.err || { tail -5 $O/stamps_c3_$v.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('$O/stamps_c3_$v.json').read().strip().splitlines()[-1])
print('$v', 'plain', round(d['fill_ms_plain'],2), 'dbg', round(d['fill_ms_dbg'],2), 'mean lag', round(d['end_lag_mean_us'],2), 'busy', [round(x['cyc_per_step_busy'],1) for x in d['by_simd'].values()])
"
  GA_LIB_PATH=$PWD/_ab/$v.so timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extra > $O/c3_$v.json 2> $O/c3_$v.err || { tail -5 $O/c3_$v.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('$O/c3_$v.json').read().strip().splitlines()[-1])
print('$v c3 call', round(d['ms_per_step'],3), 'fill', round(d['fill_ms'],3), 'walk', round(d['walk_ms'],3), 'pin', d['config']['traceback_pin']['matches_oracle'])
"
done
