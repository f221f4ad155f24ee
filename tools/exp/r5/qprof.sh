set -o pipefail
# round 5: the lane fill's query profile precomputed in HBM (launch_lane_qprof) against the profile wave building it
# (GA_LANE_QPROF_WAVE=1): lane / rc GPU tests, C5 stamps (chain head), then C5 / C3 / C2 single calls and C4
O=gpurun_out/r5_qprof
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_lane.py tests/test_gpu_rc.py tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
GA_FILL_MODE=lane GA_LANE_COLS_PER_LANE=4 LANE_STAMPS_DUMP=$O/raw_c5.npy timeout -k 10 120 python -u tools/lane_stamps.py 20000 20000 c5 > $O/stamps_c5.json 2> $O/stamps_c5.err || { tail -5 $O/stamps_c5.err; exit 1; }
python3 - <<'PY'
import numpy as np, json
st = np.load("gpurun_out/r5_qprof/raw_c5.npy").astype(np.int64)
t0 = st[:, 0].min(); tot = np.maximum(st[:, 5], 1)
for s in (0, 1, 40, 78):
    print("c5 stripe", s, "dur_us", round((st[s, 1] - st[s, 0]) / 100.0, 1), "wait edge/prof/space", [round(x, 3) for x in (st[s, 2] / tot[s], st[s, 3] / tot[s], st[s, 4] / tot[s])])
d = json.loads(open("gpurun_out/r5_qprof/stamps_c5.json").read().strip().splitlines()[-1])
print("c5 fill dbg", round(d["fill_ms_dbg"], 3))
PY
for v in 0 1; do
  for w in c5 c3 c2; do
    if [ $v = 1 ]; then export GA_LANE_QPROF_WAVE=1; else unset GA_LANE_QPROF_WAVE; fi
    timeout -k 10 300 python -u bench.py --workload $w --steps 20 --warmup 5 --no-cpu-baseline --no-extra > $O/bench_${w}_$v.json 2> $O/bench_${w}_$v.err || { tail -20 $O/bench_${w}_$v.err; exit 1; }
    python3 -c "
import json
d=json.loads(open('$O/bench_${w}_$v.json').read().strip().splitlines()[-1])
print('qprof_wave=$v $w', 'ms/step', round(d['ms_per_step'],3), 'fill', round(d.get('fill_ms',0),3), 'walk', round(d.get('walk_ms',0),3), 'pin', (d['config'].get('traceback_pin') or {}).get('matches_oracle'), 'cost', d['config'].get('cost_matches_oracle'))
"
  done
done
unset GA_LANE_QPROF_WAVE
timeout -k 10 200 python -u bench.py --workload c4 --steps 3 --warmup 1 --no-cpu-baseline --no-extra > $O/bench_c4.json 2> $O/bench_c4.err || { tail -20 $O/bench_c4.err; exit 1; }
python3 -c "
import json
d=json.loads(open('$O/bench_c4.json').read().strip().splitlines()[-1])
print('c4 fill', round(d['fill_ms'],2), 'cost', d['config'].get('cost_matches_oracle'))
"
