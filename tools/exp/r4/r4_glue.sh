set -o pipefail
# round 4: exec-free checkpoint stores in the lean sub-chunk, the compiler path's reads landed in-path, the row-m/2
# probe; lane / rc tests, probe stamps (C3 shape, 1M x 125k slab), the C3 bench line
O=gpurun_out/r4_glue
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_lane.py tests/test_gpu_rc.py -m gpu > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash tools/exp/r4/r4_probe.sh || exit 1
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/c3.json 2> $O/c3.err || { tail -5 $O/c3.err; exit 1; }
python3 -c "
import json
d=json.loads(open('$O/c3.json').read().strip().splitlines()[-1])
print('c3 call', round(d['ms_per_step'],3), 'fill', round(d['fill_ms'],3), 'walk', round(d['walk_ms'],3), 'pin', d['config']['traceback_pin']['matches_oracle'], 'C4', round(d['c4']['fill_ms'],2), d['c4']['cost_matches_oracle'])
"
