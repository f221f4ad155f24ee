set -o pipefail
# round 5: the final library (rebuilt from the committed source) -- full GPU suite, smoke, the default bench line
O=gpurun_out/r5_check
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_suite.txt 2>&1 || { tail -40 $O/gpu_suite.txt; exit 1; }
tail -1 $O/gpu_suite.txt
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { tail -20 $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
timeout -k 10 300 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
python3 -c "
import json
d=json.loads(open('$O/bench_default.json').read().strip().splitlines()[-1])
print('value', d['value'], 'ms/step', d['ms_per_step'], 'fill', d['fill_ms'], 'walk', d['walk_ms'], 'c4', d['c4']['fill_ms'], 'pin', d['config']['traceback_pin']['matches_oracle'])
"
