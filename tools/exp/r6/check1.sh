set -o pipefail
# round 6: the knob split (shipped env knobs + context options), the jump walk behind the experiments build, the
# readlane-carry walk tests and the C4 full-traceback pin: GPU suite, then the c4tb bench line with its pin
export TMPDIR=/tmp
O=gpurun_out/r6_check1
mkdir -p $O
bash tools/exp/r6/probe2.sh || exit 1
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_suite.txt 2>&1 || { tail -40 $O/gpu_suite.txt; exit 1; }
tail -1 $O/gpu_suite.txt
timeout -k 10 300 python -u bench.py --workload c4tb --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_c4tb.json 2> $O/bench_c4tb.err || { tail -20 $O/bench_c4tb.err; exit 1; }
python3 -c "
import json
d=json.loads(open('$O/bench_c4tb.json').read().strip().splitlines()[-1])
print('c4tb', round(d['ms_per_step'],1), 'ms', d['config'].get('traceback_pin'), d['config'].get('cost_matches_oracle'))
"
