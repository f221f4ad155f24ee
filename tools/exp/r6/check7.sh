set -o pipefail
# round 6: 2 columns per lane for DNA recompute fills and the cone-3 window as defaults: GPU suite, then the bench lines
export TMPDIR=/tmp
O=gpurun_out/r6_check7
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_suite.txt 2>&1 || { tail -30 $O/gpu_suite.txt; exit 1; }
tail -2 $O/gpu_suite.txt
b() {
  name=$1; w=$2; shift 2
  timeout -k 10 300 python -u bench.py --workload $w --steps 20 --warmup 5 --no-cpu-baseline --no-extra "$@" > $O/bench_$name.json 2> $O/bench_$name.err || { tail -20 $O/bench_$name.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('$O/bench_$name.json').read().strip().splitlines()[-1])
print('$name', round(d['ms_per_step'],3), 'fill', round(d.get('fill_ms') or 0,3), 'walk', round(d.get('walk_ms') or 0,3), 'tiebreak', round(d.get('host_tiebreak_ms') or 0,3), d.get('fill_kind'), (d['config'].get('traceback_pin') or {}).get('matches_oracle'), 'frac', d['roofline'].get('frac'))
"
}
b c3 c3
b c2 c2
b c5 c5
b c4tb c4tb --steps 3 --warmup 1
b c4tbcone1 c4tb --steps 3 --warmup 1 --opt GA_RC_CONE=1
