set -o pipefail
# round 5: cache slot owner tags -- rc GPU tests (incl. the lost-tag repair test) and the C3 / C2 calls
O=gpurun_out/r5_tags
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_rc.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
for w in c3 c2 c3 c5; do
  timeout -k 10 300 python -u bench.py --workload $w --steps 20 --warmup 5 --no-cpu-baseline --no-extra > $O/bench_$w.json 2> $O/bench_$w.err || { tail -20 $O/bench_$w.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('$O/bench_$w.json').read().strip().splitlines()[-1])
print('$w', 'ms/step', round(d['ms_per_step'],3), 'fill', round(d.get('fill_ms',0),3), 'walk', round(d.get('walk_ms',0),3), 'pin', (d['config'].get('traceback_pin') or {}).get('matches_oracle'))
"
done
bash tools/exp/r5/rc_every.sh
