set -o pipefail
# round 6: lean ramp everywhere (C4's TD 8 fill too) and the threaded tie-break table with contiguous ranges: the
# table bench, the GPU suite, the default line (C3 + C4), C5 / C2 lines, and a kernel trace of C5 single calls
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6_check2
mkdir -p $O
timeout -k 10 120 ./globalign_amd/_lib/ga_host_selftest bench 200001 > $O/rng_bench.txt 2>&1 || { cat $O/rng_bench.txt; exit 1; }
cat $O/rng_bench.txt
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_suite.txt 2>&1 || { tail -40 $O/gpu_suite.txt; exit 1; }
tail -1 $O/gpu_suite.txt
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
python3 -c "
import json
d=json.loads(open('$O/bench_default.json').read().strip().splitlines()[-1])
print('c3', round(d['ms_per_step'],3), 'fill', round(d['fill_ms'],3), 'walk', round(d['walk_ms'],3), 'tiebreak', round(d['host_tiebreak_ms'],3), d['config']['traceback_pin']['matches_oracle'], '| c4', round(d['c4']['fill_ms'],2), d['c4']['cost_matches_oracle'])
"
for t in 1 4 8; do
  timeout -k 10 200 python -u bench.py --workload c3 --steps 10 --warmup 3 --no-cpu-baseline --no-extra --opt GA_RNG_THREADS=$t > $O/bench_c3_rng$t.json 2> $O/bench_c3_rng$t.err || { tail -20 $O/bench_c3_rng$t.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('$O/bench_c3_rng$t.json').read().strip().splitlines()[-1])
print('c3 rng threads $t', round(d['ms_per_step'],3), 'tiebreak', round(d['host_tiebreak_ms'],3))
"
done
for w in c5 c2; do
  timeout -k 10 200 python -u bench.py --workload $w --steps 20 --warmup 5 --no-cpu-baseline --no-extra > $O/bench_$w.json 2> $O/bench_$w.err || { tail -20 $O/bench_$w.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('$O/bench_$w.json').read().strip().splitlines()[-1])
print('$w', round(d['ms_per_step'],3), 'fill', round(d['fill_ms'],3), 'walk', round(d['walk_ms'],3), 'tiebreak', round(d.get('host_tiebreak_ms',0),3), (d['config'].get('traceback_pin') or {}).get('matches_oracle'))
"
done
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/trace_c5 -o run -- python3 $R/bench.py --workload c5 --no-cpu-baseline --no-extra --steps 5 --warmup 2 > $O/trace_c5.log 2>&1 || { tail -20 $O/trace_c5.log; exit 1; }
cp $(find $O/trace_c5 -name "*kernel_trace.csv" | head -1) $O/c5_kernel_trace.csv
echo trace ok
