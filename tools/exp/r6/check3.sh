set -o pipefail
# round 6: call-overhead trims (pinned walk results, the fill's result words copied beside the walk, the walk's
# position words cleared before the fill, the spread boundary kernels from 4k codes), sequential tie-break table again:
# GPU suite, C3 / C5 / C2 lines, C5 kernel trace; then the 8-rank rehearsal
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6_check3
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_suite.txt 2>&1 || { tail -40 $O/gpu_suite.txt; exit 1; }
tail -1 $O/gpu_suite.txt
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
python3 -c "
import json
d=json.loads(open('$O/bench_default.json').read().strip().splitlines()[-1])
print('c3', round(d['ms_per_step'],3), 'fill', round(d['fill_ms'],3), 'walk', round(d['walk_ms'],3), 'tiebreak', round(d['host_tiebreak_ms'],3), d['config']['traceback_pin']['matches_oracle'], '| c4', round(d['c4']['fill_ms'],2), d['c4']['cost_matches_oracle'])
"
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
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/trace_c3 -o run -- python3 $R/bench.py --workload c3 --no-cpu-baseline --no-extra --steps 3 --warmup 1 > $O/trace_c3.log 2>&1 || { tail -20 $O/trace_c3.log; exit 1; }
cp $(find $O/trace_c3 -name "*kernel_trace.csv" | head -1) $O/c3_kernel_trace.csv
cd $R
bash tools/exp/r6/dist8.sh || exit 1
