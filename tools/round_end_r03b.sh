# Round 3 (second session) round-end evidence on the final tree: the whole GPU suite and smoke, the default bench
# line (C3 one call per step, with C4, pipelined and CPU legs), C5 / C2 lines, rocprofv3 kernel stats of the default line
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03b
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/gpu_suite.txt 2>&1 || { tail -40 $O/gpu_suite.txt; exit 1; }
tail -2 $O/gpu_suite.txt
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" >> $O/gpu_suite.txt 2>&1 || { tail -5 $O/gpu_suite.txt; exit 1; }
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
timeout -k 10 400 python -u bench.py --workload c4tb --no-cpu-baseline --no-extra --steps 3 --warmup 1 > $O/bench_c4tb.json 2> $O/bench_c4tb.err || { tail -20 $O/bench_c4tb.err; exit 1; }
for W in c5 c2; do
  timeout -k 10 200 python -u bench.py --workload $W --no-cpu-baseline --no-extra --steps 20 --warmup 5 > $O/bench_$W.json 2> $O/bench_$W.err || { tail -20 $O/bench_$W.err; exit 1; }
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats_default -o run -- python3 bench.py --no-cpu-baseline --no-extra --steps 20 --warmup 5 > $O/stats_default.log 2>&1 || { tail -20 $O/stats_default.log; exit 1; }
find $O -name "*kernel_stats.csv" | head -3
