# round-end evidence: full GPU suite, the default bench line (C3 pipelined + C4 point + CPU legs), rocprofv3
# kernel stats of it, the C3 lane-kernel traceback fill's and the C4 fill's FETCH/WRITE/SQ passes (each its
# own run), the walk micro-benchmarks
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/gpu_check.log 2>&1 || { tail -40 gpurun_out/gpu_check.log; exit 1; }
tail -1 gpurun_out/gpu_check.log
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/check_bench.json 2> gpurun_out/check_bench.err || { tail -20 gpurun_out/check_bench.err; exit 1; }
for W in c5 c2; do
  timeout -k 10 200 python -u bench.py --workload $W --no-cpu-baseline --no-extra > gpurun_out/check_bench_$W.json 2> gpurun_out/check_bench_$W.err || { tail -20 gpurun_out/check_bench_$W.err; exit 1; }
done
bash tools/profile_c3_lane.sh
O=gpurun_out/prof3
W=c4
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/fetch_$W -o run -- python3 bench.py --workload $W --no-cpu-baseline --no-extra --steps 1 --warmup 0 > $O/fetch_$W.log 2>&1 || { tail -20 $O/fetch_$W.log; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/write_$W -o run -- python3 bench.py --workload $W --no-cpu-baseline --no-extra --steps 1 --warmup 0 > $O/write_$W.log 2>&1 || { tail -20 $O/write_$W.log; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAVES --kernel-trace --output-format csv -d $O/sq_$W -o run -- python3 bench.py --workload $W --no-cpu-baseline --no-extra --steps 1 --warmup 0 > $O/sq_$W.log 2>&1 || { tail -20 $O/sq_$W.log; exit 1; }
timeout -k 10 60 ./tools/micro/walk_next > $O/walk_next.txt 2>&1 || { cat $O/walk_next.txt; exit 1; }
find $O -name "*.csv" | sort
