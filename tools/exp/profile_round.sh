# rocprofv3 kernel stats + FETCH/WRITE (separate passes) + SQ instruction counters for c4 and c3
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/prof
mkdir -p $O
for W in c4 c3; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats_$W -o run -- python3 bench.py --workload $W --no-cpu-baseline --no-extra --steps 3 --warmup 1 > $O/stats_$W.log 2>&1 || { tail -20 $O/stats_$W.log; exit 1; }
  timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/fetch_$W -o run -- python3 bench.py --workload $W --no-cpu-baseline --no-extra --steps 1 --warmup 0 > $O/fetch_$W.log 2>&1 || { tail -20 $O/fetch_$W.log; exit 1; }
  timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/write_$W -o run -- python3 bench.py --workload $W --no-cpu-baseline --no-extra --steps 1 --warmup 0 > $O/write_$W.log 2>&1 || { tail -20 $O/write_$W.log; exit 1; }
  timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAVES --kernel-trace --output-format csv -d $O/sq_$W -o run -- python3 bench.py --workload $W --no-cpu-baseline --no-extra --steps 1 --warmup 0 > $O/sq_$W.log 2>&1 || { tail -20 $O/sq_$W.log; exit 1; }
done
find $O -name "*.csv" | sort
