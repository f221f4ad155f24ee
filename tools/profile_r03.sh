# round 3 (recompute walk): rocprofv3 kernel stats of the default bench line (C3 single calls), then
# FETCH_SIZE / WRITE_SIZE / SQ passes (each its own run) of one C3 call (the rc lane fill is its largest
# fill dispatch, walk_rc_kernel the walk)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/prof_r03
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats_default -o run -- python3 bench.py --no-cpu-baseline --no-extra --steps 20 --warmup 5 > $O/stats_default.log 2>&1 || { tail -20 $O/stats_default.log; exit 1; }
tail -1 $O/stats_default.log
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/fetch_c3 -o run -- python3 bench.py --no-cpu-baseline --no-extra --steps 1 --warmup 1 > $O/fetch_c3.log 2>&1 || { tail -20 $O/fetch_c3.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/write_c3 -o run -- python3 bench.py --no-cpu-baseline --no-extra --steps 1 --warmup 1 > $O/write_c3.log 2>&1 || { tail -20 $O/write_c3.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAVES --kernel-trace --output-format csv -d $O/sq_c3 -o run -- python3 bench.py --no-cpu-baseline --no-extra --steps 1 --warmup 1 > $O/sq_c3.log 2>&1 || { tail -20 $O/sq_c3.log; exit 1; }
find $O -name "*.csv" | sort
