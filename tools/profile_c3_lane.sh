# round 2 (pipelined lane-kernel C3): rocprofv3 kernel stats of the default bench line, then FETCH_SIZE /
# WRITE_SIZE / SQ passes (each its own run) of one C3 lane-kernel traceback fill (fill_lane_kernel<4,4,1,8>),
# and the walk-chain microbenchmark
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/prof3
mkdir -p $O
timeout -k 10 60 ./tools/micro/walk_chain > $O/walk_chain.txt 2>&1 || { cat $O/walk_chain.txt; exit 1; }
cat $O/walk_chain.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats_default -o run -- python3 bench.py --no-cpu-baseline --steps 20 --warmup 5 > $O/stats_default.log 2>&1 || { tail -20 $O/stats_default.log; exit 1; }
export GA_FILL_MODE=lane GA_LANE_COLS_PER_LANE=4 GA_FILL_NWC=4 GA_LANE_QROWS=2048
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/fetch_c3 -o run -- python3 tools/fill_only.py 100000 100000 1 > $O/fetch_c3.log 2>&1 || { tail -20 $O/fetch_c3.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/write_c3 -o run -- python3 tools/fill_only.py 100000 100000 1 > $O/write_c3.log 2>&1 || { tail -20 $O/write_c3.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAVES --kernel-trace --output-format csv -d $O/sq_c3 -o run -- python3 tools/fill_only.py 100000 100000 1 > $O/sq_c3.log 2>&1 || { tail -20 $O/sq_c3.log; exit 1; }
find $O -name "*.csv" | sort
