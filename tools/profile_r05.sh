set -o pipefail
# round 5: the roofline inputs of every bench line from THIS tree, refreshed after the round-5 fill changes: for each workload (c3, c4, c5,
# c2) one FETCH_SIZE, one WRITE_SIZE and one SQ pass (each its own run, rocprofv3 --pmc with --kernel-trace only)
# over one bench call, and the kernel stats of the default bench line; summarised into profiles/r05/ by
# tools/pmc_traffic.py / tools/pmc_valu.py (the largest fill dispatch of each run)
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/prof_r05
mkdir -p $O
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats_default -o run -- python3 $R/bench.py --no-cpu-baseline --no-extra --steps 20 --warmup 5 > $O/stats_default.log 2>&1 || { tail -20 $O/stats_default.log; exit 1; }
tail -1 $O/stats_default.log
for w in c3 c4 c5 c2; do
  timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/fetch_$w -o run -- python3 $R/bench.py --workload $w --no-cpu-baseline --no-extra --steps 1 --warmup 1 > $O/fetch_$w.log 2>&1 || { tail -20 $O/fetch_$w.log; exit 1; }
  timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/write_$w -o run -- python3 $R/bench.py --workload $w --no-cpu-baseline --no-extra --steps 1 --warmup 1 > $O/write_$w.log 2>&1 || { tail -20 $O/write_$w.log; exit 1; }
  timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU --kernel-trace --output-format csv -d $O/sq_$w -o run -- python3 $R/bench.py --workload $w --no-cpu-baseline --no-extra --steps 1 --warmup 1 > $O/sq_$w.log 2>&1 || { tail -20 $O/sq_$w.log; exit 1; }
  echo "$w done"
done
cd $R
for w in c3 c4 c5 c2; do
  f=$(find $O/fetch_$w -name "*counter_collection.csv" | head -1)
  wr=$(find $O/write_$w -name "*counter_collection.csv" | head -1)
  sq=$(find $O/sq_$w -name "*counter_collection.csv" | head -1)
  python3 tools/pmc_traffic.py $f $wr profiles/r05/traffic_$w.json "rocprofv3 FETCH_SIZE / WRITE_SIZE passes of one bench.py --workload $w call (tools/profile_r05.sh)" > /dev/null || exit 1
  python3 tools/pmc_valu.py $sq profiles/r05/valu_$w.json "rocprofv3 SQ pass of one bench.py --workload $w call (tools/profile_r05.sh)" > /dev/null || exit 1
done
cp $(find $O/stats_default -name "*kernel_stats.csv" | head -1) profiles/r05/rocprof_default_kernel_stats.csv
mkdir -p gpurun_out/prof_r05_out && cp profiles/r05/traffic_*.json profiles/r05/valu_*.json profiles/r05/rocprof_default_kernel_stats.csv gpurun_out/prof_r05_out/
head -4 profiles/r05/rocprof_default_kernel_stats.csv
