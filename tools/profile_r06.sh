set -o pipefail
# round 6: the roofline inputs of every bench line from THIS tree, refreshed after the round-6 fill changes (the lean ramp): for each workload (c3, c4, c5,
# c2) one FETCH_SIZE, one WRITE_SIZE and one SQ pass (each its own run, rocprofv3 --pmc with --kernel-trace only)
# over one bench call, and the kernel stats of the default bench line; summarised into profiles/r06/ by
# tools/pmc_traffic.py / tools/pmc_valu.py (the largest fill dispatch of each run)
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/prof_r06
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
  python3 tools/pmc_traffic.py $f $wr profiles/r06/traffic_$w.json "rocprofv3 FETCH_SIZE / WRITE_SIZE passes of one bench.py --workload $w call (tools/profile_r06.sh)" > /dev/null || exit 1
  python3 tools/pmc_valu.py $sq profiles/r06/valu_$w.json "rocprofv3 SQ pass of one bench.py --workload $w call (tools/profile_r06.sh)" > /dev/null || exit 1
done
cp $(find $O/stats_default -name "*kernel_stats.csv" | head -1) profiles/r06/rocprof_default_kernel_stats.csv
mkdir -p gpurun_out/prof_r06_out && cp profiles/r06/traffic_*.json profiles/r06/valu_*.json profiles/r06/rocprof_default_kernel_stats.csv gpurun_out/prof_r06_out/
head -4 profiles/r06/rocprof_default_kernel_stats.csv
# lane stamps of the final fills: the C3 shape (TD 4) and C4's N = 8 slab shape (1M x 125k, TD 2)
GA_FILL_MODE=lane GA_LANE_COLS_PER_LANE=4 timeout -k 10 120 python -u tools/lane_stamps.py 100000 100000 > gpurun_out/prof_r06_out/stamps_c3td4.json 2> gpurun_out/prof_r06_out/stamps_c3td4.err || exit 1
GA_FILL_MODE=lane GA_LANE_COLS_PER_LANE=2 timeout -k 10 200 python -u tools/lane_stamps.py 1000000 125000 > gpurun_out/prof_r06_out/stamps_slab125k.json 2> gpurun_out/prof_r06_out/stamps_slab125k.err || exit 1
python3 -c "
import json
for f in ('stamps_c3td4', 'stamps_slab125k'):
    d=json.loads(open('gpurun_out/prof_r06_out/'+f+'.json').read().strip().splitlines()[-1])
    s=d['steady_state']
    print(f, 'plain', round(d['fill_ms_plain'],2), 'busy cyc/step', round(s['cyc_per_step_after_first_edge_median'],1), 'ns/step', round(s['ns_per_step_after_first_edge_median'],1), 'lags intra/cross', round(d['end_lag_intra_wg_us'],2), round(d['end_lag_cross_wg_us'],2), 'steady wait', s['wait_edge_steady_frac_median'])
"
