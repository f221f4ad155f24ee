# round 2: lane-kernel hand-off reader probes one row while its writer is behind: parity, C4 / C3 timing,
# C4 FETCH / WRITE passes
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/hp
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_lane.py -x -q --timeout 240 --timeout-method thread > $O/lane.log 2>&1 || { tail -30 $O/lane.log; exit 1; }
tail -1 $O/lane.log
timeout -k 10 300 python -u bench.py --workload c4 --steps 3 --warmup 1 --no-cpu-baseline > $O/c4.json 2> $O/c4.err || { tail -20 $O/c4.err; exit 1; }
python -c "import json;d=json.load(open('$O/c4.json'));print('c4', round(d['ms_per_step'],2), d['config']['cost_matches_oracle'])"
timeout -k 10 300 python -u bench.py --workload c3 --no-cpu-baseline --no-extra > $O/c3.json 2> $O/c3.err || { tail -20 $O/c3.err; exit 1; }
python -c "import json;d=json.load(open('$O/c3.json'));print('c3', round(d['ms_per_step'],3), d['config']['traceback_pin']['matches_oracle'])"
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/fetch_c4 -o run -- python3 bench.py --workload c4 --no-cpu-baseline --no-extra --steps 1 --warmup 0 > $O/fetch_c4.log 2>&1 || { tail -20 $O/fetch_c4.log; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/write_c4 -o run -- python3 bench.py --workload c4 --no-cpu-baseline --no-extra --steps 1 --warmup 0 > $O/write_c4.log 2>&1 || { tail -20 $O/write_c4.log; exit 1; }
python tools/pmc_traffic.py $O/fetch_c4/run_counter_collection.csv $O/write_c4/run_counter_collection.csv $O/traffic_c4.json x
