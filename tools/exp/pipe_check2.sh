# round 2: pipelined tests (all fill modes) + the C3 bench with the lane-fill pipeline default
set -o pipefail
mkdir -p gpurun_out/exp
timeout -k 10 400 python -u -m pytest tests/test_gpu_many.py tests/test_gpu_lane.py -x -q --timeout 240 --timeout-method thread > gpurun_out/exp/many2.log 2>&1 || { tail -30 gpurun_out/exp/many2.log; exit 1; }
tail -2 gpurun_out/exp/many2.log
for W in c3 c5 c2; do
  timeout -k 10 200 python -u bench.py --workload $W --steps 20 --warmup 5 --no-cpu-baseline --no-extra > gpurun_out/exp/pc2_$W.json 2> gpurun_out/exp/pc2_$W.err || { tail -20 gpurun_out/exp/pc2_$W.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/exp/pc2_$W.json'));print('$W', round(d['ms_per_step'],3), 'fill', round(d['fill_ms'],2), 'walk', round(d['walk_ms'],2), 'lat', round(d['latency_ms_per_alignment'],2), d['config']['traceback_pin'])"
done
