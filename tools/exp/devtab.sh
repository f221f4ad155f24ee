# round 2: device-resident tie-break stream for pipelined walks: pipeline parity, C2 / C5 / C3 bench lines
set -o pipefail
mkdir -p gpurun_out/exp
timeout -k 10 400 python -u -m pytest tests/test_gpu_many.py -x -q --timeout 240 --timeout-method thread > gpurun_out/exp/devtab.log 2>&1 || { tail -30 gpurun_out/exp/devtab.log; exit 1; }
tail -1 gpurun_out/exp/devtab.log
for W in c2 c5 c3; do
  timeout -k 10 200 python -u bench.py --workload $W --no-cpu-baseline --no-extra > gpurun_out/exp/dt_$W.json 2> gpurun_out/exp/dt_$W.err || { tail -20 gpurun_out/exp/dt_$W.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/exp/dt_$W.json'));print('$W', round(d['ms_per_step'],3), 'fill', round(d['fill_ms'],2), 'walk', round(d['walk_ms'],3), d['config']['traceback_pin']['matches_oracle'])"
done
