# round 2: walks take the pending slot whose fill ended first (default) / slot k % S (GA_PIPE_SLOT_ORDER=fixed):
# pipeline parity, then C3 twice each way
set -o pipefail
mkdir -p gpurun_out/exp
timeout -k 10 200 python -u -m pytest tests/test_gpu_many.py -x -q --timeout 120 --timeout-method thread > gpurun_out/exp/so_tests.log 2>&1 || { tail -30 gpurun_out/exp/so_tests.log; exit 1; }
tail -1 gpurun_out/exp/so_tests.log
for R in 1 2; do
  for O in any fixed; do
    GA_PIPE_SLOT_ORDER=$O timeout -k 10 200 python -u bench.py --workload c3 --no-cpu-baseline --no-extra > gpurun_out/exp/so_${O}_$R.json 2> gpurun_out/exp/so_${O}_$R.err || { tail -20 gpurun_out/exp/so_${O}_$R.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/exp/so_${O}_$R.json'));print('c3 $O', round(d['ms_per_step'],3), 'fill', round(d['fill_ms'],2), 'walk', round(d['walk_ms'],3), d['config']['cost_matches_oracle'], d['config']['traceback_pin']['matches_oracle'])"
  done
done
