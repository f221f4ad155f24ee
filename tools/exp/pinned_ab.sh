# round 2: per-launch pipeline walks: result words and levels in pinned memory (default) / device + hipMemcpy
set -o pipefail
mkdir -p gpurun_out/exp
for R in 1 2 3; do
  for P in 1 0; do
    GA_PIPE_PINNED_IO=$P timeout -k 10 200 python -u bench.py --workload c3 --no-cpu-baseline --no-extra > gpurun_out/exp/pab_${P}_$R.json 2> gpurun_out/exp/pab_${P}_$R.err || { tail -20 gpurun_out/exp/pab_${P}_$R.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/exp/pab_${P}_$R.json'));print('c3 pinned=$P', round(d['ms_per_step'],3), 'fill', round(d['fill_ms'],2), 'walk', round(d['walk_ms'],3), d['config']['cost_matches_oracle'], d['config']['traceback_pin']['matches_oracle'])"
  done
done
