# round 2: C5 / C2 with the faster walk: row-scan fills in flight (2 / 3 / 4), eight hardware queues
set -o pipefail
mkdir -p gpurun_out/exp
for W in c5 c2; do
  for F in 2 3 4; do
    GA_PIPE_FILLS=$F timeout -k 10 200 python -u bench.py --workload $W --no-cpu-baseline --no-extra > gpurun_out/exp/p5_${W}_$F.json 2> gpurun_out/exp/p5_${W}_$F.err || { tail -20 gpurun_out/exp/p5_${W}_$F.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/exp/p5_${W}_$F.json'));print('$W F$F', round(d['ms_per_step'],3), 'fill', round(d['fill_ms'],2), 'walk', round(d['walk_ms'],2), d['config']['traceback_pin']['matches_oracle'])"
  done
done
