# round 2: walk chain on / off, repeated: C3 (lane fills) twice, C5 and C2 (row-scan fills)
set -o pipefail
mkdir -p gpurun_out/exp
for W in ${WLS:-c3 c5 c2 c3}; do
  for CH in 1 0; do
    GA_PIPE_CHAIN=$CH timeout -k 10 200 python -u bench.py --workload $W --no-cpu-baseline --no-extra > gpurun_out/exp/ab_${W}_$CH.json 2> gpurun_out/exp/ab_${W}_$CH.err || { tail -20 gpurun_out/exp/ab_${W}_$CH.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/exp/ab_${W}_$CH.json'));print('$W chain=$CH', round(d['ms_per_step'],3), 'fill', round(d['fill_ms'],2), 'walk', round(d['walk_ms'],3), d['config']['cost_matches_oracle'], d['config']['traceback_pin']['matches_oracle'])"
  done
done
