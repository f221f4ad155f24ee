# STALE: the knobs this script sets were removed from ga_host.cpp in round 4, so it now measures the
# default path; kept only as the record of the measurement DESIGN.md cites.
# round 2: walk chain with fill 0 alone on the chip before the other fills (GA_CHAIN_STAGGER=1) / all at once
set -o pipefail
mkdir -p gpurun_out/exp
for R in 1 2; do
for W in c2 c5; do
  for G in 1 0; do
    GA_CHAIN_STAGGER=$G timeout -k 10 200 python -u bench.py --workload $W --no-cpu-baseline --no-extra > gpurun_out/exp/st_${W}_$G.json 2> gpurun_out/exp/st_${W}_$G.err || { tail -20 gpurun_out/exp/st_${W}_$G.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/exp/st_${W}_$G.json'));print('$W stagger=$G', round(d['ms_per_step'],3), 'fill', round(d['fill_ms'],2), 'walk', round(d['walk_ms'],3), d['config']['cost_matches_oracle'], d['config']['traceback_pin']['matches_oracle'])"
  done
done
done
