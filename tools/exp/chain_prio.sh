# STALE: the knobs this script sets were removed from ga_host.cpp in round 4, so it now measures the
# default path; kept only as the record of the measurement DESIGN.md cites.
# round 2: the walk chain's stream priority (least / normal / greatest) against per-walk launches: C5 / C3
set -o pipefail
mkdir -p gpurun_out/exp
for W in c5 c3; do
  for P in lo normal hi; do
    GA_CHAIN_PRIO=$P timeout -k 10 200 python -u bench.py --workload $W --no-cpu-baseline --no-extra > gpurun_out/exp/cprio_${W}_$P.json 2> gpurun_out/exp/cprio_${W}_$P.err || { tail -20 gpurun_out/exp/cprio_${W}_$P.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/exp/cprio_${W}_$P.json'));print('$W $P', round(d['ms_per_step'],3), 'fill', round(d['fill_ms'],2), 'walk', round(d['walk_ms'],3), d['config']['cost_matches_oracle'], d['config']['traceback_pin']['matches_oracle'])"
  done
  GA_PIPE_CHAIN=0 timeout -k 10 200 python -u bench.py --workload $W --no-cpu-baseline --no-extra > gpurun_out/exp/cprio_${W}_off.json 2> gpurun_out/exp/cprio_${W}_off.err || { tail -20 gpurun_out/exp/cprio_${W}_off.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/exp/cprio_${W}_off.json'));print('$W off', round(d['ms_per_step'],3), 'fill', round(d['fill_ms'],2), 'walk', round(d['walk_ms'],3))"
done
