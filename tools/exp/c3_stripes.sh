# C3/C5 pipelined bench under stripe-width / waves-per-workgroup overrides (DESIGN.md 5.2 choice of T)
set -o pipefail
mkdir -p gpurun_out/exp
for W in c3 c5; do
  for cfg in "1 0" "2 0" "2 4" "2 8" "1 4"; do
    set -- $cfg
    export GA_COLS_PER_LANE=$1 GA_FILL_NWC=$2
    timeout -k 10 200 python -u bench.py --workload $W --steps 20 --warmup 5 --no-cpu-baseline --no-extra > gpurun_out/exp/st_${W}_T$1_N$2.json 2> gpurun_out/exp/st_${W}_T$1_N$2.err || { tail -20 gpurun_out/exp/st_${W}_T$1_N$2.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/exp/st_${W}_T$1_N$2.json'));print('$W T=$1 nwc=$2', round(d['ms_per_step'],3), 'fill', round(d['fill_ms'],2), 'walk', round(d['walk_ms'],2), 'lat', round(d['latency_ms_per_alignment'],2), d['config']['traceback_pin']['matches_oracle'])"
  done
done
