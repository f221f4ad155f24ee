# pipelined C3 / C5 with two fills co-resident per CU (LDS floor below 80 KB), lane and row-scan traceback fills
set -o pipefail
mkdir -p gpurun_out/exp
run() {  # tag env...
  tag=$1; shift
  env "$@" timeout -k 10 200 python -u bench.py --workload $W --steps 20 --warmup 5 --no-cpu-baseline --no-extra > gpurun_out/exp/lb2_${W}_$tag.json 2> gpurun_out/exp/lb2_${W}_$tag.err || { tail -20 gpurun_out/exp/lb2_${W}_$tag.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/exp/lb2_${W}_$tag.json'));print('$W $tag', round(d['ms_per_step'],3), 'fill', round(d['fill_ms'],2), 'walk', round(d['walk_ms'],2), 'rng', round(d['host_tiebreak_ms'],2), 'lat', round(d['latency_ms_per_alignment'],2), d['config']['traceback_pin']['matches_oracle'])"
}
for W in c3 c5; do
  run row_default GA_FILL_MODE=row
  run row_floor0 GA_FILL_MODE=row GA_FILL_LDS_FLOOR=0
  run lane2_floor0 GA_FILL_MODE=lane GA_LANE_COLS_PER_LANE=2 GA_FILL_NWC=4 GA_FILL_LDS_FLOOR=0 GA_LANE_QROWS=2048
  run lane1_floor0 GA_FILL_MODE=lane GA_LANE_COLS_PER_LANE=1 GA_FILL_NWC=8 GA_FILL_LDS_FLOOR=0 GA_LANE_QROWS=1024
  run lane2n8_floor0 GA_FILL_MODE=lane GA_LANE_COLS_PER_LANE=2 GA_FILL_NWC=8 GA_FILL_LDS_FLOOR=0 GA_LANE_QROWS=1024
done
