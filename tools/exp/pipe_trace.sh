# round 2: timeline of the pipelined C3 / C5 steps (GA_PIPE_TRACE) under fill-placement variants
set -o pipefail
mkdir -p gpurun_out/exp
run() {  # tag workload env...
  tag=$1; W=$2; shift 2
  rm -f gpurun_out/exp/trace_${W}_$tag.jsonl
  env GA_PIPE_TRACE=gpurun_out/exp/trace_${W}_$tag.jsonl "$@" timeout -k 10 200 python -u bench.py --workload $W --steps 20 --warmup 0 --no-cpu-baseline --no-extra > gpurun_out/exp/pt_${W}_$tag.json 2> gpurun_out/exp/pt_${W}_$tag.err || { tail -20 gpurun_out/exp/pt_${W}_$tag.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/exp/pt_${W}_$tag.json'));print('$W $tag', round(d['ms_per_step'],3), 'fill', round(d['fill_ms'],2), 'walk', round(d['walk_ms'],2), 'rng', round(d['host_tiebreak_ms'],2), d['config']['traceback_pin']['matches_oracle'])"
}
run row c3
run floor0 c3 GA_FILL_LDS_FLOOR=0
run fills3 c3 GA_PIPE_FILLS=3
run lane2 c3 GA_FILL_MODE=lane GA_LANE_COLS_PER_LANE=2 GA_FILL_NWC=4 GA_FILL_LDS_FLOOR=0 GA_LANE_QROWS=2048
run row c5
