# round 2: pipelined C3 with lane-kernel traceback fills: fills in flight x LDS floor x stripe width sweep
set -o pipefail
mkdir -p gpurun_out/exp
run() {  # tag workload env...
  tag=$1; W=$2; shift 2
  rm -f gpurun_out/exp/trace_${W}_$tag.jsonl
  env GA_PIPE_TRACE=gpurun_out/exp/trace_${W}_$tag.jsonl "$@" timeout -k 10 200 python -u bench.py --workload $W --steps 20 --warmup 3 --no-cpu-baseline --no-extra > gpurun_out/exp/pl_${W}_$tag.json 2> gpurun_out/exp/pl_${W}_$tag.err || { tail -20 gpurun_out/exp/pl_${W}_$tag.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/exp/pl_${W}_$tag.json'));print('$W $tag', round(d['ms_per_step'],3), 'fill', round(d['fill_ms'],2), 'walk', round(d['walk_ms'],2), 'lat', round(d['latency_ms_per_alignment'],2), d['config']['traceback_pin']['matches_oracle'])"
}
L="GA_FILL_MODE=lane"
run lt4p2 c3 $L GA_LANE_QROWS=2048 GA_LANE_COLS_PER_LANE=4 GA_FILL_NWC=4
run lt4p3 c3 $L GA_LANE_QROWS=2048 GA_LANE_COLS_PER_LANE=4 GA_FILL_NWC=4 GA_PIPE_FILLS=3
run lt4p4 c3 $L GA_LANE_QROWS=2048 GA_LANE_COLS_PER_LANE=4 GA_FILL_NWC=4 GA_PIPE_FILLS=4
run lt4f40p4 c3 $L GA_LANE_QROWS=2048 GA_LANE_COLS_PER_LANE=4 GA_FILL_NWC=4 GA_FILL_LDS_FLOOR=40000 GA_PIPE_FILLS=4
run lt4f30p4 c3 $L GA_LANE_QROWS=1024 GA_LANE_COLS_PER_LANE=4 GA_FILL_NWC=4 GA_FILL_LDS_FLOOR=30000 GA_PIPE_FILLS=4
run lt4f30p3 c3 $L GA_LANE_QROWS=1024 GA_LANE_COLS_PER_LANE=4 GA_FILL_NWC=4 GA_FILL_LDS_FLOOR=30000 GA_PIPE_FILLS=3
run lt4n8f54p3 c3 $L GA_LANE_QROWS=1024 GA_LANE_COLS_PER_LANE=4 GA_FILL_NWC=8 GA_FILL_LDS_FLOOR=54000 GA_PIPE_FILLS=3
run lt2f30p4 c3 $L GA_LANE_QROWS=1024 GA_LANE_COLS_PER_LANE=2 GA_FILL_NWC=4 GA_FILL_LDS_FLOOR=30000 GA_PIPE_FILLS=4
run rowf30p4 c3 GA_FILL_MODE=row GA_FILL_LDS_FLOOR=30000 GA_PIPE_FILLS=4
