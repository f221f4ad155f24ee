# round 2: 16-step sub-chunks for lane-kernel traceback fills (GA_LANE_TB_SUB=16): parity, then C3 pipelined
set -o pipefail
mkdir -p gpurun_out/exp
GA_LANE_TB_SUB=16 timeout -k 10 400 python -u -m pytest tests/test_gpu_lane.py tests/test_gpu_many.py -x -q --timeout 240 --timeout-method thread > gpurun_out/exp/tbsub.log 2>&1 || { tail -30 gpurun_out/exp/tbsub.log; exit 1; }
tail -2 gpurun_out/exp/tbsub.log
run() {  # tag workload env...
  tag=$1; W=$2; shift 2
  rm -f gpurun_out/exp/trace_${W}_$tag.jsonl
  env GA_PIPE_TRACE=gpurun_out/exp/trace_${W}_$tag.jsonl "$@" timeout -k 10 200 python -u bench.py --workload $W --steps 20 --warmup 5 --no-cpu-baseline --no-extra > gpurun_out/exp/ts_${W}_$tag.json 2> gpurun_out/exp/ts_${W}_$tag.err || { tail -20 gpurun_out/exp/ts_${W}_$tag.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/exp/ts_${W}_$tag.json'));print('$W $tag', round(d['ms_per_step'],3), 'fill', round(d['fill_ms'],2), 'walk', round(d['walk_ms'],2), 'lat', round(d['latency_ms_per_alignment'],2), d['config']['traceback_pin']['matches_oracle'])"
}
run sub8 c3
run sub16 c3 GA_LANE_TB_SUB=16
run sub16lat c3 GA_LANE_TB_SUB=16 GA_FILL_MODE=lane GA_LANE_COLS_PER_LANE=4 GA_FILL_NWC=4
