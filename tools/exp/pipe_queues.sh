# round 2: more hardware queues per process (GPU_MAX_HW_QUEUES=8): four lane fills in flight on queues of
# their own beside the walk's, with and without two fill workgroups per CU
set -o pipefail
mkdir -p gpurun_out/exp
run() {  # tag workload env...
  tag=$1; W=$2; shift 2
  rm -f gpurun_out/exp/trace_${W}_$tag.jsonl
  env GA_PIPE_TRACE=gpurun_out/exp/trace_${W}_$tag.jsonl "$@" timeout -k 10 200 python -u bench.py --workload $W --steps 20 --warmup 5 --no-cpu-baseline --no-extra > gpurun_out/exp/q_${W}_$tag.json 2> gpurun_out/exp/q_${W}_$tag.err || { tail -20 gpurun_out/exp/q_${W}_$tag.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/exp/q_${W}_$tag.json'));print('$W $tag', round(d['ms_per_step'],3), 'fill', round(d['fill_ms'],2), 'walk', round(d['walk_ms'],2), d['config']['traceback_pin']['matches_oracle'])"
}
run base c3
run q8 c3 GPU_MAX_HW_QUEUES=8
run q8f4 c3 GPU_MAX_HW_QUEUES=8 GA_PIPE_FILLS=4
run q8f4s6 c3 GPU_MAX_HW_QUEUES=8 GA_PIPE_FILLS=4 GA_PIPE_SLOTS=6
run q8f4fl c3 GPU_MAX_HW_QUEUES=8 GA_PIPE_FILLS=4 GA_FILL_LDS_FLOOR=40000
run q8f4s6fl c3 GPU_MAX_HW_QUEUES=8 GA_PIPE_FILLS=4 GA_PIPE_SLOTS=6 GA_FILL_LDS_FLOOR=40000
run q8c5f3 c5 GPU_MAX_HW_QUEUES=8 GA_PIPE_FILLS=3
