# round 2: pipeline slots (fill k+S reuses walk k's buffers) x fills in flight x fill-stream priority
set -o pipefail
mkdir -p gpurun_out/exp
run() {  # tag workload env...
  tag=$1; W=$2; shift 2
  rm -f gpurun_out/exp/trace_${W}_$tag.jsonl
  env GA_PIPE_TRACE=gpurun_out/exp/trace_${W}_$tag.jsonl "$@" timeout -k 10 200 python -u bench.py --workload $W --steps 20 --warmup 5 --no-cpu-baseline --no-extra > gpurun_out/exp/sl_${W}_$tag.json 2> gpurun_out/exp/sl_${W}_$tag.err || { tail -20 gpurun_out/exp/sl_${W}_$tag.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/exp/sl_${W}_$tag.json'));print('$W $tag', round(d['ms_per_step'],3), 'fill', round(d['fill_ms'],2), 'walk', round(d['walk_ms'],2), d['config']['traceback_pin']['matches_oracle'])"
}
run base c3
run s5 c3 GA_PIPE_SLOTS=5
run s6 c3 GA_PIPE_SLOTS=6
run f4n c3 GA_PIPE_FILLS=4 GA_PIPE_FILL_PRIO=normal GA_PIPE_SLOTS=6
run f4nf40 c3 GA_PIPE_FILLS=4 GA_PIPE_FILL_PRIO=normal GA_PIPE_SLOTS=6 GA_FILL_LDS_FLOOR=40000
run f3n c3 GA_PIPE_FILL_PRIO=normal GA_PIPE_SLOTS=5
run base c5
run s4 c5 GA_PIPE_SLOTS=4
run base c2
run s4 c2 GA_PIPE_SLOTS=4
