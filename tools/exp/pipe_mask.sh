# round 2: pipelined C3 / C5 with the walk on CUs of its own (GA_PIPE_WALK_CUS) and two fills per CU
set -o pipefail
mkdir -p gpurun_out/exp
run() {  # tag workload env...
  tag=$1; W=$2; shift 2
  rm -f gpurun_out/exp/trace_${W}_$tag.jsonl
  env GA_PIPE_TRACE=gpurun_out/exp/trace_${W}_$tag.jsonl "$@" timeout -k 10 200 python -u bench.py --workload $W --steps 20 --warmup 3 --no-cpu-baseline --no-extra > gpurun_out/exp/pm_${W}_$tag.json 2> gpurun_out/exp/pm_${W}_$tag.err || { tail -20 gpurun_out/exp/pm_${W}_$tag.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/exp/pm_${W}_$tag.json'));print('$W $tag', round(d['ms_per_step'],3), 'fill', round(d['fill_ms'],2), 'walk', round(d['walk_ms'],2), 'rng', round(d['host_tiebreak_ms'],2), d['config']['traceback_pin']['matches_oracle'])"
}
run row c3
run m1 c3 GA_PIPE_WALK_CUS=1
run m1f54 c3 GA_PIPE_WALK_CUS=1 GA_FILL_LDS_FLOOR=54000
run m1f54p3 c3 GA_PIPE_WALK_CUS=1 GA_FILL_LDS_FLOOR=54000 GA_PIPE_FILLS=3
run m1f54p4 c3 GA_PIPE_WALK_CUS=1 GA_FILL_LDS_FLOOR=54000 GA_PIPE_FILLS=4
run m1lane c3 GA_PIPE_WALK_CUS=1 GA_FILL_MODE=lane GA_LANE_COLS_PER_LANE=2 GA_FILL_NWC=4 GA_FILL_LDS_FLOOR=54000 GA_LANE_QROWS=2048
run m1t2 c3 GA_PIPE_WALK_CUS=1 GA_FILL_LDS_FLOOR=54000 GA_COLS_PER_LANE=2 GA_FILL_NWC=4
run row c5
run m1f54 c5 GA_PIPE_WALK_CUS=1 GA_FILL_LDS_FLOOR=54000
run m1f54p3 c5 GA_PIPE_WALK_CUS=1 GA_FILL_LDS_FLOOR=54000 GA_PIPE_FILLS=3
