# lane-skewed traceback fills: standalone fill time and the pipelined bench (C3, C5) per stripe width
set -o pipefail
mkdir -p gpurun_out/exp
for td in 1 2 4; do
  for nwc in 4 8; do
    GA_FILL_MODE=lane GA_LANE_COLS_PER_LANE=$td GA_FILL_NWC=$nwc timeout -k 10 120 python -u tools/fill_sweep.py 100000 100000 3 1 >> gpurun_out/exp/lane_tb_fill.jsonl || exit 1
  done
done
timeout -k 10 120 python -u tools/fill_sweep.py 100000 100000 3 1 >> gpurun_out/exp/lane_tb_fill.jsonl || exit 1
for W in c3 c5; do
  for cfg in "1 4" "1 8" "2 4" "2 8" "4 4"; do
    set -- $cfg
    [ $W = c5 ] && [ $1 = 4 ] && continue
    GA_FILL_MODE=lane GA_LANE_COLS_PER_LANE=$1 GA_FILL_NWC=$2 timeout -k 10 200 python -u bench.py --workload $W --steps 20 --warmup 5 --no-cpu-baseline --no-extra > gpurun_out/exp/lb_${W}_T$1_N$2.json 2> gpurun_out/exp/lb_${W}_T$1_N$2.err || { tail -20 gpurun_out/exp/lb_${W}_T$1_N$2.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/exp/lb_${W}_T$1_N$2.json'));print('$W T=$1 nwc=$2', round(d['ms_per_step'],3), 'fill', round(d['fill_ms'],2), 'walk', round(d['walk_ms'],2), 'rng', round(d['host_tiebreak_ms'],2), 'lat', round(d['latency_ms_per_alignment'],2), d['config']['traceback_pin']['matches_oracle'])"
  done
done
python -c "
import json
for l in open('gpurun_out/exp/lane_tb_fill.jsonl'): d=json.loads(l); print(d['kind'], [round(x,2) for x in d['fill_ms']], d['cost'])"
