# round 2: pipelined walks chained in one launch (walk_chain_kernel) against one launch per walk
# (GA_PIPE_CHAIN=0): pipeline parity, then C2 / C5 / C3 bench lines both ways
set -o pipefail
mkdir -p gpurun_out/exp
timeout -k 10 300 python -u -m pytest tests/test_gpu_many.py -x -q --timeout 120 --timeout-method thread > gpurun_out/exp/chain_tests.log 2>&1 || { tail -30 gpurun_out/exp/chain_tests.log; exit 1; }
tail -1 gpurun_out/exp/chain_tests.log
for W in c2 c5 c3; do
  for CH in 1 0; do
    rm -f gpurun_out/exp/trace_chain_${W}_$CH.jsonl
    GA_PIPE_CHAIN=$CH GA_PIPE_TRACE=gpurun_out/exp/trace_chain_${W}_$CH.jsonl timeout -k 10 200 python -u bench.py --workload $W --no-cpu-baseline --no-extra > gpurun_out/exp/chain_${W}_$CH.json 2> gpurun_out/exp/chain_${W}_$CH.err || { tail -20 gpurun_out/exp/chain_${W}_$CH.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/exp/chain_${W}_$CH.json'));print('$W chain=$CH', round(d['ms_per_step'],3), 'fill', round(d['fill_ms'],2), 'walk', round(d['walk_ms'],3), d['config']['cost_matches_oracle'], d['config']['traceback_pin']['matches_oracle'])"
  done
done
