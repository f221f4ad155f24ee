set -o pipefail
mkdir -p gpurun_out/exp
timeout -k 10 300 python -u -m pytest tests/test_gpu_many.py -x -q --timeout 200 --timeout-method thread > gpurun_out/exp/many.log 2>&1 || { tail -30 gpurun_out/exp/many.log; exit 1; }
tail -1 gpurun_out/exp/many.log
for W in c3 c5 c2; do
  for F in auto 2 3 4; do
    if [ $F = auto ]; then unset GA_PIPE_FILLS; else export GA_PIPE_FILLS=$F; fi
    timeout -k 10 200 python -u bench.py --workload $W --steps 20 --warmup 5 --no-cpu-baseline --no-extra > gpurun_out/exp/pf_${W}_$F.json 2> gpurun_out/exp/pf_${W}_$F.err || { tail -20 gpurun_out/exp/pf_${W}_$F.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/exp/pf_${W}_$F.json'));print('$W F=$F', round(d['ms_per_step'],3), 'fill', round(d['fill_ms'],2), 'walk', round(d['walk_ms'],2), 'rng', round(d['host_tiebreak_ms'],2), d['config']['traceback_pin']['matches_oracle'])"
  done
done
unset GA_PIPE_FILLS
