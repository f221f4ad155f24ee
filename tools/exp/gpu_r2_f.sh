# round 2: pipelined C3/C5 with the leaner table producer; LDS-floor experiment (2+ fill workgroups per CU)
set -o pipefail
mkdir -p gpurun_out/exp
timeout -k 10 300 python -u -m pytest tests/test_gpu_many.py -x -q --timeout 300 --timeout-method thread > gpurun_out/exp/many.log 2>&1 || { tail -30 gpurun_out/exp/many.log; exit 1; }
for W in c3 c5; do
  for F in default 0 40000; do
    if [ $F = default ]; then unset GA_FILL_LDS_FLOOR; else export GA_FILL_LDS_FLOOR=$F; fi
    timeout -k 10 300 python -u bench.py --workload $W --steps 20 --warmup 5 --no-cpu-baseline --no-extra > gpurun_out/exp/bench_${W}_$F.json 2> gpurun_out/exp/bench_${W}_$F.err || { tail -20 gpurun_out/exp/bench_${W}_$F.err; exit 1; }
  done
done
unset GA_FILL_LDS_FLOOR
