set -o pipefail
# end-of-round evidence: GPU suite, bench lines for every workload, rocprofv3 summaries (tools/exp/profile_round.sh)
cd /root/repo
O=gpurun_out/final
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 400 python -u bench.py > $O/bench_default_c4.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
for W in c3 c5 c2; do
  timeout -k 10 300 python -u bench.py --workload $W --no-cpu-baseline > $O/bench_$W.json 2>> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
done
timeout -k 10 400 python -u bench.py --workload c4tb --steps 2 --warmup 1 --no-cpu-baseline > $O/bench_c4tb.json 2>> $O/bench.err || exit 1
timeout -k 10 200 python -u tools/fill_stamps.py 100000 100000 --tb > $O/fill_stamps_c3.json || exit 1
bash tools/exp/profile_round.sh
