# round 2: extended VALU microbench, co-residency at default priority, the new bench line, a
# 2-rank gloo rehearsal of the launcher (ranks share the one GPU)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 ./tools/micro/valu_rate > gpurun_out/valu_rate.txt 2>&1 &&
timeout -k 10 240 python -u tools/coresidency.py > gpurun_out/coresidency.txt 2>&1 &&
timeout -k 10 400 python -u bench.py > gpurun_out/bench_n1.json 2> gpurun_out/bench_n1.err &&
GA_DIST_BACKEND=gloo timeout -k 10 300 python -u bench.py --gpus 2 --workload c2 --steps 3 --warmup 1 > gpurun_out/bench_gloo2_c2.json 2> gpurun_out/bench_gloo2_c2.err
echo "rc=$?"
