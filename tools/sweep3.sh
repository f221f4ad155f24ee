set -o pipefail
timeout -k 5 60 tools/micro/row_bench_t > gpurun_out/row_bench_t.txt || exit 1
for T in 4 2; do for NW in 4 8; do
  GA_FILL_NWC=$NW GA_COLS_PER_LANE=$T timeout -k 5 120 python -u tools/fill_sweep.py 250000 1000000 3 0 >> gpurun_out/sweep3.txt || exit 1
done; done
