set -o pipefail
# N=8 slab shape (1M rows x 125k columns): stripe width / workgroup size
mkdir -p gpurun_out
for t in 1 2 4 8; do for w in 4 8; do
  echo "T=$t nwc=$w $(GA_COLS_PER_LANE=$t GA_FILL_NWC=$w timeout -k 10 120 python -u tools/fill_sweep.py 1000000 125000 3 0)" >> gpurun_out/sweep16.txt || exit 1
done; done
for t in 1 2 4; do
  echo "T=$t 250k $(GA_COLS_PER_LANE=$t timeout -k 10 120 python -u tools/fill_sweep.py 1000000 250000 3 0)" >> gpurun_out/sweep16.txt || exit 1
done
