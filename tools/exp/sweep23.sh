set -o pipefail
# pace of short chains: one workgroup, 1..4 stripes, 1M rows (diag TD=1,2 and row scan)
mkdir -p gpurun_out
for n in 64 128 256 512 2048; do
  echo "diag td=1 $(GA_FILL_MODE=diag GA_DIAG_COLS_PER_LANE=1 timeout -k 10 120 python -u tools/fill_sweep.py 1000000 $n 2 0)" >> gpurun_out/sweep23.txt || exit 1
  echo "diag td=2 $(GA_FILL_MODE=diag GA_DIAG_COLS_PER_LANE=2 timeout -k 10 120 python -u tools/fill_sweep.py 1000000 $n 2 0)" >> gpurun_out/sweep23.txt || exit 1
  echo "row $(GA_COLS_PER_LANE=1 timeout -k 10 120 python -u tools/fill_sweep.py 1000000 $n 2 0)" >> gpurun_out/sweep23.txt || exit 1
done
