set -o pipefail
for n in 64 256 1024 16384; do
  GA_COLS_PER_LANE=1 GA_FILL_NWC=4 timeout -k 5 120 python -u tools/fill_stamps.py 100000 $n >> gpurun_out/stamps10.txt || exit 1
done
for n in 128 512 2048 32768; do
  GA_COLS_PER_LANE=2 GA_FILL_NWC=4 timeout -k 5 120 python -u tools/fill_stamps.py 100000 $n >> gpurun_out/stamps10.txt || exit 1
done
