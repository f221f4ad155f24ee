set -o pipefail
for NW in 8 4; do
GA_FILL_NWC=$NW GA_COLS_PER_LANE=8 timeout -k 5 120 python -u tools/fill_stamps.py 100000 1000000 >> gpurun_out/stamps6.txt || exit 1
done
GA_COLS_PER_LANE=1 timeout -k 5 120 python -u tools/fill_stamps.py 100000 100000 --tb >> gpurun_out/stamps6.txt || exit 1
