set -o pipefail
GA_COLS_PER_LANE=16 GA_FILL_NWC=4 timeout -k 5 120 python -u tools/fill_sweep.py 250000 1000000 3 0 >> gpurun_out/sweep13.txt || exit 1
timeout -k 5 120 python -u tools/fill_sweep.py 250000 1000000 3 0 >> gpurun_out/sweep13.txt || exit 1
GA_COLS_PER_LANE=16 GA_FILL_NWC=4 timeout -k 5 120 python -u tools/fill_stamps.py 100000 1000000 >> gpurun_out/stamps13.txt || exit 1
