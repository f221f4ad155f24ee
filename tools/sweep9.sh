set -o pipefail
for T in 1 2; do
GA_COLS_PER_LANE=$T timeout -k 5 120 python -u tools/fill_stamps.py 100000 100000 --tb >> gpurun_out/stamps9.txt || exit 1
done
GA_COLS_PER_LANE=8 timeout -k 5 120 python -u tools/fill_stamps.py 100000 1000000 >> gpurun_out/stamps9.txt || exit 1
timeout -k 5 120 python -u tools/fill_sweep.py 1000000 1000000 2 0 >> gpurun_out/sweep9.txt || exit 1
for T in 1 2; do GA_COLS_PER_LANE=$T timeout -k 5 120 python -u tools/fill_sweep.py 100000 100000 3 1 >> gpurun_out/sweep9.txt || exit 1; done
