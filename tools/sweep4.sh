set -o pipefail
for T in 4 2; do
  GA_COLS_PER_LANE=$T timeout -k 5 120 python -u tools/fill_stamps.py 100000 1000000 >> gpurun_out/stamps4.txt || exit 1
  GA_COLS_PER_LANE=$T timeout -k 5 120 python -u tools/fill_stamps.py 100000 100000 --tb >> gpurun_out/stamps4.txt || exit 1
done
for f in 70000 60000; do for T in 4 2; do
  GA_FILL_LDS_FLOOR=$f GA_COLS_PER_LANE=$T timeout -k 5 120 python -u tools/fill_sweep.py 250000 1000000 3 0 >> gpurun_out/sweep4.txt || exit 1
done; done
