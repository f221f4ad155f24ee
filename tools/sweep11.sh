set -o pipefail
for T in 4 2 1; do
GA_COLS_PER_LANE=$T timeout -k 5 120 python -u tools/fill_sweep.py 65536 1000000 3 1 >> gpurun_out/sweep11.txt || exit 1
GA_COLS_PER_LANE=$T timeout -k 5 120 python -u tools/fill_sweep.py 65536 1000000 2 0 >> gpurun_out/sweep11.txt || exit 1
done
export TMPDIR=/tmp
GA_COLS_PER_LANE=4 timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/w11 -o run -- python3 tools/fill_sweep.py 65536 1000000 1 1 > gpurun_out/w11.log 2>&1 || exit 1
