set -o pipefail
GA_FILL_MODE=diag timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/parity_diag.log 2>&1 || { tail -40 gpurun_out/parity_diag.log; exit 1; }
tail -2 gpurun_out/parity_diag.log
for NW in 8 4; do
GA_FILL_NWC=$NW GA_FILL_MODE=diag timeout -k 5 120 python -u tools/fill_stamps.py 100000 1000000 >> gpurun_out/stamps7.txt || exit 1
done
GA_FILL_MODE=diag timeout -k 5 120 python -u tools/fill_sweep.py 1000000 1000000 2 0 >> gpurun_out/sweep7.txt || exit 1
