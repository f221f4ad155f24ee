set -o pipefail
timeout -k 5 200 python -u tools/diag_check.py > gpurun_out/diag_check.txt 2>&1 || exit 1
grep -v amdgpu gpurun_out/diag_check.txt
for NW in 8 4; do
GA_FILL_NWC=$NW GA_FILL_MODE=diag timeout -k 5 120 python -u tools/fill_stamps.py 100000 1000000 >> gpurun_out/stamps8.txt || exit 1
done
GA_FILL_MODE=diag timeout -k 5 120 python -u tools/fill_sweep.py 1000000 1000000 2 0 >> gpurun_out/sweep8.txt || exit 1
