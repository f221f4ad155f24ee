set -o pipefail
# pace along the chain (per-stripe row time samples): anti-diagonal TD=1,2 vs row scan at the N=8 slab shape
mkdir -p gpurun_out
GA_FILL_MODE=diag GA_DIAG_COLS_PER_LANE=2 timeout -k 10 120 python -u tools/fill_stamps.py 1000000 125000 > gpurun_out/s26_d2.json || exit 1
GA_FILL_MODE=diag GA_DIAG_COLS_PER_LANE=1 timeout -k 10 120 python -u tools/fill_stamps.py 1000000 125000 > gpurun_out/s26_d1.json || exit 1
timeout -k 10 120 python -u tools/fill_stamps.py 1000000 125000 > gpurun_out/s26_r.json || exit 1
