# Round 3 (second session): walker trims (widening pinned in its group, fused level accumulation, per-iteration
# entry pointer) -- walk-heavy parity, the C3 call by recompute-worker count, the C5 walk's accounting
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/r3b_sld2.txt
: > $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_rc.py tests/test_gpu_banded.py tests/test_gpu_many.py -m gpu -x -q --timeout 120 --timeout-method thread >> $O 2>&1 || { tail -30 $O; exit 1; }
timeout -k 10 200 python -u tools/exp/r3_rc_diag.py 100000 96:48:1 128:48:1 160:48:1 200:48:1 160:64:1 >> $O 2>&1 || { tail -30 $O; exit 1; }
timeout -k 10 120 python -u tools/walk_diag.py c5 >> $O 2>&1 || exit 1
timeout -k 10 120 python -u tools/walk_diag.py c2 >> $O 2>&1 || exit 1
