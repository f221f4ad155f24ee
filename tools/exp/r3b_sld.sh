# Round 3 (second session): walk tie-break entries by scalar loads -- walk-heavy parity, then the C3 call
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/r3b_sld.txt
: > $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_rc.py tests/test_gpu_banded.py tests/test_gpu_many.py -m gpu -x -q --timeout 120 --timeout-method thread >> $O 2>&1 || { tail -30 $O; exit 1; }
timeout -k 10 120 python -u tools/exp/r3_rc_diag.py 100000 96:48:1 >> $O 2>&1 || { tail -30 $O; exit 1; }
timeout -k 10 200 python -u bench.py --workload c5 --no-cpu-baseline --no-extra --steps 10 --warmup 3 >> $O 2>&1 || exit 1
timeout -k 10 200 python -u bench.py --workload c2 --no-cpu-baseline --no-extra --steps 10 --warmup 3 >> $O 2>&1 || exit 1
