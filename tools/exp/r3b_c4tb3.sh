# Round 3 (second session): checkpoint spacing chosen with the geometry (C4: TD 8 at 64 steps, 141 GB)
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/r3b_c4tb3.txt
: > $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_rc.py -m gpu -x -q --timeout 120 --timeout-method thread >> $O 2>&1 || { tail -30 $O; exit 1; }
timeout -k 10 120 python -u tools/exp/r3_rc_diag.py 100000 64:48:1 >> $O 2>&1 || { tail -20 $O; exit 1; }
timeout -k 10 400 python -u bench.py --workload c4tb --no-cpu-baseline --no-extra --steps 3 --warmup 1 >> $O 2>&1 || { tail -20 $O; exit 1; }
