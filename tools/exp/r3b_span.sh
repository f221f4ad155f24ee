# Round 3 (second session): recompute candidates 16 x 16 blocks deep (GA_RC_SPAN) at C3 and C4 with traceback
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/r3b_span.txt
: > $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_rc.py -m gpu -x -q --timeout 120 --timeout-method thread >> $O 2>&1 || { tail -30 $O; exit 1; }
for sp in 8 16; do
  echo "== span $sp" >> $O
  GA_RC_SPAN=$sp timeout -k 10 200 python -u tools/exp/r3_rc_diag.py 100000 64:48:1 64:64:1 >> $O 2>&1 || { tail -20 $O; exit 1; }
  GA_RC_SPAN=$sp timeout -k 10 300 python -u tools/exp/r3_rc_diag.py 1000000 64:48:1 64:64:1 >> $O 2>&1 || { tail -20 $O; exit 1; }
done
