# Round 3 (second session): recompute workers below 96 (the walker's tile loads slow down with more)
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/r3b_servers.txt
: > $O
timeout -k 10 300 python -u tools/exp/r3_rc_diag.py 100000 48:48:1 40:48:1 32:48:1 24:48:1 32:64:1 48:64:1 >> $O 2>&1 || { tail -30 $O; exit 1; }
