# Round 3 (second session): C4 with full traceback through the recompute walk by checkpoint spacing
# (every 256: the default budget; 128 / 64 need 78 / 156 GB of checkpoints at TD 4), and the alignment
# against the banded path's (digests of the strings and the random state)
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/r3b_c4rc.txt
: > $O
timeout -k 10 600 python -u tools/exp/r3b_c4rc.py >> $O 2>&1 || { tail -20 $O; exit 1; }
