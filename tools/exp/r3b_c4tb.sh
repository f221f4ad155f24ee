# Round 3 (second session): C4 with full traceback on one GPU -- now through the recompute walk (it takes every
# problem from 2^32 cells), against the banded path of rounds 1-2 (GA_RC=0)
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/r3b_c4tb.txt
: > $O
echo "== rc (default)" >> $O
timeout -k 10 400 python -u bench.py --workload c4tb --no-cpu-baseline --no-extra --steps 2 --warmup 1 >> $O 2>&1 || { tail -20 $O; exit 1; }
echo "== banded (GA_RC=0)" >> $O
GA_RC=0 timeout -k 10 400 python -u bench.py --workload c4tb --no-cpu-baseline --no-extra --steps 2 --warmup 1 >> $O 2>&1 || { tail -20 $O; exit 1; }
