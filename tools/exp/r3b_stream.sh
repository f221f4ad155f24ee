# Round 3 (second session): the stored-words single call decodes its walk's levels while the walk runs
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/r3b_stream.txt
: > $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_blocked.py tests/test_gpu_lane.py tests/test_io_parity.py -m gpu -x -q --timeout 120 --timeout-method thread >> $O 2>&1 || { tail -30 $O; exit 1; }
for W in c5 c2; do
  for cfg in "GA_WALK_NOSTREAM=1" "GA_X=0" "GA_WALK_NOSTREAM=1" "GA_X=0"; do
    echo "== $W $cfg" >> $O
    env $cfg timeout -k 10 200 python -u bench.py --workload $W --no-cpu-baseline --no-extra --steps 20 --warmup 5 >> $O 2>&1 || exit 1
  done
done
