set -o pipefail
# banded traceback at C4: band height (traceback-word budget) vs refill work and per-band ramps
mkdir -p gpurun_out
for mb in 16384 32768 131072; do
  echo "budget_mb=$mb $(GA_TB_BUDGET_MB=$mb timeout -k 10 400 python -u bench.py --workload c4tb --steps 1 --warmup 1 --no-cpu-baseline 2>>gpurun_out/sweep32.err)" >> gpurun_out/sweep32.txt || exit 1
done
