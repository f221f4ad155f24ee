set -o pipefail
# N=2 / N=4 slab shapes: stripe width and workgroup size (one wave per SIMD vs two)
mkdir -p gpurun_out
for n in 500000 250000; do for cfg in "8 4" "4 4" "4 8" "2 8" "2 4"; do set -- $cfg
  echo "n=$n T=$1 nwc=$2 $(GA_FILL_MODE=row GA_COLS_PER_LANE=$1 GA_FILL_NWC=$2 timeout -k 10 120 python -u tools/fill_sweep.py 1000000 $n 2 0)" >> gpurun_out/sweep40.txt || exit 1
done; done
echo "n=500000 auto $(timeout -k 10 120 python -u tools/fill_sweep.py 1000000 500000 2 0)" >> gpurun_out/sweep40.txt
echo "n=250000 auto $(timeout -k 10 120 python -u tools/fill_sweep.py 1000000 250000 2 0)" >> gpurun_out/sweep40.txt
