set -o pipefail
# C3 fill with traceback words: stripe width / workgroup size after the hand-off changes
mkdir -p gpurun_out
for cfg in "1 8" "1 4" "2 4" "2 8"; do set -- $cfg
  echo "T=$1 nwc=$2 $(GA_COLS_PER_LANE=$1 GA_FILL_NWC=$2 timeout -k 10 120 python -u tools/fill_sweep.py 100000 100000 3 1)" >> gpurun_out/sweep39.txt || exit 1
done
