set -o pipefail
for shape in "1000000 128" "1000000 512" "1000000 2048" "1000000 8192"; do
  set -- $shape
  GA_FILL_MODE=lane GA_LANE_COLS_PER_LANE=2 GA_FILL_NWC=4 timeout -k 10 120 python -u tools/lane_stamps.py $1 $2 || exit 1
done
