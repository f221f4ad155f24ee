set -o pipefail
mkdir -p gpurun_out/r4_dump
O=gpurun_out/r4_dump
for i in 1 2; do
  LANE_STAMPS_DUMP=$O/slab_$i.npy GA_FILL_MODE=lane timeout -k 10 120 python -u tools/lane_stamps.py 1000000 125000 > $O/slab_$i.json 2> $O/slab_$i.err || { tail -5 $O/slab_$i.err; exit 1; }
  LANE_STAMPS_DUMP=$O/c3_$i.npy GA_FILL_MODE=lane timeout -k 10 120 python -u tools/lane_stamps.py 100000 100000 > $O/c3_$i.json 2> $O/c3_$i.err || { tail -5 $O/c3_$i.err; exit 1; }
done
ls $O
