set -o pipefail
# round 4: the out-path in a wave of its own (GA_LANE_OUTWAVE=1, the default) against the IO wave's (0): lane / rc /
# slab / co-residency tests, lane stamps (C3 shape and the 1M x 125k slab) and the C3 bench line for both
O=gpurun_out/r4_outw
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_lane.py tests/test_gpu_rc.py tests/test_distributed_gpu.py tests/test_coresidency_gpu.py -m gpu > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for v in 1 0; do
  GA_LANE_OUTWAVE=$v GA_FILL_MODE=lane timeout -k 10 120 python -u tools/lane_stamps.py 100000 100000 > $O/stamps_c3_$v.json 2> $O/stamps_c3_$v.err || { tail -5 $O/stamps_c3_$v.err; exit 1; }
  GA_LANE_OUTWAVE=$v GA_FILL_MODE=lane timeout -k 10 120 python -u tools/lane_stamps.py 1000000 125000 > $O/stamps_slab_$v.json 2> $O/stamps_slab_$v.err || { tail -5 $O/stamps_slab_$v.err; exit 1; }
  GA_LANE_OUTWAVE=$v timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/c3_$v.json 2> $O/c3_$v.err || { tail -5 $O/c3_$v.err; exit 1; }
done
python3 tools/exp/r4/r4_lagsum.py $O 1 0
