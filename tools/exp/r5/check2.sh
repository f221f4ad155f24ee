set -o pipefail
# round 5: the tie-to-tie walk's first GPU run: perm semantics + trip micro-benchmark, the recompute suite (jump
# walk by default), the walk accounting at C3 (jump / words), and the C3 bench line
O=gpurun_out/r5_check2
mkdir -p $O
timeout -k 10 60 tools/micro/jump_trip > $O/jump_trip.txt 2>&1; cat $O/jump_trip.txt; timeout -k 10 60 tools/micro/lane_pk16 > $O/lane_pk16.txt 2>&1; cat $O/lane_pk16.txt
GA_RC_JUMP=1 timeout -k 10 900 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_rc.py -m gpu > $O/tests.log 2>&1; rc=$?
tail -5 $O/tests.log; grep -E "FAIL|Error|error" $O/tests.log | head -20; [ $rc -eq 0 ] || exit $rc
GA_RC_JUMP=1 timeout -k 10 300 python -u tools/exp/r5/rc_diag.py 100000 64:64 128:64 > $O/rc_diag_jump.txt 2>&1; rc=$?; cat $O/rc_diag_jump.txt; [ $rc -eq 0 ] || exit $rc
GA_RC_JUMP=0 timeout -k 10 300 python -u tools/exp/r5/rc_diag.py 100000 64:64 > $O/rc_diag_words.txt 2>&1; rc=$?; cat $O/rc_diag_words.txt; [ $rc -eq 0 ] || exit $rc
GA_RC_JUMP=1 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/c3.json 2> $O/c3.err; rc=$?; tail -c 1500 $O/c3.json; exit $rc
