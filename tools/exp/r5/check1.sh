set -o pipefail
# round 5: trip micro-benchmark; the recompute / distributed GPU suites after the window-liveness, NOMEM-fallback
# and 8-rank changes
O=gpurun_out/r5_check1
mkdir -p $O
timeout -k 10 60 tools/micro/jump_trip > $O/jump_trip.txt 2>&1 && cat $O/jump_trip.txt &&
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_rc.py tests/test_distributed_gpu.py -m gpu > $O/tests.log 2>&1; rc=$?
tail -5 $O/tests.log; grep -E "FAIL|Error" $O/tests.log | head -20; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/exp/r5/rc_diag.py 100000 64:64 32:64 128:64 > $O/rc_diag.txt 2>&1; rc=$?; cat $O/rc_diag.txt; exit $rc
