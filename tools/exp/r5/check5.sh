set -o pipefail
# round 5: the window 32 block rows x 8 stripes deep (cache 64 x 32), cone weights; word walk unchanged
O=gpurun_out/r5_check5
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_rc.py -m gpu -k "worker_pools or deep_window or jump or stripe_widths" > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log; grep -E "FAIL|Error" $O/tests.log | head -10; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/exp/r5/rc_diag.py 100000 64:64 > $O/rc_diag_words.txt 2>&1; rc=$?; cat $O/rc_diag_words.txt; [ $rc -eq 0 ] || exit $rc
GA_RC_JUMP=1 timeout -k 10 400 python -u tools/exp/r5/rc_diag.py 100000 128:64:1 128:64:2 128:64:3 192:64:3 128:48:3 > $O/rc_diag_jump.txt 2>&1; rc=$?; cat $O/rc_diag_jump.txt; exit $rc
