set -o pipefail
# round 5: trip loop with full / partial anchor modes; TD 2 fills (smaller recompute blocks) for both walks
O=gpurun_out/r5_check6
mkdir -p $O
GA_RC_JUMP=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_rc.py -m gpu > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log; grep -E "FAIL|Error" $O/tests.log | head -10; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/exp/r5/rc_diag.py 100000 64:64 > $O/rc_diag_words.txt 2>&1; rc=$?; cat $O/rc_diag_words.txt; [ $rc -eq 0 ] || exit $rc
GA_RC_JUMP=1 timeout -k 10 300 python -u tools/exp/r5/rc_diag.py 100000 64:64:1 128:64:1 128:64:2 > $O/rc_diag_jump.txt 2>&1; rc=$?; cat $O/rc_diag_jump.txt; [ $rc -eq 0 ] || exit $rc
GA_LANE_COLS_PER_LANE=2 timeout -k 10 200 python -u tools/exp/r5/rc_diag.py 100000 64:64 > $O/rc_diag_words_td2.txt 2>&1; rc=$?; cat $O/rc_diag_words_td2.txt; [ $rc -eq 0 ] || exit $rc
GA_LANE_COLS_PER_LANE=2 GA_RC_JUMP=1 timeout -k 10 300 python -u tools/exp/r5/rc_diag.py 100000 128:64:1 192:64:2 > $O/rc_diag_jump_td2.txt 2>&1; rc=$?; cat $O/rc_diag_jump_td2.txt; exit $rc
