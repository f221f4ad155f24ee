set -o pipefail
# round 5: the pipelined trip loop: the recompute suite under the jump walk, the walk accounting at C3 by workers /
# window, the C3 bench line
O=gpurun_out/r5_check3
mkdir -p $O
GA_RC_JUMP=1 timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_rc.py -m gpu > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log; grep -E "FAIL|Error" $O/tests.log | head -10; [ $rc -eq 0 ] || exit $rc
GA_RC_JUMP=1 timeout -k 10 300 python -u tools/exp/r5/rc_diag.py 100000 64:64 128:64 128:32 192:32 > $O/rc_diag_jump.txt 2>&1; rc=$?; cat $O/rc_diag_jump.txt; exit $rc
