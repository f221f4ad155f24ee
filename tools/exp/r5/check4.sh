set -o pipefail
# round 5: the jump workers' two-phase group (16 LUT loads in flight): jump suites, C3 accounting by servers
O=gpurun_out/r5_check4
mkdir -p $O
GA_RC_JUMP=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_rc.py -m gpu -k "jump or dna or stripe_widths or protein" > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log; grep -E "FAIL|Error" $O/tests.log | head -10; [ $rc -eq 0 ] || exit $rc
GA_RC_JUMP=1 timeout -k 10 300 python -u tools/exp/r5/rc_diag.py 100000 64:64 128:64 255:64 > $O/rc_diag_jump.txt 2>&1; rc=$?; cat $O/rc_diag_jump.txt; exit $rc
