# Round 3: streamed walk decode: the rc suite three times as shipped, then with GA_RC_DECODE_CHECK (level
# words that changed after the host decoded them)
set -o pipefail
T="tests/test_gpu_rc.py"
for k in 1 2 3 4; do
  timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread $T 2>&1 | grep -E "passed|failed|decode check|^E  .*Assert" | head -8
done
for k in 1 2; do
  GA_RC_DECODE_CHECK=1 timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread $T 2>&1 | grep -E "passed|failed|decode check" | head -8
done
