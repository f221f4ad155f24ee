# round 2: the whole GPU suite (new: io parity, edited dp_array walks, in-process devices, C3/C5 pins)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?
tail -5 gpurun_out/gpu_tests.log
exit $rc
