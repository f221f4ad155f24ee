set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 ./tools/micro/valu_rate > gpurun_out/valu_rate.txt 2>&1 &&
timeout -k 10 240 python -u tools/coresidency.py > gpurun_out/coresidency.txt 2>&1 &&
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
echo "rc=$?"
tail -3 gpurun_out/gpu_tests.log
