set -o pipefail
# edge prefetch row: baseline (u=0) vs u=1,2,3 -- parity, stamps at C3 (tb) and N=8-like 100k x 125k, C4 fill
mkdir -p gpurun_out
for v in base 1 2 3; do
  if [ $v = base ]; then unset GA_LIB_PATH; else export GA_LIB_PATH=$PWD/globalign_amd/_lib/var/lib_eu$v.so; fi
  timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_blocked.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t14_$v.log 2>&1 || { tail -30 gpurun_out/t14_$v.log; exit 1; }
  tail -1 gpurun_out/t14_$v.log
  timeout -k 10 120 python -u tools/fill_stamps.py 100000 100000 --tb > gpurun_out/s14_c3_$v.json 2>gpurun_out/s14_$v.err || exit 1
  timeout -k 10 120 python -u tools/fill_stamps.py 1000000 125000 > gpurun_out/s14_n8_$v.json 2>>gpurun_out/s14_$v.err || exit 1
  echo "$v $(timeout -k 10 120 python -u tools/fill_sweep.py 1000000 1000000 3 0)" >> gpurun_out/sweep14.txt || exit 1
done
