set -o pipefail
# (ran against one-off builds with the IO wave idle s_sleep as a macro, since removed: no effect at C4, C3 or the 1M x 125k fills)
# IO-wave idle sleep (s_sleep N per empty round): its spinning shares SIMD 0 with two compute waves
mkdir -p gpurun_out
for v in base 2 4 8; do
  if [ $v = base ]; then unset GA_LIB_PATH; else export GA_LIB_PATH=$PWD/globalign_amd/_lib/var/lib_s$v.so; fi
  echo "$v c4 $(timeout -k 10 120 python -u tools/fill_sweep.py 1000000 1000000 2 0)" >> gpurun_out/sweep52.txt || exit 1
  echo "$v c3 $(timeout -k 10 120 python -u tools/fill_sweep.py 100000 100000 3 1)" >> gpurun_out/sweep52.txt || exit 1
  echo "$v n8diag $(timeout -k 10 120 python -u tools/fill_sweep.py 1000000 125000 3 0)" >> gpurun_out/sweep52.txt || exit 1
  echo "$v n8row $(GA_FILL_MODE=row timeout -k 10 120 python -u tools/fill_sweep.py 1000000 125000 3 0)" >> gpurun_out/sweep52.txt || exit 1
done
