set -o pipefail
# the upper half of a workgroup's compute waves at a higher issue priority (C4 waves 0-3 wait 37 %)
mkdir -p gpurun_out
for v in base prio; do
  if [ $v = base ]; then unset GA_LIB_PATH; else export GA_LIB_PATH=$PWD/globalign_amd/_lib/var/lib_prio.so; fi
  echo "$v c4 $(timeout -k 10 120 python -u tools/fill_sweep.py 1000000 1000000 3 0)" >> gpurun_out/sweep46.txt || exit 1
  echo "$v c3 $(timeout -k 10 120 python -u tools/fill_sweep.py 100000 100000 3 1)" >> gpurun_out/sweep46.txt || exit 1
  echo "$v n8 $(GA_FILL_MODE=row timeout -k 10 120 python -u tools/fill_sweep.py 1000000 125000 3 0)" >> gpurun_out/sweep46.txt || exit 1
done
export GA_LIB_PATH=$PWD/globalign_amd/_lib/var/lib_prio.so
timeout -k 10 200 python -u tools/fill_stamps.py 1000000 1000000 > gpurun_out/s46_c4_prio.json || exit 1
