set -o pipefail
# (ran against a one-off build with a T = 6 / NWC = 12 instantiation, since removed: 354 ms vs 313 ms for T = 8 / NWC = 8)
# C4 with 6 columns per lane and 12 compute waves per workgroup (3 waves per SIMD), experiment build
mkdir -p gpurun_out
export GA_LIB_PATH=$PWD/globalign_amd/_lib/var/lib_t6.so
echo "T6 nwc12 small $(GA_COLS_PER_LANE=6 GA_FILL_NWC=12 timeout -k 10 120 python -u tools/fill_sweep.py 20000 50000 2 0)" >> gpurun_out/sweep51.txt || exit 1
echo "T8 nwc8 small $(timeout -k 10 120 python -u tools/fill_sweep.py 20000 50000 2 0)" >> gpurun_out/sweep51.txt || exit 1
echo "T6 nwc12 c4 $(GA_COLS_PER_LANE=6 GA_FILL_NWC=12 timeout -k 10 120 python -u tools/fill_sweep.py 1000000 1000000 3 0)" >> gpurun_out/sweep51.txt || exit 1
echo "T6 nwc8 c4 $(GA_COLS_PER_LANE=6 GA_FILL_NWC=8 timeout -k 10 120 python -u tools/fill_sweep.py 1000000 1000000 3 0)" >> gpurun_out/sweep51.txt || exit 1
echo "T8 nwc8 c4 $(timeout -k 10 120 python -u tools/fill_sweep.py 1000000 1000000 3 0)" >> gpurun_out/sweep51.txt || exit 1
