set -o pipefail
# round 4, final tree: the GPU suite, then the PMC / kernel-stats profiles every bench line's roofline reads
# (tools/profile_r04.sh -> profiles/r04, copied to gpurun_out/prof_r04_out)
O=gpurun_out/r4_final
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_suite.txt 2>&1 || { tail -40 $O/gpu_suite.txt; exit 1; }
tail -2 $O/gpu_suite.txt
bash tools/profile_r04.sh > $O/profile.log 2>&1 || { tail -30 $O/profile.log; exit 1; }
tail -5 $O/profile.log
