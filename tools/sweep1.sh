set -e
for f in "" 50000 30000 0; do
  if [ -z "$f" ]; then unset GA_FILL_LDS_FLOOR; else export GA_FILL_LDS_FLOOR=$f; fi
  timeout -k 5 120 python -u tools/fill_sweep.py 250000 1000000 4 0 >> gpurun_out/sweep1.txt
  timeout -k 5 120 python -u tools/fill_sweep.py 100000 100000 4 1 >> gpurun_out/sweep1.txt
done
