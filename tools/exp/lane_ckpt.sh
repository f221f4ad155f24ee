# round 2: the banded traceback's checkpoint pass through the lane kernel: parity, then C4 with traceback
set -o pipefail
mkdir -p gpurun_out/exp
timeout -k 10 600 python -u -m pytest tests/test_gpu_banded.py tests/test_gpu_lane.py -x -q --timeout 300 --timeout-method thread > gpurun_out/exp/ckpt.log 2>&1 || { tail -30 gpurun_out/exp/ckpt.log; exit 1; }
tail -1 gpurun_out/exp/ckpt.log
timeout -k 10 300 python -u bench.py --workload c4tb --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/exp/c4tb.json 2> gpurun_out/exp/c4tb.err || { tail -20 gpurun_out/exp/c4tb.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/exp/c4tb.json'));print('c4tb', round(d['ms_per_step'],1), 'fill', round(d['fill_ms'],1), 'walk', round(d['walk_ms'],1), d['config']['cost_matches_oracle'])"
