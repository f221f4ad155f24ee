# round 2: per-launch pipeline walks writing their result words and levels to pinned host memory (no
# hipMemcpy in the hand-over): pipeline parity, C3 timeline, C3 twice
set -o pipefail
mkdir -p gpurun_out/exp
timeout -k 10 200 python -u -m pytest tests/test_gpu_many.py -x -q --timeout 120 --timeout-method thread > gpurun_out/exp/pio_tests.log 2>&1 || { tail -30 gpurun_out/exp/pio_tests.log; exit 1; }
tail -1 gpurun_out/exp/pio_tests.log
rm -f gpurun_out/exp/trace_pio.jsonl
GA_PIPE_TRACE=gpurun_out/exp/trace_pio.jsonl timeout -k 10 200 python -u bench.py --workload c3 --no-cpu-baseline --no-extra > gpurun_out/exp/pio_t.json 2> gpurun_out/exp/pio_t.err || { tail -20 gpurun_out/exp/pio_t.err; exit 1; }
python - <<'PY'
import json
r = [json.loads(l) for l in open("gpurun_out/exp/trace_pio.jsonl")][-20:]
print("first_walk", round(r[0]["walk0"], 2), "last_end", round(r[-1]["walk1"], 2), "ms_per_step", json.load(open("gpurun_out/exp/pio_t.json"))["ms_per_step"])
print(" gaps", [round(r[k]["walk0"] - r[k - 1]["walk1"], 2) for k in range(1, 20)])
PY
for R in 1 2; do
  timeout -k 10 200 python -u bench.py --workload c3 --no-cpu-baseline --no-extra > gpurun_out/exp/pio_$R.json 2> gpurun_out/exp/pio_$R.err || { tail -20 gpurun_out/exp/pio_$R.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/exp/pio_$R.json'));print('c3', round(d['ms_per_step'],3), 'fill', round(d['fill_ms'],2), 'walk', round(d['walk_ms'],3), d['config']['cost_matches_oracle'], d['config']['traceback_pin']['matches_oracle'])"
done
