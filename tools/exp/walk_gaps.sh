# round 2: the pipelined C3 steps' walk-to-walk gaps and fill waits (GA_PIPE_TRACE)
set -o pipefail
mkdir -p gpurun_out/exp
rm -f gpurun_out/exp/trace_c3_gaps.jsonl
GA_PIPE_TRACE=gpurun_out/exp/trace_c3_gaps.jsonl timeout -k 10 300 python -u bench.py --workload c3 --no-cpu-baseline --no-extra > gpurun_out/exp/gaps.json 2> gpurun_out/exp/gaps.err || { tail -20 gpurun_out/exp/gaps.err; exit 1; }
python - <<'PY'
import json
rows = [json.loads(l) for l in open("gpurun_out/exp/trace_c3_gaps.jsonl")][-20:]
w = [r["walk0"] for r in rows]
print("first_walk", rows[0]["walk0"], "steady", (w[-1] - w[-11]) / 10, "last_end", rows[-1]["walk1"])
print("gaps", [round(rows[k]["walk0"] - rows[k - 1]["walk1"], 3) for k in range(1, 20)])
print("fill_ready_to_walk", [round(rows[k]["walk0"] - rows[k]["fill1"], 2) for k in range(1, 20)])
print("walks", [round(r["walk1"] - r["walk0"], 2) for r in rows])
print("ms_per_step", json.load(open("gpurun_out/exp/gaps.json"))["ms_per_step"])
PY
