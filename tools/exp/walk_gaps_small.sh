# round 2: walk-to-walk hand-over gaps of the pipelined C5 / C2 / C3 steps (GA_PIPE_TRACE)
set -o pipefail
mkdir -p gpurun_out/exp
for W in c5 c2 c3; do
  rm -f gpurun_out/exp/trace_${W}_gaps.jsonl
  GA_PIPE_TRACE=gpurun_out/exp/trace_${W}_gaps.jsonl timeout -k 10 300 python -u bench.py --workload $W --no-cpu-baseline --no-extra > gpurun_out/exp/gaps_$W.json 2> gpurun_out/exp/gaps_$W.err || { tail -20 gpurun_out/exp/gaps_$W.err; exit 1; }
  W=$W python - <<'PY'
import json, os
w = os.environ["W"]
rows = [json.loads(l) for l in open(f"gpurun_out/exp/trace_{w}_gaps.jsonl")][-20:]
print(w, "first_walk", round(rows[0]["walk0"], 3), "last_end", round(rows[-1]["walk1"], 3))
print(" gaps", [round(rows[k]["walk0"] - rows[k - 1]["walk1"], 3) for k in range(1, 20)])
print(" fill_ready_to_walk", [round(rows[k]["walk0"] - rows[k]["fill1"], 2) for k in range(1, 20)])
print(" walks", [round(r["walk1"] - r["walk0"], 3) for r in rows])
print(" fills", [round(r["fill1"] - r["fill0"], 3) for r in rows])
d = json.load(open(f"gpurun_out/exp/gaps_{w}.json"))
print(" ms_per_step", d["ms_per_step"], "pin", d["config"]["traceback_pin"]["matches_oracle"])
PY
done
