# round 2: the first r pipeline fills through the row scan (GA_PIPE_ROW_FIRST), C3
set -o pipefail
mkdir -p gpurun_out/exp
for R in 0 1 2; do
  rm -f gpurun_out/exp/trace_c3_rf$R.jsonl
  GA_PIPE_ROW_FIRST=$R GA_PIPE_TRACE=gpurun_out/exp/trace_c3_rf$R.jsonl timeout -k 10 300 python -u bench.py --workload c3 --no-cpu-baseline --no-extra > gpurun_out/exp/rf$R.json 2> gpurun_out/exp/rf$R.err || { tail -20 gpurun_out/exp/rf$R.err; exit 1; }
  python - <<PY
import json
rows = [json.loads(l) for l in open("gpurun_out/exp/trace_c3_rf$R.jsonl")][-20:]
d = json.load(open("gpurun_out/exp/rf$R.json"))
print("rf$R", round(d["ms_per_step"], 3), d["config"]["traceback_pin"]["matches_oracle"], "walk starts", [round(r["walk0"], 1) for r in rows[:5]], "last end", round(rows[-1]["walk1"], 1))
PY
done
