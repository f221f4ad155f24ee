# round 2: what the chained walks wait for (result[12..14]: wait time, polls with the fill / the entries not ready)
set -o pipefail
mkdir -p gpurun_out/exp
for W in c2 c5; do
  rm -f gpurun_out/exp/trace_cw_$W.jsonl
  GA_PIPE_TRACE=gpurun_out/exp/trace_cw_$W.jsonl timeout -k 10 200 python -u bench.py --workload $W --no-cpu-baseline --no-extra > gpurun_out/exp/cw_$W.json 2> gpurun_out/exp/cw_$W.err || { tail -20 gpurun_out/exp/cw_$W.err; exit 1; }
  W=$W python - <<'PY'
import json, os
w = os.environ["W"]
r = [json.loads(l) for l in open(f"gpurun_out/exp/trace_cw_{w}.jsonl")][-20:]
print(w, "ms_per_step", round(json.load(open(f"gpurun_out/exp/cw_{w}.json"))["ms_per_step"], 3), "walks", round(sum(x["walk_ms"] for x in r), 2))
print(" wait_us", [round(x["chain_wait_us"]) for x in r])
print(" polls fill/tab", [(x["polls_fill"], x["polls_tab"]) for x in r])
PY
done
