# round 2: C3 timeline with walks taking slots in fill-completion order (GA_PIPE_TRACE)
set -o pipefail
mkdir -p gpurun_out/exp
for O in any fixed; do
rm -f gpurun_out/exp/trace_so_$O.jsonl
GA_PIPE_SLOT_ORDER=$O GA_PIPE_TRACE=gpurun_out/exp/trace_so_$O.jsonl timeout -k 10 200 python -u bench.py --workload c3 --no-cpu-baseline --no-extra > gpurun_out/exp/sot_$O.json 2> gpurun_out/exp/sot_$O.err || { tail -20 gpurun_out/exp/sot_$O.err; exit 1; }
O=$O python - <<'PY'
import json, os
o = os.environ["O"]
r = [json.loads(l) for l in open(f"gpurun_out/exp/trace_so_{o}.jsonl")][-20:]
print(o, "first_walk", round(r[0]["walk0"], 2), "last_end", round(r[-1]["walk1"], 2), "ms_per_step", json.load(open(f"gpurun_out/exp/sot_{o}.json"))["ms_per_step"])
print(" gaps", [round(r[k]["walk0"] - r[k - 1]["walk1"], 2) for k in range(1, 20)])
print(" fills", [round(x["fill1"] - x["fill0"], 2) for x in r])
PY
done
