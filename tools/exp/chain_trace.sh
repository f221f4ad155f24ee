# round 2: timelines of the chained walks (GA_PIPE_TRACE): per alignment fill time, walker time and the
# host's view of each walk's end; C3 chained / per-walk launches
set -o pipefail
mkdir -p gpurun_out/exp
for CH in 1 0; do
  rm -f gpurun_out/exp/trace_ct_$CH.jsonl
  GA_PIPE_CHAIN=$CH GA_PIPE_TRACE=gpurun_out/exp/trace_ct_$CH.jsonl timeout -k 10 200 python -u bench.py --workload c3 --no-cpu-baseline --no-extra > gpurun_out/exp/ct_$CH.json 2> gpurun_out/exp/ct_$CH.err || { tail -20 gpurun_out/exp/ct_$CH.err; exit 1; }
done
python - <<'PY'
import json
r = [json.loads(l) for l in open("gpurun_out/exp/trace_ct_1.jsonl")][-20:]
t = [x["walk_done_host"] for x in r]
print("chain done_host", [round(v, 2) for v in t])
print("chain waits", [round(t[k] - t[k - 1] - r[k]["walk_ms"], 2) for k in range(1, 20)])
print("chain fills", [round(x["fill_ms"], 2) for x in r])
r = [json.loads(l) for l in open("gpurun_out/exp/trace_ct_0.jsonl")][-20:]
print("off walk0", [round(x["walk0"], 2) for x in r])
print("off gaps", [round(r[k]["walk0"] - r[k - 1]["walk1"], 2) for k in range(1, 20)])
print("off fills", [round(x["fill1"] - x["fill0"], 2) for x in r])
print("off fill0", [round(x["fill0"], 2) for x in r])
for CH in (1, 0):
    print(CH, json.load(open(f"gpurun_out/exp/ct_{CH}.json"))["ms_per_step"])
PY
