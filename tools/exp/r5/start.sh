set -o pipefail
# round 5, second session's first GPU call: the GPU suite on this tree, the default bench line, C5 / C2 single calls,
# then the C4 A/B of the round-4 lane changes (c4ab.sh)
O=gpurun_out/r5_start
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_suite.txt 2>&1 || { tail -40 $O/gpu_suite.txt; exit 1; }
tail -2 $O/gpu_suite.txt
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
for w in c5 c2; do
  timeout -k 10 200 python -u bench.py --workload $w --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_$w.json 2> $O/bench_$w.err || { tail -20 $O/bench_$w.err; exit 1; }
done
python3 - <<'PY'
import json
O = "gpurun_out/r5_start"
for f in ("bench_default", "bench_c5", "bench_c2"):
    d = json.loads(open(f"{O}/{f}.json").read().strip().splitlines()[-1])
    s = f"{f}: ms/step {d['ms_per_step']:.3f} fill {d.get('fill_ms', 0):.3f} walk {d.get('walk_ms', 0):.3f} tb {d.get('host_tiebreak_ms')} kind {d.get('fill_kind')}"
    if "c4" in d:
        s += f" | C4 {d['c4']['fill_ms']:.2f} ok {d['c4']['cost_matches_oracle']}"
    pin = (d["config"].get("traceback_pin") or {}).get("matches_oracle")
    print(s, "pin", pin, "cost_ok", d["config"].get("cost_matches_oracle"))
PY
bash tools/exp/r5/c4ab.sh
