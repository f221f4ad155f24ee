# round 2 (walk chain): full GPU suite, the default bench line, C5 / C2 lines, rocprofv3 kernel stats of the C5 line
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/rc/gpu_check.log 2>&1 || { tail -40 gpurun_out/rc/gpu_check.log; exit 1; }
tail -1 gpurun_out/rc/gpu_check.log
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/rc/bench_default.json 2> gpurun_out/rc/bench_default.err || { tail -20 gpurun_out/rc/bench_default.err; exit 1; }
for W in c5 c2; do
  timeout -k 10 200 python -u bench.py --workload $W --no-cpu-baseline --no-extra > gpurun_out/rc/bench_$W.json 2> gpurun_out/rc/bench_$W.err || { tail -20 gpurun_out/rc/bench_$W.err; exit 1; }
done
timeout -s KILL 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/rc/prof_c5 -o run -- python3 bench.py --workload c5 --no-cpu-baseline --no-extra > gpurun_out/rc/prof_c5.log 2>&1 || { tail -20 gpurun_out/rc/prof_c5.log; exit 1; }
python - <<'PY'
import json
for f in ["bench_default", "bench_c5", "bench_c2"]:
    d = json.load(open(f"gpurun_out/rc/{f}.json"))
    print(f, d["value"], round(d["ms_per_step"], 3), d["config"]["cost_matches_oracle"], d["config"].get("traceback_pin", {}).get("matches_oracle"))
PY
find gpurun_out/rc/prof_c5 -name "*stats*.csv" | sort
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()"
