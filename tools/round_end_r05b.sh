set -o pipefail
# round 5, final tree: smoke, the default bench line (as the driver runs it), the C5 / C2 / C4-with-traceback lines,
# and the rocprof kernel stats of the default line (the GPU suite ran on this tree in tools/exp/r5/walk_pipe.sh)
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5_final
mkdir -p $O
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { tail -20 $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
timeout -k 10 300 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
for w in c5 c2; do
  timeout -k 10 200 python -u bench.py --workload $w --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_$w.json 2> $O/bench_$w.err || { tail -20 $O/bench_$w.err; exit 1; }
done
timeout -k 10 300 python -u bench.py --workload c4tb --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_c4tb.json 2> $O/bench_c4tb.err || { tail -20 $O/bench_c4tb.err; exit 1; }
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats_default -o run -- python3 $R/bench.py --no-cpu-baseline --no-extra --steps 20 --warmup 5 > $O/stats_default.log 2>&1 || { tail -20 $O/stats_default.log; exit 1; }
cp $(find $O/stats_default -name "*kernel_stats.csv" | head -1) $O/rocprof_default_kernel_stats.csv
head -4 $O/rocprof_default_kernel_stats.csv
cd $R
python3 - <<'PY'
import json
O = "gpurun_out/r5_final"
for f in ("bench_default", "bench_c5", "bench_c2", "bench_c4tb"):
    d = json.loads(open(f"{O}/{f}.json").read().strip().splitlines()[-1])
    r = d.get("roofline") or {}
    s = f"{f}: value {d['value']:.4g} ms/step {d['ms_per_step']:.3f} fill {d.get('fill_ms', 0):.3f} walk {d.get('walk_ms', 0):.3f} kind {d.get('fill_kind')} frac {r.get('frac')}"
    if "c4" in d:
        s += f" | C4 {d['c4']['fill_ms']:.2f} ok {d['c4']['cost_matches_oracle']} frac {d['c4']['roofline'].get('frac')}"
    pin = (d["config"].get("traceback_pin") or {}).get("matches_oracle")
    print(s, "pin", pin, "cost_ok", d["config"].get("cost_matches_oracle"))
PY
