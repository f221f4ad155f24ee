set -o pipefail
# round 4: why the lane fill's in-kernel step (112 cycles at TD 2) is far above the bare step (52-76 cycles in
# tools/micro/lane_fine): instruction-cache and issue counters of the C3-shape score-only lane fill
mkdir -p gpurun_out/r4_pmc
O=$GRAFT_REPO_ROOT/gpurun_out/r4_pmc
cd /tmp && export TMPDIR=/tmp
export GA_FILL_MODE=lane
for f in 0 1; do
  export GA_LANE_FINE=$f
  timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_VALU SQ_INSTS_SALU -d $O/f${f}_a -o run -- python3 $GRAFT_REPO_ROOT/tools/fill_score.py 100000 100000 2 > $O/f${f}_a.log 2>&1 || { tail -20 $O/f${f}_a.log; exit 1; }
  timeout -s KILL 90 rocprofv3 --pmc SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d $O/f${f}_b -o run -- python3 $GRAFT_REPO_ROOT/tools/fill_score.py 100000 100000 2 > $O/f${f}_b.log 2>&1 || { tail -20 $O/f${f}_b.log; exit 1; }
done
cd $GRAFT_REPO_ROOT
python3 - <<'PY'
import csv, glob, collections
for f in (0, 1):
    vals = collections.defaultdict(float)
    for p in ("a", "b"):
        for fn in glob.glob(f"gpurun_out/r4_pmc/f{f}_{p}/**/*counter_collection.csv", recursive=True):
            rows = [r for r in csv.DictReader(open(fn)) if "fill_lane_kernel" in r["Kernel_Name"]]
            last = max(int(r["Dispatch_Id"]) for r in rows)
            for r in rows:
                if int(r["Dispatch_Id"]) == last:
                    vals[r["Counter_Name"]] += float(r["Counter_Value"])
    print(f"fine {f}: " + ", ".join(f"{k} {v:.4g}" for k, v in sorted(vals.items())))
PY
