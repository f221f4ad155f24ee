#!/bin/bash
# Quick GPU iteration for the fill kernel: parity tests, then stamps at C3 (2 waves/SIMD) and 50k (1 wave/SIMD).
mkdir -p gpurun_out
tag=${1:-x}
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -m gpu -q -x > gpurun_out/t_$tag.log 2>&1; rc=$?
tail -3 gpurun_out/t_$tag.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/fill_stamps.py 100000 100000 --tb > gpurun_out/s100_$tag.json 2>gpurun_out/s_$tag.err || exit 1
timeout -k 10 200 python tools/fill_stamps.py 50000 50000 --tb > gpurun_out/s50_$tag.json 2>>gpurun_out/s_$tag.err || exit 1
python - "$tag" <<'PY'
import json, sys
t = sys.argv[1]
for k in ("s100", "s50"):
    d = json.load(open(f"gpurun_out/{k}_{t}.json"))
    print(k, "fill_ms %.2f row_ns %.1f (min %.1f) cyc/row %.0f clk %.2f GHz lag_intra_us %.2f lag_cross_us %.2f ramp_us %.0f walk_ms %.2f rng_ms %.2f" % (
        d["fill_kernel_ms"], d["row_ns_median"], d["row_ns_min"], d["cycles_per_row_median"], d["clock_ghz_median"],
        d["lag_intra_slab_us"], d["lag_cross_slab_us"], d["last_stripe_start_us"], d["walk"]["walk_ms"], d["walk"]["rng_ms"]))
    print("   first stripes row_ns", ["%.0f" % x for x in d["first_stripes_row_ns"]])
PY
