set -o pipefail
# round 5: the chain head of the lane fills (stripe 0 and every workgroup's first stripe): duration, busy cycles per step
# and what it waited for -- C3 shape at TD 4 (the recompute fill's width), C4 (TD 8, two rounds), 1M x 125k (slab at N=8)
O=gpurun_out/r5_head
mkdir -p $O
run() {
  name=$1; shift
  env GA_FILL_MODE=lane "$@" LANE_STAMPS_DUMP=$O/raw_$name.npy timeout -k 10 300 python -u tools/lane_stamps.py $M $N > $O/stamps_$name.json 2> $O/stamps_$name.err || { tail -5 $O/stamps_$name.err; exit 1; }
  python3 - $name $M <<'PY'
import json, sys
import numpy as np
name, m = sys.argv[1], int(sys.argv[2])
st = np.load(f"gpurun_out/r5_head/raw_{name}.npy").astype(np.int64)
d = json.loads(open(f"gpurun_out/r5_head/stamps_{name}.json").read().strip().splitlines()[-1])
t0 = st[:, 0].min(); tot = np.maximum(st[:, 5], 1)
dur = (st[:, 1] - st[:, 0]) / 100.0
busy = (tot - st[:, 2] - st[:, 3] - st[:, 4]) / (m + 63)
print(name, "TD", d["TD"], "stripes", d["nstripes"], "fill_dbg", round(d["fill_ms_dbg"], 3), "last_end_us", d["last_end_us"])
for s in sorted({0, 1, 2, 3, 4, 5, d["nstripes"] // 2, d["nstripes"] - 1}):
    print(f"  stripe {s} dur_us {dur[s]:.1f} end_us {(st[s,1]-t0)/100:.1f} busy {busy[s]:.1f} wait edge/prof/space",
          [round(float(x), 4) for x in (st[s, 2] / tot[s], st[s, 3] / tot[s], st[s, 4] / tot[s])])
print("  median busy", round(float(np.median(busy)), 1), "median space wait", round(float(np.median(st[:, 4] / tot)), 4))
PY
}
M=100000 N=100000 run c3td4 GA_LANE_COLS_PER_LANE=4
M=1000000 N=125000 run slab125k GA_X=0
M=1000000 N=1000000 run c4 GA_X=0
