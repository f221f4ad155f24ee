set -o pipefail
# round 5: raw lane stamps of the C5-shape fill (protein) and the same shape in DNA: per stripe waits (edges, profile,
# ring space) and durations, to see what holds the chain's head back at 24 codes
O=gpurun_out/r5_c5
mkdir -p $O
export GA_FILL_MODE=lane GA_LANE_COLS_PER_LANE=4
LANE_STAMPS_DUMP=$O/raw_c5.npy timeout -k 10 120 python -u tools/lane_stamps.py 20000 20000 c5 > $O/stamps_c5b.json 2> $O/stamps_c5b.err || { tail -5 $O/stamps_c5b.err; exit 1; }
LANE_STAMPS_DUMP=$O/raw_dna20k.npy timeout -k 10 120 python -u tools/lane_stamps.py 20000 20000 > $O/stamps_dna20kb.json 2> $O/stamps_dna20kb.err || { tail -5 $O/stamps_dna20kb.err; exit 1; }
python3 - <<'PY'
import numpy as np
for w in ("c5", "dna20k"):
    st = np.load(f"gpurun_out/r5_c5/raw_{w}.npy").astype(np.int64)
    t0 = st[:, 0].min()
    dur = (st[:, 1] - st[:, 0]) / 100.0
    tot = np.maximum(st[:, 5], 1)
    for s in (0, 1, 2, 3, 4, 40, 78):
        print(w, "stripe", s, "dur_us", round(dur[s], 1), "end_us", round((st[s, 1] - t0) / 100.0, 1),
              "wait edge/prof/space", [round(x, 3) for x in (st[s, 2] / tot[s], st[s, 3] / tot[s], st[s, 4] / tot[s])],
              "busy cyc/step", round((tot[s] - st[s, 2] - st[s, 3] - st[s, 4]) / 20063, 1))
PY
