"""Summarise a rocprofv3 SQ counter pass (SQ_INSTS_VALU, SQ_INSTS_SALU, SQ_INSTS_LDS, SQ_WAVES, ...) of the
fill kernel into profiles/<out>.json: instructions per launch (wave-instructions; the largest dispatch).

    python tools/pmc_valu.py <sq counter_collection.csv> <out.json> "<source>"
"""
import csv
import json
import sys

vals, name = {}, None
for r in csv.DictReader(open(sys.argv[1])):
    if not any(k in r["Kernel_Name"] for k in ("fill_kernel", "fill_diag_kernel", "fill_lane_kernel")):
        continue
    c, v = r["Counter_Name"], float(r["Counter_Value"])
    if v >= vals.get(c, 0.0):
        vals[c] = v
        name = r["Kernel_Name"]
out = {"source": sys.argv[3], "kernel": name, "units": "wave-instructions per launch (SQ counters summed over the chip)"}
out.update({k.lower() + "_per_launch": v for k, v in sorted(vals.items())})
json.dump(out, open(sys.argv[2], "w"), indent=1)
print(json.dumps(out))
