"""Per-dispatch counter values of a kernel from rocprofv3's SQLite output (rocprofv3 7.x writes
<dir>/<name>_results.db unless --output-format csv is given).

    python tools/rocpd_pmc.py <results.db> [kernel-substring]      -> {counter: value} of the kernel's last dispatch
"""
import json
import sqlite3
import sys


def last_dispatch(db, sub="fill_lane_kernel"):
    cur = sqlite3.connect(db).cursor()
    rows = cur.execute("select dispatch_id, name, counter_name, counter_value, duration from pmc_events").fetchall()
    rows = [r for r in rows if sub in (r[1] or "")]
    if not rows:
        return {}, None
    last = max(r[0] for r in rows)
    vals = {}
    for d, name, c, v, dur in rows:
        if d == last:
            vals[c] = vals.get(c, 0.0) + float(v)
            kname, kdur = name, dur
    return vals, {"kernel": kname, "duration_ns": kdur, "dispatch": last}


if __name__ == "__main__":
    v, meta = last_dispatch(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "fill_lane_kernel")
    print(json.dumps({"meta": meta, "counters": v}))
