"""Summarise tools/exp/r4/r4_*.sh runs: lane-stamp lags (C3 shape, 1M x 125k slab) and the C3 bench line per variant.

    python tools/exp/r4/r4_lagsum.py <dir> <variant> [<variant> ...]
"""
import json
import sys


def last_json(path):
    return json.loads(open(path).read().strip().splitlines()[-1])


def main():
    O, vs = sys.argv[1], sys.argv[2:]
    for v in vs:
        for w in ("c3", "slab"):
            d = last_json(f"{O}/stamps_{w}_{v}.json")
            ld = d["lag_distribution"]
            busy = [round(x["cyc_per_step_busy"], 1) for x in d["by_simd"].values()]
            print(f"{v} {w}: dbg {d['fill_ms_dbg']:.2f} plain {d['fill_ms_plain']:.2f} intra {d['end_lag_intra_wg_us']:.2f} "
                  f"cross {d['end_lag_cross_wg_us']:.2f} mean {d['end_lag_mean_us']:.2f} busy {busy} "
                  f"by_wave {[round(x, 2) for x in d['end_lag_by_wave_us'].values()]}")
            print(f"    pct {ld['end_lag_pct_us']} max {ld['end_lag_max_us']:.1f} sum {ld['end_lag_sum_ms']} "
                  f"links {ld['cross_wg_links']}")
        d = last_json(f"{O}/c3_{v}.json")
        print(f"{v} bench c3: call {d['ms_per_step']:.3f} fill {d['fill_ms']:.3f} walk {d['walk_ms']:.3f} "
              f"pin {d['config']['traceback_pin']['matches_oracle']} C4 {d['c4']['fill_ms']:.2f} "
              f"ok {d['c4']['cost_matches_oracle']}")


if __name__ == "__main__":
    main()
