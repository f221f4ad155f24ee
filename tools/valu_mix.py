#!/usr/bin/env python3
"""Static VALU op mix of a kernel's hottest loop (the assembly from `make -C globalign_amd/csrc asm`).

The fill is VALU-issue bound, and gfx950 issues VALU forms at different rates:
profiles/r02/valu_rate.txt (tools/micro/valu_rate.hip) measures 4 cycles per wave64 op per
SIMD for full-rate forms (v_add/sub_u32, v_and/or, v_min_i16) when two waves share a SIMD,
8 for v_min/max_i32, shifts and v_add_co, ~8.5 for three-source VOP3 forms.  The chip's issue
peak for THIS kernel's mix is then 1024 SIMDs x 2.4 GHz / (mean SIMD cycles per op), which is
what bench.py divides SQ_INSTS_VALU / kernel time by.

    python tools/valu_mix.py <asm.s> <kernel symbol> [--json out.json] [--skip-blocks-with v_cndmask]
"""
import argparse
import collections
import json
import re

# SIMD cycles per wave64 op with >= 2 waves per SIMD (profiles/r02/valu_rate.txt, per-wave column / 2)
MEASURED = {
    "v_min_i32": 4.02, "v_min_u32": 4.02, "v_max_i32": 4.02, "v_max_u32": 4.02, "v_sub_u32": 2.02,
    "v_add_u32": 2.02, "v_subrev_u32": 2.02, "v_and_b32": 2.02, "v_or_b32": 2.02, "v_xor_b32": 2.02,
    "v_min_i16": 2.02, "v_lshlrev_b32": 4.02, "v_lshrrev_b32": 4.02, "v_ashrrev_i32": 4.02,
    "v_add_co_u32": 4.02, "v_sub_i32": 4.23, "v_med3_i32": 4.24, "v_lshl_or_b32": 4.24, "v_or3_b32": 4.24,
    "v_pk_min_i16": 4.24, "v_pk_add_u16": 4.24, "v_cvt_pk_u16_u32": 4.24, "v_perm_b32": 4.24,
    "v_add3_u32": 4.24, "v_bfe_i32": 4.24, "v_bfe_u32": 4.24, "v_min3_i32": 4.24, "v_min3_u32": 4.24,
    "v_pk_min_u16": 4.24, "v_add_lshl_u32": 4.24, "v_pk_max_i16": 4.24,
    # DPP / SDWA forms are priced as themselves (the _dpp / _sdwa suffix is kept)
    "v_min_i32_dpp": 4.24, "v_mov_b32_dpp": 4.24, "v_mov_b32": 2.02, "v_add_u32_sdwa": 4.24,
}


def cost(op):
    base = op[:-4] if op.endswith("_e32") or op.endswith("_e64") else op
    if base in MEASURED:
        return MEASURED[base], True
    base = base[:-4] if base.endswith("_dpp") else base[:-5] if base.endswith("_sdwa") else base
    if base in MEASURED:
        return MEASURED[base], True
    return 4.02, False  # unmeasured forms priced as the common half-rate v_min_i32


def kernel_body(path, sym):
    lines = open(path).read().split("\n")
    start = next(k for k, l in enumerate(lines) if l.startswith(sym + ":"))
    end = next(k for k in range(start, len(lines)) if lines[k].startswith(".Lfunc_end"))
    return lines[start:end]


def drop_blocks_with(lines, op):
    """The loop's lines without the basic blocks (label to label) that contain `op`: the lane kernel's
    masked steps (v_cndmask) run in 4 of ~10^5 sub-chunks, so its executed mix is the fast path's."""
    out, block = [], []
    for l in lines:
        if re.match(r"^\.LBB\w+:", l) or re.match(r"^; %bb\.", l):
            if not any(x.strip().startswith(op) for x in block):
                out += block
            block = []
        block.append(l)
    if not any(x.strip().startswith(op) for x in block):
        out += block
    return out


def hottest_loop(body, skip_op=None):
    labels = {}
    for k, l in enumerate(body):
        mm = re.match(r"^(\.LBB\w+):", l)
        if mm:
            labels[mm.group(1)] = k
    best = None
    for k, l in enumerate(body):
        mm = re.match(r"^\s+s_(cbranch_\w+|branch)\s+(\.LBB\w+)", l)
        if mm and mm.group(2) in labels and labels[mm.group(2)] < k:
            lo = labels[mm.group(2)]
            seg = body[lo:k + 1] if skip_op is None else drop_blocks_with(body[lo:k + 1], skip_op)
            ops = [x.split()[0] for x in seg if x.strip().startswith("v_")]
            valu = [o for o in ops if not o.startswith(("v_readfirstlane", "v_readlane", "v_writelane"))]
            if best is None or len(valu) > len(best[2]):
                best = (lo, k, valu)
    return best


def asm_block_ops(body, op):
    """VALU ops of the largest inline-asm statement (;;#ASMSTART .. ;;#ASMEND) holding `op`: the lane kernel's lean
    sub-chunk (ga_lane_asm.h LaneSub), which is its whole steady-state step stream"""
    best, cur, inside = [], [], False
    for l in body:
        t = l.strip()
        if t.startswith(";;#ASMSTART"):
            inside, cur = True, []
        elif t.startswith(";;#ASMEND"):
            inside = False
            if any(x.startswith(op) for x in cur) and len(cur) > len(best):
                best = cur
        elif inside and t.startswith("v_"):
            cur.append(t.split()[0])
    return best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("asm")
    ap.add_argument("symbol")
    ap.add_argument("--json")
    ap.add_argument("--skip-blocks-with", default=None, help="drop basic blocks of the loop holding this op")
    ap.add_argument("--asm-block-with", default=None, help="price the largest inline-asm statement holding this op")
    a = ap.parse_args()
    if a.asm_block_with:
        lo, hi, ops = -1, -1, asm_block_ops(kernel_body(a.asm, a.symbol), a.asm_block_with)
    else:
        lo, hi, ops = hottest_loop(kernel_body(a.asm, a.symbol), a.skip_blocks_with)
    hist = collections.Counter(ops)
    cyc = sum(cost(o)[0] * c for o, c in hist.items())
    unmeasured = sorted({o for o in hist if not cost(o)[1]})
    mean = cyc / max(1, len(ops))
    out = {"symbol": a.symbol, "loop_lines": [lo, hi], "valu_ops_in_loop": len(ops),
           "simd_cycles_in_loop": cyc, "mean_simd_cycles_per_op": mean,
           "peak_valu_insts_per_s": 256 * 4 * 2.4e9 / mean, "unmeasured_forms_priced_at_v_min_i32": unmeasured,
           "skipped_blocks_with": a.skip_blocks_with, "asm_block_with": a.asm_block_with,
           "histogram": dict(hist.most_common())}
    print(json.dumps(out, indent=1))
    if a.json:
        json.dump(out, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
