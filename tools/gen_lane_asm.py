"""Generate globalign_amd/csrc/ga_lane_asm.h: the lane-skewed fill's unmasked score-only step as hand-scheduled
gfx950 asm, one specialisation per (TD columns per lane, profile byte U, leading nop), and the
sub-chunk's row store from lane 63.

    python tools/gen_lane_asm.py        (rewrites the header; the build uses the committed copy)

A step of TD columns (the same int32 recurrence as ga_lane.h lane_step, Ho form):
    M_k  = Hd_k + sub'(a_i, b_j)      Hd_0 = HLp (the left lane's H' of the step before), Hd_k = H_{k-1}
    X    = h1'(i, left)  (v_add_u32_dpp: the left lane's h1' shifted in, zero-filled in lane 0, plus the edge
                          register ex, which holds the stripe's left edge in lane 0 and 0 in lanes 1..63)
    HLn  = H'(i, left)   (the same with eh: the next step's diagonal)
One VALU each and a fresh destination: the compiler's form copied the edge into the DPP's destination first
(v_mov, then an s_nop for the old-operand hazard).
    per column k: H_k = min3(M_k, X, Y_k); T = H_k + o; X = min(X, T); Y_k = min(Y_k, T)
The last column's H' goes to a fresh register hn, so lane 63's (hn, X) of every step of a sub-chunk stay in
registers until lk_store_rows writes them to the output ring.  A step computes every M' before its DPPs, so >= 2
instructions separate any VALU write from a DPP that reads it (the DPPs' wait states on gfx950; the compiler
does not look inside asm): at TD >= 2 the M's alone, at TD = 1 M0 and an s_nop 0.  Up to four consecutive steps
(the same profile dwords) form one asm statement: between statements the compiler pads an s_nop of its own.
"""
import os

HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, "..", "globalign_amd", "csrc", "ga_lane_asm.h")


def block(td, u0, n):
    """n consecutive steps (profile bytes u0 .. u0+n-1 of the same dwords) in one asm statement."""
    lines = []
    for s in range(n):
        u = u0 + s
        sel = f"BYTE_{u}"
        xl = "%[Xl]" if s == 0 else f"%[X{s - 1}]"
        hlp = "%[HLp]" if s == 0 else f"%[HLn{s - 1}]"
        hlast = "%[Hlast]" if s == 0 else f"%[hn{s - 1}]"
        hd = [hlp] + [f"%[H{k}]" for k in range(td - 1)]
        for k in range(td):
            lines.append(f"v_add_u32_sdwa %[M{k}], sext(%[q{k}]), {hd[k]} dst_sel:DWORD dst_unused:UNUSED_PAD "
                         f"src0_sel:{sel} src1_sel:DWORD")
        if td == 1 and s == 0:
            lines.append("s_nop 0")  # M0 alone does not cover the DPPs' two wait states after compiler code
        # the left lane's value shifted in, plus the edge register (0 in lanes 1..63, the left edge in lane 0)
        lines.append(f"v_add_u32_dpp %[X{s}], {xl}, %[ex{s}] wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1")
        lines.append(f"v_add_u32_dpp %[HLn{s}], {hlast}, %[eh{s}] wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1")
        for k in range(td):
            dst = f"%[hn{s}]" if k == td - 1 else f"%[H{k}]"
            lines.append(f"v_min3_i32 {dst}, %[M{k}], %[X{s}], %[Y{k}]")
            lines.append(f"v_add_u32 %[T], %[o], {dst}")
            lines.append(f"v_min_i32 %[X{s}], %[X{s}], %[T]")
            lines.append(f"v_min_i32 %[Y{k}], %[Y{k}], %[T]")
    body = "\n".join(f'        "{ln}\\n\\t"' for ln in lines[:-1]) + f'\n        "{lines[-1]}"'
    outs = [f'[X{s}] "=&v"(X[{s}])' for s in range(n)] + [f'[HLn{s}] "=&v"(HLn[{s}])' for s in range(n)] + \
           [f'[hn{s}] "=&v"(hn[{s}])' for s in range(n)] + [f'[H{k}] "+v"(H[{k}])' for k in range(td - 1)] + \
           [f'[Y{k}] "+v"(Y[{k}])' for k in range(td)] + ['[T] "=&v"(T)'] + [f'[M{k}] "=&v"(M[{k}])' for k in range(td)]
    ins = ['[Xl] "v"(Xl)', '[HLp] "v"(HLp)', f'[Hlast] "v"(H[{td - 1}])'] + \
          [f'[ex{s}] "v"(ex[{s}])' for s in range(n)] + [f'[eh{s}] "v"(eh[{s}])' for s in range(n)] + \
          [f'[q{k}] "v"(q[{k}])' for k in range(td)] + ['[o] "s"(o)']
    return f"""template <>
struct LaneAsm<{td}, {u0}, {n}> {{
    // steps with profile bytes {u0} .. {u0 + n - 1}; ex / eh: the steps' edge registers; oh / ox: lane 63's rows out
    __device__ __forceinline__ static void run(int (&H)[{td}], int (&Y)[{td}], int& Xl, int& HLp, const int* eh,
                                               const int* ex, const uint32_t (&q)[{td}], int o, int* oh, int* ox) {{
        int X[{n}], HLn[{n}], hn[{n}], T, M[{td}];
        asm volatile(
{body}
        : {", ".join(outs)}
        : {", ".join(ins)});
        H[{td - 1}] = hn[{n - 1}];
        Xl = X[{n - 1}];
        HLp = HLn[{n - 1}];
#pragma unroll
        for (int s = 0; s < {n}; s++) {{
            oh[s] = hn[s];
            ox[s] = X[s];
        }}
    }}
}};
"""


def fine_block(td):
    """One 4-step block of the fine-grained hand-over: step 0, then the producer's counter and the next block's
    edge rows read from LDS (ca / ea: their addresses), steps 1 .. 3, and a wait for the reads, all in one asm
    statement, so that no compiler code can touch the loads' registers before they land."""
    lines = []
    for s in range(4):
        xl = "%[Xl]" if s == 0 else f"%[X{s - 1}]"
        hlp = "%[HLp]" if s == 0 else f"%[HLn{s - 1}]"
        hlast = "%[Hlast]" if s == 0 else f"%[hn{s - 1}]"
        hd = [hlp] + [f"%[H{k}]" for k in range(td - 1)]
        for k in range(td):
            lines.append(f"v_add_u32_sdwa %[M{k}], sext(%[q{k}]), {hd[k]} dst_sel:DWORD dst_unused:UNUSED_PAD "
                         f"src0_sel:BYTE_{s} src1_sel:DWORD")
        if td == 1 and s == 0:
            lines.append("s_nop 0")
        lines.append(f"v_add_u32_dpp %[X{s}], {xl}, %[ex{s}] wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1")
        lines.append(f"v_add_u32_dpp %[HLn{s}], {hlast}, %[eh{s}] wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1")
        for k in range(td):
            dst = f"%[hn{s}]" if k == td - 1 else f"%[H{k}]"
            lines.append(f"v_min3_i32 {dst}, %[M{k}], %[X{s}], %[Y{k}]")
            lines.append(f"v_add_u32 %[T], %[o], {dst}")
            lines.append(f"v_min_i32 %[X{s}], %[X{s}], %[T]")
            lines.append(f"v_min_i32 %[Y{k}], %[Y{k}], %[T]")
        if s == 0:
            lines += ["ds_read_b32 %[cv], %[ca]", "ds_read_b128 %[N0], %[ea]", "ds_read_b128 %[N1], %[ea] offset:16"]
    lines.append("s_waitcnt lgkmcnt(0)")
    body = "\n".join(f'        "{ln}\\n\\t"' for ln in lines[:-1]) + f'\n        "{lines[-1]}"'
    outs = [f'[X{s}] "=&v"(X[{s}])' for s in range(4)] + [f'[HLn{s}] "=&v"(HLn[{s}])' for s in range(4)] + \
           [f'[hn{s}] "=&v"(hn[{s}])' for s in range(4)] + [f'[H{k}] "+v"(H[{k}])' for k in range(td - 1)] + \
           [f'[Y{k}] "+v"(Y[{k}])' for k in range(td)] + ['[T] "=&v"(T)'] + [f'[M{k}] "=&v"(M[{k}])' for k in range(td)] + \
           ['[cv] "=&v"(cv)', '[N0] "=&v"(N0)', '[N1] "=&v"(N1)']
    ins = ['[Xl] "v"(Xl)', '[HLp] "v"(HLp)', f'[Hlast] "v"(H[{td - 1}])'] + \
          [f'[ex{s}] "v"(ex[{s}])' for s in range(4)] + [f'[eh{s}] "v"(eh[{s}])' for s in range(4)] + \
          [f'[q{k}] "v"(q[{k}])' for k in range(td)] + ['[o] "s"(o)', '[ca] "v"(ca)', '[ea] "v"(ea)']
    return f"""template <>
struct LaneBlk<{td}> {{
    // four steps (profile bytes 0 .. 3) with the fine hand-over's reads after the first: cv = the producer's
    // counter (LDS address ca), N0 / N1 = the next block's four edge rows (ea); oh / ox: lane 63's rows out
    __device__ __forceinline__ static void run(int (&H)[{td}], int (&Y)[{td}], int& Xl, int& HLp, const int* eh,
                                               const int* ex, const uint32_t (&q)[{td}], int o, int* oh, int* ox,
                                               unsigned ca, unsigned ea, unsigned& cv, lk_v4i& N0, lk_v4i& N1) {{
        int X[4], HLn[4], hn[4], T, M[{td}];
        asm volatile(
{body}
        : {", ".join(outs)}
        : {", ".join(ins)}
        : "memory");
        H[{td - 1}] = hn[3];
        Xl = X[3];
        HLp = HLn[3];
#pragma unroll
        for (int s = 0; s < 4; s++) {{
            oh[s] = hn[s];
            ox[s] = X[s];
        }}
    }}
}};
"""


def store_rows():
    lines = ["s_mov_b64 %[saved], exec", "s_mov_b64 exec, %[m63]"]
    for u in range(15):
        lines.append(f"ds_write2_b32 %[b1], %[h{u}], %[x{u}] offset0:{2 * u} offset1:{2 * u + 1}")
    lines.append("ds_write2_b32 %[b2], %[h15], %[x15] offset1:1")
    lines += ["s_mov_b64 exec, 1", "ds_write_b64 %[pc], %[cp]", "s_mov_b64 exec, %[saved]", "s_nop 4"]
    body = "\n".join(f'        "{ln}\\n\\t"' for ln in lines[:-1]) + f'\n        "{lines[-1]}"'
    ins = ['[b1] "v"(b1)', '[b2] "v"(b2)', '[pc] "v"(pc)', '[cp] "v"(cp)', '[m63] "s"(m63)'] + \
          [f'[h{u}] "v"(h[{u}])' for u in range(16)] + [f'[x{u}] "v"(x[{u}])' for u in range(16)]
    return f"""// Lane 63's 16 rows of a sub-chunk (h[u], x[u]: the H' and h1' of step u) into the output ring, then lane 0's
// counters {{cons, prod}}: rows u < 15 at LDS address b1 + 8u, row 15 at b2 (its slot may wrap past the ring's
// end); LDS executes a wave's operations in order, so the rows land before the counters
__device__ __forceinline__ void lk_store_rows(unsigned b1, unsigned b2, unsigned pc, lk_v2u cp, const int (&h)[16],
                                              const int (&x)[16]) {{
    const unsigned long long m63 = 1ull << 63;
    unsigned long long saved;
    asm volatile(
{body}
        : [saved] "=&s"(saved)
        : {", ".join(ins)}
        : "memory");
}}
"""


def store_rows4(d):
    lines = ["s_mov_b64 %[saved], exec", "s_mov_b64 exec, %[m63]"]
    for u in range(4):
        r = 4 * d + u
        if r < 15:
            lines.append(f"ds_write2_b32 %[b1], %[h{u}], %[x{u}] offset0:{2 * r} offset1:{2 * r + 1}")
        else:
            lines.append(f"ds_write2_b32 %[b2], %[h{u}], %[x{u}] offset1:1")
    lines += ["ds_write_b64 %[pc], %[cp]", "s_mov_b64 exec, %[saved]", "s_nop 4"]
    body = "\n".join(f'        "{ln}\\n\\t"' for ln in lines[:-1]) + f'\n        "{lines[-1]}"'
    ins = ['[b1] "v"(b1)', '[b2] "v"(b2)', '[pc] "v"(pc)', '[cp] "v"(cp)', '[m63] "s"(m63)'] + \
          [f'[h{u}] "v"(h[{u}])' for u in range(4)] + [f'[x{u}] "v"(x[{u}])' for u in range(4)]
    return f"""template <>
__device__ __forceinline__ void lk_store_rows4<{d}>(unsigned b1, unsigned b2, unsigned pc, lk_v2u cp, const int* h,
                                                  const int* x) {{
    const unsigned long long m63 = 1ull << 63;
    unsigned long long saved;
    asm volatile(
{body}
        : [saved] "=&s"(saved)
        : {", ".join(ins)}
        : "memory");
}}
"""


def store_rows4_decl():
    return """// Lane 63's 4 rows of block D of a sub-chunk (h[u], x[u]: the H' and h1' of step 4D + u) into the output ring,
// then the counters {cons, prod} (lane 63 writes them too, so one exec mask): the sub-chunk's rows r < 15 at LDS
// address b1 + 8r, row 15 at b2 (its slot may wrap past the ring's end); the fine-grained hand-over of the asm
// sub-chunks (ga_lane.hip)
template <int D>
__device__ __forceinline__ void lk_store_rows4(unsigned b1, unsigned b2, unsigned pc, lk_v2u cp, const int* h,
                                               const int* x);
"""


def main():
    parts = ["""// ga_lane_asm.h -- GENERATED by tools/gen_lane_asm.py (do not edit): the lane-skewed fill's unmasked
// score-only step as hand-scheduled gfx950 asm (DESIGN.md 5.6) and the sub-chunk's row store.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "ga_lane.h"

namespace ga {

template <int TD, int U0, int N>
struct LaneAsm;
typedef int lk_v4i __attribute__((ext_vector_type(4)));
template <int TD>
struct LaneBlk;
"""]
    for td in (1, 2, 4, 8):
        for u0 in range(4):
            for n in range(1, 5 - u0):
                parts.append(block(td, u0, n))
    for td in (1, 2, 4, 8):
        parts.append(fine_block(td))
    parts.append(store_rows())
    parts.append(store_rows4_decl())
    for d in range(4):
        parts.append(store_rows4(d))
    parts.append("}  // namespace ga\n")
    with open(OUT, "w") as f:
        f.write("\n".join(parts))
    print(OUT)


if __name__ == "__main__":
    main()
