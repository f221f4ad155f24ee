"""Generate globalign_amd/csrc/ga_lane_asm.h: the lane-skewed fill's unmasked score-only step as hand-scheduled
gfx950 asm, one specialisation per (TD columns per lane, profile byte U, leading nop), and the
sub-chunk's row store from lane 63.

    python tools/gen_lane_asm.py [out]  (rewrites the header, or writes `out`; the build uses the committed copy,
                                         tests/test_host_cpu.py checks that it still matches this generator)

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


def sub_chunk(td, rs):
    """One whole 16-step sub-chunk of the score-only lane fill as one asm statement (LaneSub<TD, RS>):
      * the steps, with fresh registers X{s} / hn{s} per step (lane 63's row s stays in them);
      * after step 1 the next sub-chunk's profile dwords (2 ds_read2_b32 per column, qb{k}: the lane's window);
      * after step RS the producer's counter (ca) and then the next sub-chunk's 16 edge rows (8 ds_read_b128 at ea:
        lane 0 its input ring, lanes 1..63 the zero block);
      * lane 63's 16 rows moved into lanes 48..63 of four registers by v_mov_b32_dpp row_shl:(15-u) with a bank
        mask, bank by bank from its top lane down (each lane's last write is its own row): rows 0..7 while the
        later steps run, rows 8..15 at the end; banks 1 and 3 go to (Rha, Rxa), banks 0 and 2 to (Rhb, Rxb), so that
        no DPP waits on the previous write of its own destination;
      * two ds_write2_b32 of those rows (wa / wb: the ring slots of lanes 48..63 of the register's banks, a scratch
        slot for every other lane) and the counters {cons, prod} (wc, lane 0), all lanes active (no exec change);
      * one wait for the reads (the three writes may still be in flight).
    Every DPP reads registers written >= 2 VALU earlier (gfx950's wait states; the compiler does not look inside)."""
    def step(s):
        u = s % 4
        xl = "%[Xl]" if s == 0 else f"%[X{s - 1}]"
        hlp = "%[HLp]" if s == 0 else f"%[HLn{(s - 1) % 2}]"
        hlast = "%[Hlast]" if s == 0 else f"%[hn{s - 1}]"
        hd = [hlp] + [f"%[H{k}]" for k in range(td - 1)]
        out = [f"v_add_u32_sdwa %[M{k}], sext(%[q{k}_{s // 4}]), {hd[k]} dst_sel:DWORD dst_unused:UNUSED_PAD "
               f"src0_sel:BYTE_{u} src1_sel:DWORD" for k in range(td)]
        if td == 1 and s == 0:
            out.append("s_nop 1")
        out += [f"v_add_u32_dpp %[X{s}], {xl}, %[ex{s}] wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1",
                f"v_add_u32_dpp %[HLn{s % 2}], {hlast}, %[eh{s}] wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1"]
        for k in range(td):
            dst = f"%[hn{s}]" if k == td - 1 else f"%[H{k}]"
            out += [f"v_min3_i32 {dst}, %[M{k}], %[X{s}], %[Y{k}]", f"v_add_u32 %[T], %[o], {dst}",
                    f"v_min_i32 %[X{s}], %[X{s}], %[T]", f"v_min_i32 %[Y{k}], %[Y{k}], %[T]"]
        return out

    def tp(reg, val, u):
        b = u // 4
        ctl = "quad_perm:[0,1,2,3]" if u == 15 else f"row_shl:{15 - u}"
        return f"v_mov_b32_dpp %[{reg}], %[{val}{u}] {ctl} row_mask:0x8 bank_mask:{1 << b:#x}"

    def chain(b):
        ab = "a" if b & 1 else "b"
        out = []
        for i in (3, 2, 1, 0):
            u = 4 * b + i
            out += [tp("Rh" + ab, "hn", u), tp("Rx" + ab, "X", u)]
        return out

    lines = []
    for s in range(16):
        st = step(s)
        if s in (5, 6, 9, 10):
            # rows of block 0 (during steps 5-6) and block 1 (steps 9-10): four transposes per step, spread out
            blk = 0 if s < 8 else 1
            tps = chain(blk)[(s - 1) % 4 * 4 // 4 * 0 + (0 if s in (5, 9) else 4):][:4]
            per = max(1, len(st) // 5)
            out = []
            for i, ln in enumerate(st):
                out.append(ln)
                if tps and i >= 2 and (i - 2) % per == 0:
                    out.append(tps.pop(0))
            out += tps
            st = out
        lines += st
        if s == 1:
            for k in range(td):
                lines += [f"ds_read2_b32 %[qa{k}], %[qb{k}] offset0:0 offset1:4",
                          f"ds_read2_b32 %[qc{k}], %[qb{k}] offset0:8 offset1:12"]
        if s == rs:
            lines += ["ds_read_b32 %[cv], %[ca]"] + [f"ds_read_b128 %[E{k}], %[ea] offset:{16 * k}" for k in range(8)]
    # rows 8..15 (banks 2 and 3) at the end, the two register pairs interleaved
    b2, b3 = chain(2), chain(3)
    for i in range(8):
        lines += [b2[i], b3[i]]
    lines += ["ds_write2_b32 %[wa], %[Rha], %[Rxa] offset1:1", "ds_write2_b32 %[wb], %[Rhb], %[Rxb] offset1:1",
              "ds_write_b64 %[wc], %[cp]", "s_waitcnt lgkmcnt(3)"]
    body = "\n".join(f'        "{ln}\\n\\t"' for ln in lines[:-1]) + f'\n        "{lines[-1]}"'
    outs = [f'[X{s}] "=&v"(X[{s}])' for s in range(16)] + [f'[hn{s}] "=&v"(hn[{s}])' for s in range(16)] + \
           ['[HLn0] "=&v"(HLn[0])', '[HLn1] "=&v"(HLn[1])'] + [f'[H{k}] "+v"(H[{k}])' for k in range(td - 1)] + \
           [f'[Y{k}] "+v"(Y[{k}])' for k in range(td)] + ['[T] "=&v"(T)'] + [f'[M{k}] "=&v"(M[{k}])' for k in range(td)] + \
           ['[Rha] "=&v"(R[0])', '[Rxa] "=&v"(R[1])', '[Rhb] "=&v"(R[2])', '[Rxb] "=&v"(R[3])', '[cv] "=&v"(cv)'] + \
           [f'[E{k}] "=&v"(En[{k}])' for k in range(8)] + \
           [f'[qa{k}] "=&v"(qn[{k}][0])' for k in range(td)] + [f'[qc{k}] "=&v"(qn[{k}][1])' for k in range(td)]
    ins = ['[Xl] "v"(Xl)', '[HLp] "v"(HLp)', f'[Hlast] "v"(H[{td - 1}])', '[o] "s"(o)'] + \
          [f'[ex{s}] "v"(E[{s // 2}][{1 + 2 * (s % 2)}])' for s in range(16)] + \
          [f'[eh{s}] "v"(E[{s // 2}][{2 * (s % 2)}])' for s in range(16)] + \
          [f'[q{k}_{d}] "v"(q[{k}][{d}])' for k in range(td) for d in range(4)] + \
          ['[ca] "v"(ca)', '[ea] "v"(ea)', '[wa] "v"(wa)', '[wb] "v"(wb)', '[wc] "v"(wc)', '[cp] "v"(cp)'] + \
          [f'[qb{k}] "v"(qb[{k}])' for k in range(td)]
    return f"""template <>
struct LaneSub<{td}, {rs}> {{
    // E / q: this sub-chunk's edge rows (lane 0; 0 elsewhere) and profile dwords; En / qn / cv: the next sub-chunk's
    // (read after step {rs}) and the producer's counter read before them; R: lane 63's rows in lanes 48..63 (banks 1
    // and 3: R[0] / R[1] = H' / h1', banks 0 and 2: R[2] / R[3])
    __device__ __forceinline__ static void run(int (&H)[{td}], int (&Y)[{td}], int& Xl, int& HLp, const lk_v4i (&E)[8],
                                               const uint32_t (&q)[{td}][4], int o, unsigned ca, unsigned ea,
                                               const unsigned (&qb)[{td}], unsigned wa, unsigned wb, unsigned wc, lk_v2u cp,
                                               unsigned& cv, lk_v4i (&En)[8], lk_v2u (&qn)[{td}][2], int (&R)[4]) {{
        int X[16], hn[16], HLn[2], T, M[{td}];
        asm volatile(
{body}
        : {", ".join(outs)}
        : {", ".join(ins)}
        : "memory");
        H[{td - 1}] = hn[15];
        Xl = X[15];
        HLp = HLn[1];
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


def main(out=OUT):
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
template <int TD, int RS>
struct LaneSub;
"""]
    for td in (1, 2, 4, 8):
        for u0 in range(4):
            for n in range(1, 5 - u0):
                parts.append(block(td, u0, n))
    for td in (1, 2, 4, 8):
        for rs in (0, 12):
            parts.append(sub_chunk(td, rs))
    parts.append(store_rows())
    parts.append("}  // namespace ga\n")
    with open(out, "w") as f:
        f.write("\n".join(parts))
    print(out)


if __name__ == "__main__":
    import sys
    if len(sys.argv) > 1 and sys.argv[1].startswith("-"):
        sys.exit(__doc__)  # (an option is not an output path)
    main(sys.argv[1] if len(sys.argv) > 1 else OUT)
