"""Generate tools/micro/lane_ilv.hip: does interleaving the lane fill's per-sub-chunk LDS traffic into the step's
VALU stream hide it?  (tools/micro/lane_parts.hip prices the parts when grouped.)

One 16-step sub-chunk = 16 steps of the kernel's asm step (ga_lane_asm.h form) plus its LDS traffic:
  * 1 counter read (ds_read_b32) + 8 ds_read_b128 edge reads for the next sub-chunk (lane 0 its ring rows,
    lanes 1..63 a zero block),
  * 2 ds_read2_b32 per column: the next sub-chunk's profile dwords,
  * 16 ds_write2_b32 of lane 63's rows + 1 ds_write_b64 of the counters.
Variants (cycles per step per wave, one wave per SIMD, 256 workgroups of 4 waves):
  G  grouped: the steps, then the reads, then the writes under an exec mask (lane 63 only), as the kernel does
  I  interleaved: every LDS instruction inside the step stream (the writes from all lanes: lane 63 to the ring,
     the others to a scratch area, so no exec change), row u written during step u + 2
  B  bare steps (no LDS)

    python tools/micro/gen_lane_ilv.py && hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/micro/lane_ilv.hip \
        -o tools/micro/lane_ilv
"""
import os

HERE = os.path.dirname(os.path.abspath(__file__))


def step_lines(td, s, u):
    """VALU of step s (profile byte u) as (before_dpp, dpp, rest) line lists (operand names as in gen_lane_asm)."""
    xl = "%[Xl]" if s == 0 else f"%[X{(s - 1) % 2}]"
    hlp = "%[HLp]" if s == 0 else f"%[HLn{(s - 1) % 2}]"
    hlast = f"%[H{td - 1}]"
    hd = [hlp] + [f"%[H{k}]" for k in range(td - 1)]
    a = [f"v_add_u32_sdwa %[M{k}], sext(%[q{k}_{s // 4}]), {hd[k]} dst_sel:DWORD dst_unused:UNUSED_PAD "
         f"src0_sel:BYTE_{u} src1_sel:DWORD" for k in range(td)]
    if td == 1:
        a.append("s_nop 0")
    b = [f"v_add_u32_dpp %[X{s % 2}], {xl}, %[ex{s}] wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1",
         f"v_add_u32_dpp %[HLn{s % 2}], {hlast}, %[eh{s}] wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1"]
    c = []
    for k in range(td):
        dst = f"%[H{k}]"
        c += [f"v_min3_i32 {dst}, %[M{k}], %[X{s % 2}], %[Y{k}]", f"v_add_u32 %[T], %[o], {dst}",
              f"v_min_i32 %[X{s % 2}], %[X{s % 2}], %[T]", f"v_min_i32 %[Y{k}], %[Y{k}], %[T]"]
    # lane 63's row of this step: (H[td-1], X) copied out for the store (1 full-rate move each)
    c += [f"v_mov_b32 %[oh{s}], %[H{td - 1}]", f"v_mov_b32 %[ox{s}], %[X{s % 2}]"]
    return a, b, c


def step_fresh(td, s, u):
    """step s with fresh registers X{s}, HLn{s}, hn{s} (the gen_lane_asm form: lane 63's row stays in hn{s}, X{s})"""
    xl = "%[Xl]" if s == 0 else f"%[X{s - 1}]"
    hlp = "%[HLp]" if s == 0 else f"%[HLn{s - 1}]"
    hlast = f"%[H{td - 1}]" if s == 0 else f"%[hn{s - 1}]"
    hd = [hlp] + [f"%[H{k}]" for k in range(td - 1)]
    out = [f"v_add_u32_sdwa %[M{k}], sext(%[q{k}_{s // 4}]), {hd[k]} dst_sel:DWORD dst_unused:UNUSED_PAD "
           f"src0_sel:BYTE_{u} src1_sel:DWORD" for k in range(td)]
    if td == 1 and s == 0:
        out.append("s_nop 0")
    out += [f"v_add_u32_dpp %[X{s}], {xl}, %[ex{s}] wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1",
            f"v_add_u32_dpp %[HLn{s}], {hlast}, %[eh{s}] wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1"]
    for k in range(td):
        dst = f"%[hn{s}]" if k == td - 1 else f"%[H{k}]"
        out += [f"v_min3_i32 {dst}, %[M{k}], %[X{s}], %[Y{k}]", f"v_add_u32 %[T], %[o], {dst}",
                f"v_min_i32 %[X{s}], %[X{s}], %[T]", f"v_min_i32 %[Y{k}], %[Y{k}], %[T]"]
    return out


def transpose():
    """lane 63's rows hn{u} / X{u} into lanes 48+u of Rh / Rx (row_shl by 15-u inside row 3, bank by bank from the
    top lane down, so that each lane's last write is its own row)"""
    out = ["s_nop 1"]
    for b in (3, 2, 1, 0):
        for i in (3, 2, 1, 0):
            u = 4 * b + i
            ctl = "quad_perm:[0,1,2,3]" if u == 15 else f"row_shl:{15 - u}"
            out += [f"v_mov_b32_dpp %[Rh], %[hn{u}] {ctl} row_mask:0x8 bank_mask:{1 << b:#x}",
                    f"v_mov_b32_dpp %[Rx], %[X{u}] {ctl} row_mask:0x8 bank_mask:{1 << b:#x}", "s_nop 0"]
    return out


def kernel_n(td, parts="PET"):
    """P: profile reads, E: counter + edge reads, T: transposed publish"""
    lines = []
    for s in range(16):
        lines += step_fresh(td, s, s % 4)
        if s == 1 and "P" in parts:
            for k in range(td):
                lines += [f"ds_read2_b32 %[qa{k}], %[qb{k}] offset0:0 offset1:4",
                          f"ds_read2_b32 %[qc{k}], %[qb{k}] offset0:8 offset1:12"]
        if s == 12 and "E" in parts:
            lines += ["ds_read_b32 %[cv], %[ca]"] + [f"ds_read_b128 %[E{k}], %[ea] offset:{16 * k}" for k in range(8)]
    if "T" in parts:
        lines += transpose()
        lines += ["ds_write2_b32 %[wa], %[Rh], %[Rx] offset1:1", "ds_write_b64 %[wc], %[cp]", "s_waitcnt lgkmcnt(2)"]
    else:
        lines += ["s_waitcnt lgkmcnt(0)"]
    body = "\n".join(f'        "{ln}\\n\\t"' for ln in lines[:-1]) + f'\n        "{lines[-1]}"'
    outs = [f'[X{s}] "=&v"(X[{s}])' for s in range(16)] + [f'[HLn{s}] "=&v"(HLn[{s}])' for s in range(16)] + \
           [f'[hn{s}] "=&v"(oh[{s}])' for s in range(16)] + [f'[H{k}] "+v"(H[{k}])' for k in range(td)] + \
           [f'[Y{k}] "+v"(Y[{k}])' for k in range(td)] + ['[T] "=&v"(T)'] + [f'[M{k}] "=&v"(M[{k}])' for k in range(td)] + \
           ['[Rh] "+v"(Rh)', '[Rx] "+v"(Rx)', '[cv] "=&v"(cv)'] + [f'[E{k}] "=&v"(En[{k}])' for k in range(8)] + \
           [f'[qa{k}] "=&v"(qn[{k}][0])' for k in range(td)] + [f'[qc{k}] "=&v"(qn[{k}][1])' for k in range(td)]
    ins = ['[Xl] "v"(Xl)', '[HLp] "v"(HLp)', '[o] "s"(o)'] + \
          [f'[ex{s}] "v"(E[{s // 2}][{1 + 2 * (s % 2)}])' for s in range(16)] + \
          [f'[eh{s}] "v"(E[{s // 2}][{2 * (s % 2)}])' for s in range(16)] + \
          [f'[q{k}_{d}] "v"(q[{k}][{d}])' for k in range(td) for d in range(4)] + \
          ['[ca] "v"(ca)', '[ea] "v"(ea)', '[wa] "v"(wa)', '[wc] "v"(wc)', '[cp] "v"(cp)'] + \
          [f'[qb{k}] "v"(qb[{k}])' for k in range(td)]
    return body, outs, ins


def kernel(td, variant):
    if variant[0] == "N":
        return kernel_n(td, variant[1:] or "PET")
    lines = []
    reads = ["ds_read_b32 %[cv], %[ca]"] + [f"ds_read_b128 %[E{k}], %[ea] offset:{16 * k}" for k in range(8)]
    qreads = []
    for k in range(td):
        qreads += [f"ds_read2_b32 %[qa{k}], %[qb{k}] offset0:0 offset1:4",
                   f"ds_read2_b32 %[qc{k}], %[qb{k}] offset0:8 offset1:12"]
    writes = [f"ds_write2_b32 %[wa], %[oh{u}], %[ox{u}] offset0:{2 * u} offset1:{2 * u + 1}" for u in range(16)]
    cwrite = "ds_write_b64 %[wc], %[cp]"
    ilv = {}  # step -> LDS lines inserted after the step's DPPs
    if variant == "I":
        pend = reads + qreads
        for s in range(16):
            ins = []
            if s >= 0 and pend:
                ins += pend[:3]
                pend = pend[3:]
            if s >= 2:
                ins.append(writes[s - 2])
            ilv[s] = ins
    for s in range(16):
        a, b, c = step_lines(td, s, s % 4)
        lines += a + b
        if variant == "I":
            # spread this step's LDS instructions through its VALU (after the DPPs, between the column updates)
            ins = ilv.get(s, [])
            per = max(1, len(c) // (len(ins) + 1))
            out = []
            for i, ln in enumerate(c):
                out.append(ln)
                if ins and (i + 1) % per == 0:
                    out.append(ins.pop(0))
            out += ins
            lines += out
        else:
            lines += c
    if variant == "I":
        lines += [writes[14], writes[15], cwrite, "s_waitcnt lgkmcnt(3)"]
    elif variant == "G":
        lines += reads + qreads + ["s_mov_b64 %[sv], exec", "s_mov_b64 exec, %[m63]"] + writes + \
                 [cwrite, "s_mov_b64 exec, %[sv]", "s_waitcnt lgkmcnt(0)", "s_nop 4"]
    body = "\n".join(f'        "{ln}\\n\\t"' for ln in lines[:-1]) + f'\n        "{lines[-1]}"'
    outs = [f'[X{i}] "=&v"(X[{i}])' for i in range(2)] + [f'[HLn{i}] "=&v"(HLn[{i}])' for i in range(2)] + \
           [f'[H{k}] "+v"(H[{k}])' for k in range(td)] + [f'[Y{k}] "+v"(Y[{k}])' for k in range(td)] + \
           ['[T] "=&v"(T)'] + [f'[M{k}] "=&v"(M[{k}])' for k in range(td)] + \
           [f'[oh{u}] "=&v"(oh[{u}])' for u in range(16)] + [f'[ox{u}] "=&v"(ox[{u}])' for u in range(16)]
    if variant != "B":
        outs += ['[cv] "=&v"(cv)'] + [f'[E{k}] "=&v"(En[{k}])' for k in range(8)] + \
                [f'[qa{k}] "=&v"(qn[{k}][0])' for k in range(td)] + [f'[qc{k}] "=&v"(qn[{k}][1])' for k in range(td)]
    if variant == "G":
        outs.append('[sv] "=&s"(sv)')
    ins = ['[Xl] "v"(Xl)', '[HLp] "v"(HLp)', '[o] "s"(o)'] + \
          [f'[ex{s}] "v"(E[{s // 2}][{1 + 2 * (s % 2)}])' for s in range(16)] + \
          [f'[eh{s}] "v"(E[{s // 2}][{2 * (s % 2)}])' for s in range(16)] + \
          [f'[q{k}_{d}] "v"(q[{k}][{d}])' for k in range(td) for d in range(4)]
    if variant != "B":
        ins += ['[ca] "v"(ca)', '[ea] "v"(ea)', '[wa] "v"(wa)', '[wc] "v"(wc)', '[cp] "v"(cp)'] + \
               [f'[qb{k}] "v"(qb[{k}])' for k in range(td)]
    if variant == "G":
        ins.append('[m63] "s"(m63)')
    return body, outs, ins


def main():
    out = ['''// GENERATED by tools/micro/gen_lane_ilv.py (see its docstring)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v2i __attribute__((ext_vector_type(2)));
constexpr int LDSW = 12288;
''']
    for td in (1, 2, 4):
        for var in ("B", "G", "I", "N", "NPE", "NPT", "NET", "NT", "NE", "NP", "N-"):
            body, outs, ins = kernel(td, var)
            out.append(f'''
__global__ void __launch_bounds__(256) k_{var.replace("-", "0")}_{td}(long long* res, int* sink, int nsteps, int o) {{
    __shared__ __attribute__((aligned(16))) int lds[LDSW];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (int k = threadIdx.x; k < LDSW; k += blockDim.x) lds[k] = k < 4096 ? (k * 37) & 0x03030303 : (k < 6144 ? k : 0);
    __syncthreads();
    int H[{td}], Y[{td}], M[{td}], X[16], HLn[16], T, oh[16], ox[16], Rh = 0, Rx = 0;
    for (int k = 0; k < {td}; k++) {{ H[k] = lane + k; Y[k] = lane + 2 * k + 1; }}
    int Xl = lane + 3, HLp = lane + 1;
    v4i E[8], En[8];
    for (int k = 0; k < 8; k++) E[k] = v4i{{0, 0, 0, 0}};
    uint32_t q[{td}][4];
    v2i qn[{td}][2];
    for (int k = 0; k < {td}; k++) for (int d = 0; d < 4; d++) q[k][d] = 0x01020304u * ((lane + k + d) & 3);
    unsigned cv = 0;
    auto la = [](const int* p) {{ return (unsigned)(uintptr_t)(__attribute__((address_space(3))) const int*)p; }};
    const unsigned ca = la(lds + 8192 + 16 * ((w + 3) & 3));
    const unsigned wc = lane == 63 ? la(lds + 8192 + 16 * w) : la(lds + 9216 + 2 * lane);
    const v2i cp = v2i{{1, 2}};
    const unsigned long long m63 = 1ull << 63;
    unsigned long long sv;
    int acc = 0;
    long long t0 = __builtin_amdgcn_s_memtime();
    for (int r = 0; r < nsteps; r += 16) {{
        const unsigned ea = lane == 0 ? la(lds + 4096 + 512 * w + ((2 * r) & 255)) : la(lds + 6144);
        const unsigned wa = {"lane >= 48 ? la(lds + 4096 + 512 * ((w + 1) & 3) + ((2 * (r + lane)) & 511)) : la(lds + 9216 + 2 * lane)" if var[0] == "N" else "lane == 63 ? la(lds + 4096 + 512 * ((w + 1) & 3) + ((2 * r) & 255)) : la(lds + 9216 + 2 * lane)"};
        unsigned qb[{td}];
        for (int k = 0; k < {td}; k++) qb[k] = la(lds + ((((r + 16 - lane) & 1023) + 1031 * ((lane * 7 + k) & 3)) & 4095));
        (void)ea; (void)wa; (void)qb; (void)wc; (void)m63; (void)sv;
        asm volatile(
{body}
        : {", ".join(outs)}
        : {", ".join(ins)}
        : "memory");
        Xl = X[{1 if var[0] != "N" else 15}];
        HLp = HLn[{1 if var[0] != "N" else 15}];
        {"H[" + str(td - 1) + "] = oh[15]; acc ^= Rh + Rx;" if var[0] == "N" else ""}
        {"for (int k = 0; k < 8; k++) E[k] = En[k]; for (int k = 0; k < " + str(td) + "; k++) { q[k][0] = qn[k][0].x; q[k][1] = qn[k][0].y; q[k][2] = qn[k][1].x; q[k][3] = qn[k][1].y; } acc += (int)cv;" if var != "B" else "acc ^= oh[7] + ox[15];"}
    }}
    long long t1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) res[blockIdx.x * 16 + w] = t1 - t0;
    int z = Xl + HLp + acc;
    for (int k = 0; k < {td}; k++) z += H[k] + Y[k];
    sink[blockIdx.x * blockDim.x + threadIdx.x] = z;
}}
''')
    out.append('''
template <typename F>
double run(F kern, int n) {
    long long* d;
    int* s;
    (void)hipMalloc(&d, 16 * 256 * sizeof(long long));
    (void)hipMalloc(&s, 256 * 256 * sizeof(int));
    kern<<<256, 256>>>(d, s, n, 5);
    kern<<<256, 256>>>(d, s, n, 5);
    (void)hipDeviceSynchronize();
    std::vector<long long> h(16 * 256);
    (void)hipMemcpy(h.data(), d, h.size() * 8, hipMemcpyDeviceToHost);
    std::vector<double> v;
    for (int b = 0; b < 256; b++)
        for (int w = 0; w < 4; w++) v.push_back((double)h[b * 16 + w]);
    std::sort(v.begin(), v.end());
    (void)hipFree(d);
    (void)hipFree(s);
    return v[v.size() / 2] / n;
}

int main() {
    const int n = 1 << 14;
''')
    for td in (1, 2, 4):
        out.append(f'''    printf("TD=%d bare %6.1f  grouped %6.1f  interleaved %6.1f  transpose-publish %6.1f cyc/step/wave\\n", {td}, run(k_B_{td}, n), run(k_G_{td}, n), run(k_I_{td}, n), run(k_N_{td}, n));
    printf("TD=%d N parts: PE %6.1f  PT %6.1f  ET %6.1f  T %6.1f  E %6.1f  P %6.1f  none %6.1f\\n", {td}, run(k_NPE_{td}, n), run(k_NPT_{td}, n), run(k_NET_{td}, n), run(k_NT_{td}, n), run(k_NE_{td}, n), run(k_NP_{td}, n), run(k_N0_{td}, n));
''')
    out.append("    return 0;\n}\n")
    with open(os.path.join(HERE, "lane_ilv.hip"), "w") as f:
        f.write("".join(out))


if __name__ == "__main__":
    main()
