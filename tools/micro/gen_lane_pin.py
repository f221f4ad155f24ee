"""Generate tools/micro/lane_pin.hip: 16 lane-fill steps (the ga_lane_asm.h recurrence) in one asm statement with
the compiler's register choice ("v" constraints, U) against physical registers pinned ("{vN}" constraints, P) so
that no VALU op reads two operands from one VGPR bank (bank = register number mod 4):
    T, M_k: bank 0;  X_s, hn_s: bank 1 (even s) / 3 (odd s);  H_k, Y_k, HLn: bank 2;  q: banks 0/1;
    edges E: aligned quads (eh0, ex0, eh1, ex1) = banks 0..3, so step s's DPP adds never meet X / hn of step s-1.
Cycles per step per wave, one wave per SIMD (256 workgroups of 4 waves).

    python tools/micro/gen_lane_pin.py && hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/micro/lane_pin.hip \
        -o tools/micro/lane_pin
"""
import os

HERE = os.path.dirname(os.path.abspath(__file__))


class Alloc:
    def __init__(self, lo=96, hi=256):
        self.free = set(range(lo, hi))

    def take(self, bank, n=1, align=1):
        """n consecutive registers starting in `bank` (None: any) at a multiple of `align`"""
        for r in sorted(self.free):
            if r % align or (bank is not None and r % 4 != bank):
                continue
            if all(r + i in self.free for i in range(n)):
                for i in range(n):
                    self.free.discard(r + i)
                return r
        raise RuntimeError("out of registers")


def regs(td):
    a = Alloc()
    R = {"T": a.take(0)}
    for k in range(td):
        R[f"M{k}"] = a.take(0)
    for s in range(16):
        R[f"X{s}"] = a.take(1 if s % 2 == 0 else 3)
        R[f"hn{s}"] = a.take(1 if s % 2 == 0 else 3)
    R["HLn0"], R["HLn1"] = a.take(2), a.take(2)
    for k in range(td - 1):
        R[f"H{k}"] = a.take(2)
    for k in range(td):
        R[f"Y{k}"] = a.take(2)
    R["E"] = a.take(0, 32, 4)
    for k in range(td):
        for d in (0, 2):
            R[f"q{k}_{d}"] = a.take(0, 2, 2)
            R[f"q{k}_{d + 1}"] = R[f"q{k}_{d}"] + 1
    return R


def body(td, R, pinned):
    def v(name):
        return f"v{R[name]}" if pinned else f"%[{name}]"

    def ex(s):
        return f"v{R['E'] + 4 * (s // 2) + 1 + 2 * (s % 2)}" if pinned else f"%[ex{s}]"

    def eh(s):
        return f"v{R['E'] + 4 * (s // 2) + 2 * (s % 2)}" if pinned else f"%[eh{s}]"

    lines = []
    for s in range(16):
        u = s % 4
        xl = v("X15") if s == 0 else v(f"X{s - 1}")
        hlp = v("HLn1") if s == 0 else v(f"HLn{(s - 1) % 2}")
        hlast = v("hn15") if s == 0 else v(f"hn{s - 1}")
        hd = [hlp] + [v(f"H{k}") for k in range(td - 1)]
        for k in range(td):
            q = f"v{R[f'q{k}_{s // 4}']}" if pinned else f"%[q{k}_{s // 4}]"
            lines.append(f"v_add_u32_sdwa {v(f'M{k}')}, sext({q}), {hd[k]} dst_sel:DWORD dst_unused:UNUSED_PAD "
                         f"src0_sel:BYTE_{u} src1_sel:DWORD")
        if td == 1 and s == 0:
            lines.append("s_nop 1")
        lines += [f"v_add_u32_dpp {v(f'X{s}')}, {xl}, {ex(s)} wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1",
                  f"v_add_u32_dpp {v(f'HLn{s % 2}')}, {hlast}, {eh(s)} wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1"]
        for k in range(td):
            dst = v(f"hn{s}") if k == td - 1 else v(f"H{k}")
            lines += [f"v_min3_i32 {dst}, {v(f'M{k}')}, {v(f'X{s}')}, {v(f'Y{k}')}", f"v_add_u32 {v('T')}, %[o], {dst}",
                      f"v_min_i32 {v(f'X{s}')}, {v(f'X{s}')}, {v('T')}", f"v_min_i32 {v(f'Y{k}')}, {v(f'Y{k}')}, {v('T')}"]
    return "\n".join(f'        "{ln}\\n\\t"' for ln in lines[:-1]) + f'\n        "{lines[-1]}"'


def kernel(td, pinned):
    R = regs(td)
    b = body(td, R, pinned)
    if pinned:
        # state lives in its pinned registers across iterations: tie each in/out pair to one physical register
        outs = [f'"+{{v{R["X15"]}}}"(Xl)', f'"+{{v{R["HLn1"]}}}"(HLp)', f'"+{{v{R["hn15"]}}}"(Hl)'] + \
               [f'"+{{v{R[f"H{k}"]}}}"(H[{k}])' for k in range(td - 1)] + [f'"+{{v{R[f"Y{k}"]}}}"(Y[{k}])' for k in range(td)]
        ins = [f'"{{v[{R["E"]}:{R["E"] + 31}]}}"(E)'] + \
              [f'"{{v[{R[f"q{k}_{d}"]}:{R[f"q{k}_{d}"] + 1}]}}"(qp[{k}][{d // 2}])' for k in range(td) for d in (0, 2)] + \
              ['[o] "s"(o)']
        clob = [f'"v{R[n]}"' for n in ["T"] + [f"M{k}" for k in range(td)] + [f"X{s}" for s in range(15)] +
                [f"hn{s}" for s in range(15)] + ["HLn0"]]
        asm = f"""        asm volatile(
{b}
        : {", ".join(outs)}
        : {", ".join(ins)}
        : {", ".join(clob)});"""
        decl = f"""    v32i E;
    for (int k = 0; k < 32; k++) E[k] = (k % 2 == 1 && lane == 0) ? k : 0;
    v2u qp[{td}][2];
    for (int k = 0; k < {td}; k++) for (int d = 0; d < 2; d++) qp[k][d] = v2u{{0x01020304u * ((lane + k + d) & 3), 0x01030204u}};"""
    else:
        outs = ['[X15] "+v"(Xl)', '[HLn1] "+v"(HLp)', '[hn15] "+v"(Hl)'] + \
               [f'[X{s}] "=&v"(X[{s}])' for s in range(15)] + [f'[hn{s}] "=&v"(hn[{s}])' for s in range(15)] + \
               ['[HLn0] "=&v"(HLn0)'] + [f'[H{k}] "+v"(H[{k}])' for k in range(td - 1)] + \
               [f'[Y{k}] "+v"(Y[{k}])' for k in range(td)] + ['[T] "=&v"(T)'] + [f'[M{k}] "=&v"(M[{k}])' for k in range(td)]
        ins = [f'[ex{s}] "v"(E[{s // 2}][{1 + 2 * (s % 2)}])' for s in range(16)] + \
              [f'[eh{s}] "v"(E[{s // 2}][{2 * (s % 2)}])' for s in range(16)] + \
              [f'[q{k}_{d}] "v"(q[{k}][{d}])' for k in range(td) for d in range(4)] + ['[o] "s"(o)']
        asm = f"""        asm volatile(
{b}
        : {", ".join(outs)}
        : {", ".join(ins)});"""
        decl = f"""    v4i E[8];
    for (int k = 0; k < 8; k++) E[k] = v4i{{0, lane == 0 ? k : 0, 0, 0}};
    uint32_t q[{td}][4];
    for (int k = 0; k < {td}; k++) for (int d = 0; d < 4; d++) q[k][d] = 0x01020304u * ((lane + k + d) & 3);
    int X[16], hn[16], HLn0, T, M[{td}];"""
    name = f"k_{'P' if pinned else 'U'}_{td}"
    return f"""
__global__ void __launch_bounds__(256) {name}(long long* res, int* sink, int nsteps, int o) {{
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    int H[{td}], Y[{td}];
    for (int k = 0; k < {td}; k++) {{ H[k] = lane + k; Y[k] = lane + 2 * k + 1; }}
    int Xl = lane + 3, HLp = lane + 1, Hl = lane;
{decl}
    long long t0 = __builtin_amdgcn_s_memtime();
    for (int r = 0; r < nsteps; r += 16) {{
{asm}
    }}
    long long t1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) res[blockIdx.x * 16 + w] = t1 - t0;
    int z = Xl + HLp + Hl;
    for (int k = 0; k < {td}; k++) z += H[k] + Y[k];
    sink[blockIdx.x * blockDim.x + threadIdx.x] = z;
}}
"""


def main():
    out = ['''// GENERATED by tools/micro/gen_lane_pin.py (see its docstring)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v32i __attribute__((ext_vector_type(32)));
typedef unsigned v2u __attribute__((ext_vector_type(2)));
''']
    for td in (1, 2, 4, 8):
        out += [kernel(td, False), kernel(td, True)]
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
    for td in (1, 2, 4, 8):
        out.append(f'    printf("TD=%d compiler registers %6.1f  pinned registers %6.1f cyc/step/wave\\n", {td}, '
                   f'run(k_U_{td}, n), run(k_P_{td}, n));\n')
    out.append("    return 0;\n}\n")
    with open(os.path.join(HERE, "lane_pin.hip"), "w") as f:
        f.write("".join(out))


if __name__ == "__main__":
    main()
