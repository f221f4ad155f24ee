// Round 6: why did readlane_idx.hip read 0 for a lane select >= 64 while the walker's compiled chain
// (ga_walk.h, __builtin_amdgcn_readlane with the index's upper bytes set) is exact?  In readlane_idx.hip the select is
// written by v_readfirstlane_b32 and read by the very next instruction, a v_readlane_b32 in inline asm: a VALU SGPR
// write followed by a lane-select read without the wait states the hardware asks for (the compiler's hazard
// recognizer does not look inside inline asm).  The walker's selects are written by SALU ops.  Four variants, each
// over the same selects:
//   0  readfirstlane -> asm readlane at once (the round-5 micro)
//   1  readfirstlane -> s_nop 4 -> asm readlane
//   2  the select advanced by an asm s_add_u32 (SALU), -> asm readlane (the walker's shape)
//   3  __builtin_amdgcn_readlane on an SALU-computed select (what ga_walk.h compiles to)
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void k(unsigned* out, const unsigned* idx, int n) {
    const int lane = threadIdx.x;
    const int v = 1000 + lane;
    for (int q = 0; q < n; q++) {
        const unsigned sel = __builtin_amdgcn_readfirstlane(idx[q] + (unsigned)(lane > 64));  // in an SGPR
        unsigned r0, r1, r2, r3;
        {
            unsigned s = __builtin_amdgcn_readfirstlane(idx[q] + (unsigned)lane * 0u + (unsigned)(lane > 64));
            asm volatile("v_readlane_b32 %0, %1, %2" : "=s"(r0) : "v"(v), "s"(s));
        }
        {
            unsigned s = __builtin_amdgcn_readfirstlane(idx[q] + (unsigned)(lane > 64));
            asm volatile("s_nop 4\n\tv_readlane_b32 %0, %1, %2" : "=s"(r1) : "v"(v), "s"(s));
        }
        {
            unsigned s;
            asm volatile("s_add_u32 %0, %1, 0" : "=s"(s) : "s"(sel));
            asm volatile("v_readlane_b32 %0, %1, %2" : "=s"(r2) : "v"(v), "s"(s));
        }
        {
            unsigned s;
            asm volatile("s_add_u32 %0, %1, 0" : "=s"(s) : "s"(sel));
            r3 = (unsigned)__builtin_amdgcn_readlane(v, (int)s);
        }
        if (lane == 0) {
            out[4 * q] = r0;
            out[4 * q + 1] = r1;
            out[4 * q + 2] = r2;
            out[4 * q + 3] = r3;
        }
    }
}

int main() {
    const unsigned h[9] = {5, 69, 133, 0x12345, 0x80000005u, 64, 0x7fffffc5u, 63, 0x080109u};
    const int N = 9;
    unsigned *di, *dout, ho[4 * N];
    (void)hipMalloc(&di, sizeof(h));
    (void)hipMalloc(&dout, sizeof(ho));
    (void)hipMemcpy(di, h, sizeof(h), hipMemcpyHostToDevice);
    k<<<1, 64>>>(dout, di, N);
    (void)hipMemcpy(ho, dout, sizeof(ho), hipMemcpyDeviceToHost);
    auto lane = [](unsigned x) { return x >= 1000 ? (int)(x - 1000) : -1; };
    printf("# lane read (-1: 0 returned) per variant: 0 readfirstlane->readlane at once, 1 with s_nop 4, 2 SALU select, "
           "3 builtin on an SALU select\n");
    for (int q = 0; q < N; q++)
        printf("sel 0x%08x (low6 %2u): v0 %3d  v1 %3d  v2 %3d  v3 %3d\n", h[q], h[q] & 63, lane(ho[4 * q]),
               lane(ho[4 * q + 1]), lane(ho[4 * q + 2]), lane(ho[4 * q + 3]));
    return 0;
}
