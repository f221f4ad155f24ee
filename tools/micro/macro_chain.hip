// Microbenchmark: the walker's dependent chain per step (readlane of a window cell, the entering level's
// field, the tie-break table, the move) against a "macro step" (one readlane per one or two deterministic
// moves: the field is a precomputed code whose low 3 bits index the move's (rows, cols) and whose bits 3-4
// are the next entering level), both with the levels' 2-bit packing.  s_memtime units, one wave.
#include <hip/hip_runtime.h>
#include <cstdio>

template <int V>
__global__ void chain(long long* out, int* sink, int n) {
    const int lane = threadIdx.x & 63;
    // window cells: three 5-bit fields widened to bytes 0/8/16; V1 codes: deterministic (Lend < 3)
    const unsigned code = (unsigned)((lane * 7 + 3) % 24);
    unsigned win = (code & 31u) | (((code + 5) % 24) << 8) | (((code + 11) % 24) << 16);
    asm volatile("" : "+v"(win));
    unsigned t = 0x9e3779b9u, ix = 0, L8 = V == 2 ? 0x50000u : 0u;
    unsigned long long ops = 0;
    unsigned D = 0;
    const unsigned long long KD = 0x1002110A12080109ull;  // deltas r*8+c per didx
    const unsigned long long KLO = 0x0000a98654210210ull, KHI = 0x0000000a00000000ull;
    const unsigned N2 = 0x00ff7ff8u;
    const unsigned long long KDF = 0x9082918A92880109ull;  // deltas | second-move flag << 7
    long long t0 = __builtin_amdgcn_s_memtime();
    for (int k = 0; k < n; k++) {
        if (V == 0) {  // current walker step + packing
            const unsigned v = (unsigned)__builtin_amdgcn_readlane((int)win, (int)ix);
            L8 = (t >> ((v >> L8) & 31u)) & 0x18u;
            ix += 0x080109u >> L8;
            ops = (ops << 2) | (L8 >> 3);
            D += 1;
        } else if (V == 2) {  // macro step, lean: the code's delta byte carries the second move's flag at
            // bit 7 (so dispatches = macros + (moves >> 7)), and the codes are packed 5 bits each
            unsigned f, e, L8n;
            unsigned long long by;
            asm volatile(
                "v_readlane_b32 %0, %5, %3\n\t"
                "s_bfe_u32 %0, %0, %4\n\t"
                "s_lshl3_add_u32 %1, %0, 0x80000\n\t"
                "s_bfe_u64 s[88:89], %6, %1\n\t"
                "s_add_i32 %3, %3, s88\n\t"
                "s_and_b32 %4, %0, 0x18\n\t"
                "s_or_b32 %4, %4, 0x50000"
                : "=&s"(f), "=&s"(e), "=&s"(by), "+s"(ix), "+s"(L8) : "v"(win), "s"(KDF) : "s88", "s89");
            (void)L8n;
            ops = (ops << 5) | f;
            if (__builtin_expect(f >= 24u, 0)) { ix += 9u; L8 = 0x50000; }
        } else {  // macro step: one or two moves per readlane
            const unsigned v = (unsigned)__builtin_amdgcn_readlane((int)win, (int)ix);
            const unsigned f = (v >> L8) & 31u;
            ix += (unsigned)(KD >> ((f << 3) & 63u));
            L8 = f & 0x18u;
            const unsigned long long K = (f & 16u) ? KHI : KLO;
            const unsigned bits = (unsigned)(K >> ((f << 2) & 63u)) & 15u;
            const unsigned n2 = (N2 >> f) & 1u;
            ops = (ops << (2u + 2u * n2)) | bits;
            D += 1u + n2;
        }
        if (V != 2) ix &= 63u;
    }
    if (V == 2) D = (unsigned)n + (ix >> 7);
    long long t1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) out[blockIdx.x * 2] = t1 - t0, out[blockIdx.x * 2 + 1] = D;
    sink[blockIdx.x * blockDim.x + threadIdx.x] = (int)(ix + (unsigned)ops + (unsigned)(ops >> 32));
}

template <typename F>
void run(const char* name, F f) {
    long long* d; int* s;
    (void)hipMalloc(&d, 256 * 16);
    (void)hipMalloc(&s, 256 * 64 * 4);
    const int n = 1 << 16;
    f<<<1, 64>>>(d, s, n);
    f<<<1, 64>>>(d, s, n);
    (void)hipDeviceSynchronize();
    long long h[2] = {0, 0};
    (void)hipMemcpy(h, d, 16, hipMemcpyDeviceToHost);
    (void)hipFree(d); (void)hipFree(s);
    printf("%-40s %.1f cyc per readlane, %.2f moves each, %.1f cyc per move\n", name, (double)h[0] / n,
           (double)h[1] / n, (double)h[0] / h[1]);
}

int main() {
    run("step (readlane + table + packing)", chain<0>);
    run("macro step (one or two moves)", chain<1>);
    run("macro step, lean (flag in the delta byte)", chain<2>);
    return 0;
}
