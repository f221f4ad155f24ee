// Microbenchmark: one trip of a tie-to-tie walker (one wave, LDS only) on gfx950.
//
// The torus holds, per cell and entering level, a 16-bit jump entry: up to 8 moves of 2 bits (first move in
// bits 1:0; bit 0 = the move lowers j, bit 1 = it lowers i: diag 3, left 1, up 2; 0 = no more moves), or a tie
// (bits 1:0 = 0, the table shift in bits 6:2).  A trip: from the current state t (its cell and level known),
// one ds_read fetches t's three level entries, the entries of t's three successors and the tie-break table
// entry of t's dispatch; the walker then takes t's own entry, or, at a tie, the successor the table picks
// (its entry with the tie move prepended), and advances by that jump.  Prints cycles per trip.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

constexpr int TP = 128;

template <int V>
__global__ void trips(const uint16_t* img, const uint32_t* tabimg, long long* out, unsigned* sink, int n) {
    __shared__ uint16_t E[3 * TP * TP];
    __shared__ uint32_t tab[2048];
    const int lane = threadIdx.x & 63;
    for (int q = lane; q < 3 * TP * TP; q += 64) E[q] = img[q];
    for (int q = lane; q < 2048; q += 64) tab[q] = tabimg[q];
    __syncthreads();
    // per-lane constants: lanes 0..2 t's level entries; 3..5 the successors (diag / left / up) at their level
    // (byte offsets: rows of TP cells, planes of TP * TP cells)
    const unsigned drow = (lane == 3 || lane == 5) ? 2u * TP : 0u;
    const unsigned dcol = (lane == 3 || lane == 4) ? 2u : 0u;
    const unsigned plane = 2u * TP * TP * (unsigned)(lane < 3 ? lane : lane < 6 ? lane - 3 : 0);
    const unsigned code = lane == 3 ? 3u : lane == 4 ? 1u : lane == 5 ? 2u : 0u;  // the tie move's code
    const unsigned tabbase = (unsigned)(uintptr_t)tab;
    const unsigned ebase = (unsigned)(uintptr_t)E;
    // t's torus offset: row part ((i - 1) & (TP-1)) * 2TP, column part ((j - 1) & (TP-1)) * 2, kept unmasked in SGPRs
    unsigned roff = 0, coff = 0;
    int L = 0, D = 0;
    unsigned W = 3u;  // start: one diagonal move
    unsigned acc = 0, nb = 0;
    long long t0 = __builtin_amdgcn_s_memtime();
    for (int k = 0; k < n; k++) {
        // advance by W (up to 9 moves): 2 SALU each on the chain
        roff -= 2u * TP * (unsigned)__builtin_popcount(W & 0xaaaaau);
        coff -= 2u * (unsigned)__builtin_popcount(W & 0x55555u);
        // the fetch: per-lane address (masks wrap the torus), one u16 per lane, the table entry broadcast
        const unsigned r = (roff - drow) & (2u * TP * (TP - 1)), c = (coff - dcol) & (2u * (TP - 1));
        const unsigned addr = ebase + (r | c | plane);
        unsigned v, tb;
        asm volatile("ds_read_u16 %0, %1" : "=v"(v) : "v"(addr));
        // off the chain while the reads are in flight: dispatches, the record, the level of W's last move
        const unsigned km = __builtin_popcount((W | (W >> 1)) & 0x55555u);
        D += (int)km;
        acc = (acc << (2 * km)) ^ W;
        nb += km;
        L = (int)(3u - ((W >> (2 * km - 2)) & 3u));
        const unsigned taddr = tabbase + (((unsigned)D & 2047u) << 2);
        asm volatile("ds_read_b32 %0, %1" : "=v"(tb) : "v"(taddr));
        // (inline asm outputs count as ready at once: the wait is an asm that rewrites both)
        asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(v), "+v"(tb));
        const unsigned e = (unsigned)__builtin_amdgcn_readlane((int)v, L);
        if (V == 0) {
            if (e & 3u) {
                W = e;
            } else {
                // a tie: the table picks the level; W = the tie move, then the successor's run (if not a tie)
                const unsigned t = (unsigned)__builtin_amdgcn_readfirstlane((int)tb);
                const unsigned lvl = (t >> (((e >> 2) & 31u) + 3u)) & 3u;
                const unsigned s = (unsigned)__builtin_amdgcn_readlane((int)v, (int)(3u + lvl));
                W = (((s & 3u) ? s : 0u) << 2) | (3u - lvl);
            }
        } else {
            // successors prepared in VALU before the readlane
            const unsigned vs = (((v & 3u) ? v : 0u) << 2) | code;
            if (e & 3u) {
                W = e;
            } else {
                const unsigned t = (unsigned)__builtin_amdgcn_readfirstlane((int)tb);
                const unsigned lvl = (t >> (((e >> 2) & 31u) + 3u)) & 3u;
                W = (unsigned)__builtin_amdgcn_readlane((int)vs, (int)(3u + lvl));
            }
        }
    }
    long long t1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) {
        out[0] = t1 - t0;
        out[1] = D;
        out[2] = nb;
    }
    sink[lane] = acc + roff + coff + (unsigned)L;
}

// v_perm_b32 semantics check (the jump build selects 16-bit candidates with it): byte k of the result is byte
// sel_k of {a, b} (b = bytes 0..3, a = bytes 4..7), 0x0c gives 0x00
__global__ void perm_check(unsigned* out) {
    const unsigned a = 0x77665544u, b = 0x33221100u;
    out[0] = __builtin_amdgcn_perm(a, b, 0x05040100u);
    out[1] = __builtin_amdgcn_perm(a, b, 0x0c0c0706u);
    out[2] = __builtin_amdgcn_perm(a, b, 0x03020c0cu);
    out[3] = __builtin_amdgcn_perm(a, b, 0x0d0d0b0au);
}

static unsigned rnd(unsigned long long& s) {
    s = s * 6364136223846793005ull + 1442695040888963407ull;
    return (unsigned)(s >> 33);
}

template <typename F>
void run(const char* name, F f, const uint16_t* dimg, const uint32_t* dtab) {
    long long* d;
    unsigned* s;
    (void)hipMalloc(&d, 64);
    (void)hipMalloc(&s, 64 * 4);
    const int n = 1 << 16;
    f<<<1, 64>>>(dimg, dtab, d, s, n);
    f<<<1, 64>>>(dimg, dtab, d, s, n);
    (void)hipDeviceSynchronize();
    long long h[3];
    (void)hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
    printf("%-34s %.1f cycles per trip, %.2f moves per trip, %.1f cycles per move\n", name, (double)h[0] / n,
           (double)h[1] / n, (double)h[0] / h[1]);
    (void)hipFree(d);
    (void)hipFree(s);
}

int main() {
    // synthetic entries: 85 % runs of 1..8 moves (mostly diagonal), 15 % ties
    std::vector<uint16_t> img(3 * TP * TP);
    unsigned long long s = 12345;
    for (auto& e : img) {
        if (rnd(s) % 100 < 15) {
            e = (uint16_t)((4u + 2u * (rnd(s) % 12u)) << 2);
            continue;
        }
        const int k = 1 + (int)(rnd(s) % 8);
        unsigned w = 0;
        for (int q = 0; q < k; q++) {
            const unsigned x = rnd(s) % 10;
            w |= (x < 6 ? 3u : x < 8 ? 1u : 2u) << (2 * q);
        }
        e = (uint16_t)w;
    }
    std::vector<uint32_t> tab(2048);
    for (auto& t : tab) {  // every 2-bit field a level 0..2, as the host's table
        t = 0;
        for (int f = 0; f < 16; f++) t |= (rnd(s) % 3u) << (2 * f);
    }
    uint16_t* dimg;
    uint32_t* dtab;
    (void)hipMalloc(&dimg, img.size() * 2);
    (void)hipMalloc(&dtab, tab.size() * 4);
    (void)hipMemcpy(dimg, img.data(), img.size() * 2, hipMemcpyHostToDevice);
    (void)hipMemcpy(dtab, tab.data(), tab.size() * 4, hipMemcpyHostToDevice);
    {
        unsigned* d;
        unsigned h[4];
        (void)hipMalloc(&d, 16);
        perm_check<<<1, 64>>>(d);
        (void)hipMemcpy(h, d, 16, hipMemcpyDeviceToHost);
        printf("perm: %08x %08x %08x %08x (expect 55441100 00007766 33220000 ...)\n", h[0], h[1], h[2], h[3]);
        (void)hipFree(d);
    }
    run("trip, tie move in SALU", trips<0>, dimg, dtab);
    run("trip, tie move in VALU", trips<1>, dimg, dtab);
    return 0;
}
