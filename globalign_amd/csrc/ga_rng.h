// ga_rng.h -- the host's emulation of CPython's global `random` for the traceback's tie-breaks (no HIP: built
// into the engine and into the host self-test, ga_host_selftest.cpp, which runs it under AddressSanitizer).
//
// The reference's dispatcher (cost_ranks_dispatcher, globaligner.py:595-685) calls random.choice 18 times per
// dispatched traceback step; random.choice(seq) of length 2 or 3 is _randbelow_with_getrandbits: getrandbits(2) of
// genrand_uint32 (Modules/_randommodule.c, MT19937), drawn again while >= len.  The engine turns the MT word stream
// into one u32 per dispatch (the level the dispatcher picks for every rank set) and reconstructs random.getstate()
// after the walk's last dispatch.
#pragma once
#include <stdint.h>

#include <algorithm>
#include <cstring>
#include <vector>

namespace garng {

// ------------------------------------------------------------------ CPython MT19937
constexpr int MTN = 624, MTM = 397;

struct PyMT {
    uint32_t mt[MTN];
    int mti;
    // one MT19937 twist, branch-free and in three runs without loop-carried dependences the
    // compiler cannot vectorise (kk+1 is read before it is written; kk-227 was written long before)
    static inline uint32_t tw(uint32_t a, uint32_t b, uint32_t c) {
        const uint32_t y = (a & 0x80000000u) | (b & 0x7fffffffu);
        return c ^ (y >> 1) ^ ((0u - (y & 1u)) & 0x9908b0dfu);
    }
    void twist() {
        uint32_t* __restrict m = mt;
        for (int kk = 0; kk < MTN - MTM; kk++) m[kk] = tw(m[kk], m[kk + 1], m[kk + MTM]);
        for (int kk = MTN - MTM; kk < MTN - 1; kk++) m[kk] = tw(m[kk], m[kk + 1], m[kk + (MTM - MTN)]);
        m[MTN - 1] = tw(m[MTN - 1], m[0], m[MTM - 1]);
        mti = 0;
    }
    inline uint32_t next() {
        if (mti >= MTN) twist();
        uint32_t y = mt[mti++];
        y ^= (y >> 11);
        y ^= (y << 7) & 0x9d2c5680u;
        y ^= (y << 15) & 0xefc60000u;
        y ^= (y >> 18);
        return y;
    }
    // random.choice(seq of len n) for n in {2,3}: getrandbits(2) with rejection
    inline unsigned below(unsigned n) {
        unsigned r;
        do { r = next() >> 30; } while (r >= n);
        return r;
    }
};

// ---------------------------------------------------------------- tie-break table
// The dispatcher's 18 draws per step consume a variable number of MT words
// (getrandbits(2) with rejection: r >= size -> draw again).  The scan below
// turns the word stream into the stream of ACCEPTED draws (18 per step) four
// words at a time through a table indexed by (draw index mod 18, top-2-bit
// quartet), then builds each step's entry from draws 0-3 / 9-12.
struct QuadEntry {
    uint32_t bytes;  // accepted values, one per byte, in order (unused bytes 0)
    uint16_t meta;   // nacc (3 bits) | word offset of each acceptance (4 x 2 bits) << 3
};
struct Quad {
    QuadEntry e[18][256];
    Quad() {
        static const unsigned sz[18] = {3, 2, 2, 2, 3, 2, 2, 2, 3, 3, 2, 2, 2, 3, 2, 2, 2, 3};
        for (int d = 0; d < 18; d++)
            for (int B = 0; B < 256; B++) {
                unsigned dd = d, nacc = 0, bytes = 0, pos = 0;
                for (unsigned wi = 0; wi < 4; wi++) {
                    const unsigned r = (B >> (2 * wi)) & 3u;
                    if (r < sz[dd]) {
                        bytes |= r << (8 * nacc);
                        pos |= wi << (2 * nacc);
                        nacc++;
                        dd = (dd + 1) % 18;
                    }
                }
                e[d][B].bytes = bytes;
                e[d][B].meta = (uint16_t)(nacc | (pos << 3));
            }
    }
};

// Branch-free form of the same table: next draw index, whether a dispatch completes inside the
// quartet and the word offset (+1) of its 18th acceptance.
struct QuadEntry2 {
    uint32_t bytes;
    uint8_t nacc, nd, wrap, woff;
};
struct Quad2 {
    QuadEntry2 e[18][256];
    Quad2() {
        static const Quad Q;
        for (int d = 0; d < 18; d++)
            for (int B = 0; B < 256; B++) {
                const QuadEntry& q = Q.e[d][B];
                const unsigned nacc = q.meta & 7u;
                QuadEntry2& r = e[d][B];
                r.bytes = q.bytes;
                r.nacc = (uint8_t)nacc;
                r.nd = (uint8_t)((d + nacc) % 18);
                r.wrap = (uint8_t)(d + nacc >= 18);
                r.woff = r.wrap ? (uint8_t)(((q.meta >> (3 + 2 * (17 - d))) & 3u) + 1) : 0;
            }
    }
};

struct RngTable;
inline void fill_entries(const uint8_t* acc, int64_t from, int64_t to, RngTable& R);

constexpr int TWSNAP = 64;

inline void temper_block(const uint32_t* mt, uint32_t* out) {
    for (int k = 0; k < MTN; k++) {
        uint32_t y = mt[k];
        y ^= (y >> 11);
        y ^= (y << 7) & 0x9d2c5680u;
        y ^= (y << 15) & 0xefc60000u;
        y ^= (y >> 18);
        out[k] = y;
    }
}

// The tie-break table as a RESUMABLE stream over CPython's MT19937 words: extend(D) makes the
// entries of dispatches [0, D) available, continuing where the last call stopped.  Consecutive
// alignments (each a find_global_alignment call that starts from the state the previous one left)
// consume ONE continuous stream of accepted draws, 18 per dispatch, so alignment k's dispatches are
// the global dispatches [G_k, G_k + D_k) of the same table (ga_problem_align_many).
struct RngTable {
    std::vector<uint32_t> tab;        // per dispatch: level per candidate set (see fill_entries)
    std::vector<uint32_t> step_end;   // words consumed after each dispatch
    std::vector<PyMT> twist_snap;     // MT array after every 64th twist (index 0 = initial state)
    int mti0 = 0;
    // stream position
    PyMT g{};
    uint32_t words[MTN + 4]{};
    int q = 0, count = 0;             // next word of the current tempered block, words in it
    int64_t wbase = 0, ntw = 0, p = 0, stp = 0;
    unsigned d = 0;                   // draw index within the dispatch (0..17)
    std::vector<uint8_t> acc;         // accepted draws (values 0..2)
    int64_t built = 0;                // dispatches whose entries are in tab

    void start(const uint32_t* state) {
        std::memcpy(g.mt, state, sizeof(uint32_t) * MTN);
        g.mti = (int)state[MTN];
        mti0 = g.mti;
        twist_snap.assign(1, g);
        tab.clear();
        step_end.clear();
        acc.clear();
        wbase = ntw = p = stp = built = 0;
        d = 0;
        // the partial first block: words mti0 .. 623 of the initial array
        uint32_t tmp[MTN];
        temper_block(g.mt, tmp);
        const int first = g.mti >= MTN ? 0 : g.mti;
        count = g.mti >= MTN ? 0 : MTN - g.mti;
        std::memcpy(words, tmp + first, sizeof(uint32_t) * count);
        q = 0;
    }

    void extend(int64_t steps) {
        if (steps <= built) return;
        static const Quad2 Q;
        static const unsigned sz[18] = {3, 2, 2, 2, 3, 2, 2, 2, 3, 3, 2, 2, 2, 3, 2, 2, 2, 3};
        const int64_t need = 18 * steps;
        acc.resize(std::max<size_t>(acc.size(), (size_t)need + 8));
        step_end.resize(std::max<size_t>(step_end.size(), (size_t)steps + 4));
        while (p < need) {
            if (q >= count) {
                wbase += count;
                g.twist();
                ntw++;
                if (ntw % TWSNAP == 0) twist_snap.push_back(g);
                temper_block(g.mt, words);
                count = MTN;
                q = 0;
            }
            for (; q + 4 <= count && p < need; q += 4) {
                const unsigned B = (words[q] >> 30) | ((words[q + 1] >> 30) << 2) | ((words[q + 2] >> 30) << 4) |
                                   ((words[q + 3] >> 30) << 6);
                const QuadEntry2& e = Q.e[d][B];
                std::memcpy(acc.data() + p, &e.bytes, 4);
                step_end[stp] = (uint32_t)(wbase + q + e.woff);  // branch-free: kept only when a dispatch completes
                stp += e.wrap;
                p += e.nacc;
                d = e.nd;
            }
            // tail words of the block (count not a multiple of 4), one at a time
            for (; q + 4 > count && q < count && p < need; q++) {
                const unsigned r = words[q] >> 30;
                if (r < sz[d]) {
                    acc[p] = (uint8_t)r;
                    if (d == 17) step_end[stp++] = (uint32_t)(wbase + q + 1);
                    p++;
                    d = d == 17 ? 0 : d + 1;
                }
            }
        }
        tab.resize(steps);
        fill_entries(acc.data(), built, steps, *this);
        built = steps;
    }
};

// The per-step entries from the accepted draws (18 per dispatch; draws 0-3 / 9-12 decide).
inline void fill_entries(const uint8_t* acc, int64_t from, int64_t to, RngTable& R) {
    for (int64_t st = from; st < to; st++) {
        const uint8_t* r = acc + 18 * st;
        uint32_t e = 0;
        for (int half = 0; half < 2; half++) {
            const uint8_t* qq = r + 9 * half;
            const unsigned lv[8] = {0, 0, 1, qq[1], 2, 2u * qq[2], 1u + qq[3], qq[0]};  // S = 1..7
            // level of rank set S at bits 2S+1+14*half (ga_kernels.hip, walk layout)
            for (int S = 1; S <= 7; S++) e |= lv[S] << (2 * S + 1 + 14 * half);
        }
        R.tab[st] = e;
    }
}

// The table of `steps` dispatches from the 625-word state (MT array + index).  Twisting and
// tempering the stream is the cost (~9 ms for 2*10^5 dispatches on an EPYC 9575F); it runs
// while the device fills.  (A producer/consumer split over two threads measured no faster.)
inline void build_rng(const uint32_t* state, int64_t steps, RngTable& R) {
    R.start(state);
    R.extend(steps);
}

// MT state after the first D dispatches consumed their words.
inline void state_after(const RngTable& R, int64_t D, uint32_t* out) {
    PyMT g = R.twist_snap[0];
    if (D == 0) {
        std::memcpy(out, g.mt, sizeof(uint32_t) * MTN);
        out[MTN] = (uint32_t)g.mti;
        return;
    }
    const int64_t W = R.step_end[D - 1];
    const int64_t first = R.mti0 >= MTN ? 0 : MTN - R.mti0;
    if (W <= first) {
        g.mti = R.mti0 + (int)W;
    } else {
        const int64_t Wp = W - first;
        const int64_t tw = (Wp + MTN - 1) / MTN;           // twists needed
        const int64_t sidx = tw / TWSNAP;
        g = R.twist_snap[sidx];
        for (int64_t t = sidx * TWSNAP; t < tw; t++) g.twist();
        g.mti = (int)(Wp - (tw - 1) * MTN);
    }
    std::memcpy(out, g.mt, sizeof(uint32_t) * MTN);
    out[MTN] = (uint32_t)g.mti;
}

}  // namespace garng
