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
#include <array>
#include <atomic>
#include <cmath>
#include <cstring>
#include <thread>
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
    std::vector<uint32_t> ring;       // build_rng_threaded's scratch: twisted blocks in flight, top-bit quartets
    std::vector<uint8_t> codes;

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
        // (never shrink: a threaded build may have scanned past `steps`, build_rng_threaded)
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

// The same table on `threads` host threads (round 6: the sequential build took 5.0 ms of one host thread per C3 call,
// hidden behind the fill, but on the critical path of any faster one).  Its cost is the scan's dependent chain (each
// four-word lookup needs the draw index the last one left: ~2.5 ns a quartet) more than the MT19937 twists (0.9 ms at
// C3, sequential by nature: each block of 624 words is the previous one twisted).  So this thread twists, into a ring
// of blocks, and W = threads - 1 workers each take one contiguous range of blocks, streaming behind it:
//   1. temper each word to its top two bits and scan the range from every possible start class -- draw index mod 9:
//      draws d and d + 9 have the same size, so they accept the same words -- until the nine trajectories meet (a
//      word of top bits 2 is accepted at a size-3 draw and rejected at a size-2 one; they meet within a few hundred
//      words), then once: the range's accepted draws and end class from each start class;
//   2. (this thread, once every range is summarized) each range's start phase and first accepted draw;
//   3. each worker rescans its range from its phase with the sequential scan's branch-free quartet table, writing
//      the accepted draws and the word count at the end of every dispatch (step_end), then the entries of the
//      dispatches whose draws it holds; the few straddling two ranges are finished here.
// The words needed are not known before the scan (32 per dispatch on average, sd 5.2): the twister makes enough for
// 8 sd above the mean, and a shortfall continues sequentially (extend).  The result equals build_rng's, the stream
// position included, so the table stays resumable (tests: ga_host_selftest, test_host_cpu).
struct ClassQuad {
    uint8_t nacc[9][256], ncls[9][256];
    ClassQuad() {
        static const unsigned sz[9] = {3, 2, 2, 2, 3, 2, 2, 2, 3};
        for (int c = 0; c < 9; c++)
            for (int B = 0; B < 256; B++) {
                unsigned cc = c, na = 0;
                for (int w = 0; w < 4; w++)
                    if (((B >> (2 * w)) & 3u) < sz[cc]) {
                        na++;
                        cc = (cc + 1) % 9;
                    }
                nacc[c][B] = (uint8_t)na;
                ncls[c][B] = (uint8_t)cc;
            }
    }
};

inline void build_rng_threaded(const uint32_t* state, int64_t steps, RngTable& R, int threads) {
    const int W = threads - 1;  // workers beside the twister
    if (W < 1 || steps < 8192) return build_rng(state, steps, R);
    static const ClassQuad CQ;
    static const Quad2 Q2;
    static const unsigned sz[18] = {3, 2, 2, 2, 3, 2, 2, 2, 3, 3, 2, 2, 2, 3, 2, 2, 2, 3};
    constexpr int RINGB = 256;    // twisted blocks in flight
    constexpr int QPB = MTN / 4;  // quartets per block
    R.start(state);               // the initial array, its partial first block (R.words, R.count) and twist_snap[0]
    const int first = R.count;
    const double sd = 5.2 * std::sqrt((double)steps);
    const int64_t want = 32 * steps + (int64_t)(8 * sd) + 4096;
    const int64_t nblk = std::max<int64_t>(W, (want - first + MTN - 1) / MTN);  // twisted blocks
    R.ring.resize((size_t)RINGB * MTN);      // (scratch kept by the table: no page faults when it is reused)
    R.codes.resize((size_t)nblk * QPB);
    struct alignas(64) Range {
        int64_t b0 = 0, b1 = 0;               // blocks [b0, b1)
        int64_t cnt[9] = {};                  // accepted draws from each start class
        uint8_t ecls[9] = {};                 // end class from each start class
        int64_t p0 = 0, p1 = 0;               // its draws [p0, p1)
        unsigned d0 = 0;                      // its start phase
        std::atomic<int64_t> tempered{0};     // blocks done (the twister may reuse their ring slots)
    };
    std::vector<Range> rg(W);
    for (int w = 0; w < W; w++) {
        rg[w].b0 = nblk * w / W;
        rg[w].b1 = nblk * (w + 1) / W;
    }
    // the partial first block from phase 0, word by word
    int64_t p = 0;
    unsigned d = 0;
    const size_t max_draws = (size_t)first + (size_t)nblk * MTN + 8;
    if (R.acc.size() < max_draws) R.acc.resize(max_draws);
    if (R.step_end.size() < max_draws / 18 + 8) R.step_end.resize(max_draws / 18 + 8);
    if (R.tab.size() < (size_t)steps) R.tab.resize(steps);
    uint8_t* acc = R.acc.data();
    uint32_t* se = R.step_end.data();
    for (int w = 0; w < first; w++) {
        const unsigned r = R.words[w] >> 30;
        if (r < sz[d]) {
            acc[p] = (uint8_t)r;
            if (d == 17) se[p / 18] = (uint32_t)(w + 1);
            p++;
            d = d == 17 ? 0 : d + 1;
        }
    }
    const int64_t p_head = p;
    std::atomic<int64_t> made{0};
    std::atomic<int> phase{0};  // 1: every range has its start (phase 3 may run)
    auto spin = [](int& k) {
        if (++k > 64) std::this_thread::yield();
    };
    auto worker = [&](int w) {
        Range& G = rg[w];
        uint8_t* cd = R.codes.data();
        // 1. temper + summary, streaming behind the twister
        int64_t cnt[9];
        uint8_t cls[9];
        for (int c = 0; c < 9; c++) {
            cnt[c] = 0;
            cls[c] = (uint8_t)c;
        }
        bool met = false;
        int64_t shared = 0;
        for (int64_t b = G.b0; b < G.b1; b++) {
            for (int k = 0; made.load(std::memory_order_acquire) <= b;) spin(k);
            const uint32_t* mt = &R.ring[(size_t)(b % RINGB) * MTN];
            uint8_t* cb = cd + b * QPB;
            for (int q = 0; q < QPB; q++) {
                unsigned B = 0;
                for (int x = 0; x < 4; x++) {
                    uint32_t y = mt[4 * q + x];
                    y ^= (y >> 11);
                    y ^= (y << 7) & 0x9d2c5680u;
                    y ^= (y << 15) & 0xefc60000u;
                    y ^= (y >> 18);
                    B |= (y >> 30) << (2 * x);
                }
                cb[q] = (uint8_t)B;
            }
            G.tempered.store(b + 1 - G.b0, std::memory_order_release);
            if (!met) {
                for (int q = 0; q < QPB; q++) {
                    const unsigned B = cb[q];
                    if (met) {
                        shared += CQ.nacc[cls[0]][B];
                        cls[0] = CQ.ncls[cls[0]][B];
                        continue;
                    }
                    for (int c = 0; c < 9; c++) {
                        cnt[c] += CQ.nacc[cls[c]][B];
                        cls[c] = CQ.ncls[cls[c]][B];
                    }
                    met = true;
                    for (int c = 1; c < 9; c++) met &= cls[c] == cls[0];
                }
            } else {
                uint8_t c0 = cls[0];
                for (int q = 0; q < QPB; q++) {
                    shared += CQ.nacc[c0][cb[q]];
                    c0 = CQ.ncls[c0][cb[q]];
                }
                cls[0] = c0;
            }
        }
        for (int c = 0; c < 9; c++) {
            G.cnt[c] = cnt[c] + shared;
            G.ecls[c] = met ? cls[0] : cls[c];
        }
        G.tempered.store(G.b1 - G.b0 + 1, std::memory_order_release);  // (one past: the summary is in)
        // 3. once every start is known: the draws and dispatch ends, then the entries inside the range
        for (int k = 0; phase.load(std::memory_order_acquire) == 0;) spin(k);
        int64_t pp = G.p0, stp = pp / 18;
        unsigned dd = G.d0;
        uint32_t spill = 0;  // the step_end store of a quartet that completes no dispatch
        const int64_t nq = (G.b1 - G.b0) * QPB;
        const uint8_t* cr = cd + G.b0 * QPB;
        const int64_t wb = first + G.b0 * MTN;  // the range's first word, counted from the stream's start
        for (int64_t q = 0; q < nq; q++) {
            const QuadEntry2& e = Q2.e[dd][cr[q]];
            if (pp + 4 <= G.p1) std::memcpy(acc + pp, &e.bytes, 4);  // (junk past the accepted bytes: overwritten)
            else
                for (unsigned t = 0; t < e.nacc; t++) acc[pp + t] = (uint8_t)(e.bytes >> (8 * t));
            *(e.wrap ? se + stp : &spill) = (uint32_t)(wb + 4 * q + e.woff);
            stp += e.wrap;
            pp += e.nacc;
            dd = e.nd;
        }
        const int64_t lo = (G.p0 + 17) / 18, hi = std::min<int64_t>(G.p1 / 18, steps);
        if (lo < hi) fill_entries(acc, lo, hi, R);
    };
    std::vector<std::thread> pool;
    pool.reserve(W);
    for (int w = 0; w < W; w++) pool.emplace_back(worker, w);
    // the twister: this thread (snapshots every TWSNAP twists, as extend() takes them)
    PyMT g = R.g;
    int owner = 0;  // the range of block b
    for (int64_t b = 0; b < nblk; b++) {
        while (owner + 1 < W && b >= rg[owner + 1].b0) owner++;
        if (b >= RINGB) {  // block b reuses block b - RINGB's slot: wait until its range has tempered it
            const int64_t old = b - RINGB;
            int ow = owner;
            while (rg[ow].b0 > old) ow--;
            for (int k = 0; rg[ow].tempered.load(std::memory_order_acquire) <= old - rg[ow].b0;) spin(k);
        }
        g.twist();
        if ((b + 1) % TWSNAP == 0) R.twist_snap.push_back(g);
        std::memcpy(&R.ring[(size_t)(b % RINGB) * MTN], g.mt, sizeof(uint32_t) * MTN);
        made.store(b + 1, std::memory_order_release);
    }
    // 2. the ranges' starts, in order, once their summaries are in
    p = p_head;
    for (int w = 0; w < W; w++) {
        for (int k = 0; rg[w].tempered.load(std::memory_order_acquire) <= rg[w].b1 - rg[w].b0;) spin(k);
        const int c = (int)(d % 9);
        rg[w].p0 = p;
        rg[w].d0 = d;
        p += rg[w].cnt[c];
        d = (unsigned)((d + rg[w].cnt[c]) % 18);
        rg[w].p1 = p;
    }
    phase.store(1, std::memory_order_release);
    for (auto& t : pool) t.join();
    const int64_t total = p, ndisp = total / 18;
    // the entries no range holds whole: inside the partial first block, and those straddling two ranges
    fill_entries(acc, 0, std::min<int64_t>(steps, p_head / 18), R);
    for (int w = 0; w < W; w++)
        if (rg[w].p0 % 18 && rg[w].p0 / 18 < steps) fill_entries(acc, rg[w].p0 / 18, rg[w].p0 / 18 + 1, R);
    // the stream position after every generated word (resumable: extend continues from here)
    R.g = g;
    temper_block(g.mt, R.words);
    R.count = MTN;
    R.q = MTN;
    R.wbase = first + (nblk - 1) * MTN;
    R.ntw = nblk;
    R.p = total;
    R.stp = ndisp;
    R.d = d;
    R.acc.resize((size_t)total + 8);
    if (ndisp < steps) {  // the twister fell short (8 sd): continue sequentially
        R.built = std::min<int64_t>(ndisp, steps);
        R.tab.resize(R.built);
        R.extend(steps);
        return;
    }
    R.tab.resize(steps);
    R.built = steps;
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
