// ga_host_selftest.cpp -- CPU self-test of the engine's host-only pieces, built with AddressSanitizer and
// UndefinedBehaviorSanitizer (make -C globalign_amd/csrc asan; run by tests/test_host_asan.py):
//   * the tie-break table (ga_rng.h): RngTable's four-word scan, its resumable extend() and state_after(), against a draw-by-draw restatement of CPython's random.choice (_randbelow_with_getrandbits over
//     genrand_uint32) and the dispatcher's level rule (globaligner.py:595-685);
//   * the problem checks (ga_check.h): argument validation, the int32 range guard, the profile / word widths.
// No HIP: the engine's library is tested on the GPU; this binary covers the host logic under the sanitizers.
//
//   ga_host_selftest            all checks; exit status 0 when every one passes
//   ga_host_selftest bench S    time the table for S dispatches
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "ga_check.h"
#include "ga_rng.h"

using namespace garng;

namespace {

int failures = 0;

#define CHECK(cond, ...)                                   \
    do {                                                   \
        if (!(cond)) {                                     \
            failures++;                                    \
            std::fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
            std::fprintf(stderr, __VA_ARGS__);             \
            std::fprintf(stderr, "\n");                    \
        }                                                  \
    } while (0)

uint64_t splitmix(uint64_t& s) {
    uint64_t z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// a random 625-word state (624 words + index), as random.getstate()[1] could hold
std::vector<uint32_t> random_state(uint64_t seed) {
    std::vector<uint32_t> st(MTN + 1);
    uint64_t s = seed;
    for (int k = 0; k < MTN; k++) st[k] = (uint32_t)splitmix(s);
    st[0] |= 0x80000000u;  // never the all-zero array
    st[MTN] = (uint32_t)(splitmix(s) % (MTN + 1));
    return st;
}

// the dispatcher's level per rank set S = 1..7 from one step's 18 draws (ga_rng.h fill_entries' rule, written out
// from the dict literal, :599-671): S = 7 {0,1,2} -> draw 0; 3 {0,1} -> (0,1)[draw 1]; 5 {0,2} -> (0,2)[draw 2];
// 6 {1,2} -> (1,2)[draw 3]; singletons fixed; the mismatch half uses draws 9..12
uint32_t naive_entry(const unsigned* r) {
    uint32_t e = 0;
    for (int half = 0; half < 2; half++) {
        const unsigned* q = r + 9 * half;
        const unsigned lv[8] = {0, 0, 1, q[1] ? 1u : 0u, 2, q[2] ? 2u : 0u, q[3] ? 2u : 1u, q[0]};
        for (int S = 1; S <= 7; S++) e |= lv[S] << (2 * S + 1 + 14 * half);
    }
    return e;
}

struct Naive {
    std::vector<uint32_t> tab;
    std::map<int64_t, std::vector<uint32_t>> states;  // state after d dispatches (only where asked)
};

Naive naive_table(const std::vector<uint32_t>& st, int64_t steps, const std::vector<int64_t>& want_states) {
    static const unsigned sz[18] = {3, 2, 2, 2, 3, 2, 2, 2, 3, 3, 2, 2, 2, 3, 2, 2, 2, 3};
    PyMT g;
    std::memcpy(g.mt, st.data(), sizeof(uint32_t) * MTN);
    g.mti = (int)st[MTN];
    Naive out;
    out.tab.resize(steps);
    auto snap = [&](int64_t d) {
        for (int64_t w : want_states)
            if (w == d) {
                std::vector<uint32_t> s(MTN + 1);
                std::memcpy(s.data(), g.mt, sizeof(uint32_t) * MTN);
                s[MTN] = (uint32_t)g.mti;
                out.states[d] = s;
            }
    };
    snap(0);
    for (int64_t d = 0; d < steps; d++) {
        unsigned r[18];
        for (int k = 0; k < 18; k++) r[k] = g.below(sz[k]);
        out.tab[d] = naive_entry(r);
        snap(d + 1);
    }
    return out;
}

bool same_state(const uint32_t* a, const std::vector<uint32_t>& b) {
    // equal as CPython states: the same 624 words and index (a twisted-at-624 array equals its untwisted form only
    // through the index, so compare the next words instead when the indices differ)
    if (std::memcmp(a, b.data(), sizeof(uint32_t) * (MTN + 1)) == 0) return true;
    PyMT x, y;
    std::memcpy(x.mt, a, sizeof(uint32_t) * MTN);
    x.mti = (int)a[MTN];
    std::memcpy(y.mt, b.data(), sizeof(uint32_t) * MTN);
    y.mti = (int)b[MTN];
    for (int k = 0; k < 2 * MTN; k++)
        if (x.next() != y.next()) return false;
    return true;
}

void test_table(uint64_t seed, int64_t steps) {
    const auto st = random_state(seed);
    std::vector<int64_t> Ds = {0, 1, steps / 3, steps / 2, steps};
    for (auto& D : Ds) D = std::min(D, steps);
    const Naive nv = naive_table(st, steps, Ds);
    // sequential build
    RngTable R;
    build_rng(st.data(), steps, R);
    CHECK((int64_t)R.tab.size() == steps, "seed %llu: %zu entries for %lld steps", (unsigned long long)seed, R.tab.size(),
          (long long)steps);
    for (int64_t d = 0; d < steps && d < (int64_t)R.tab.size(); d++)
        if (R.tab[d] != nv.tab[d]) {
            CHECK(false, "seed %llu steps %lld: entry %lld %08x != %08x", (unsigned long long)seed, (long long)steps,
                  (long long)d, R.tab[d], nv.tab[d]);
            break;
        }
    for (size_t k = 0; k < Ds.size(); k++) {
        uint32_t out[MTN + 1];
        state_after(R, Ds[k], out);
        CHECK(same_state(out, nv.states.at(Ds[k])), "seed %llu: state after %lld dispatches", (unsigned long long)seed,
              (long long)Ds[k]);
    }
    // resumable: extend() in uneven chunks
    RngTable Q;
    Q.start(st.data());
    for (int64_t b = 7; b < steps + 7; b = b * 2 + 3) Q.extend(std::min(b, steps));
    Q.extend(steps);
    CHECK(Q.tab == R.tab, "seed %llu: chunked extend differs", (unsigned long long)seed);
}

void test_checks() {
    const int K = 5;
    int32_t sub[K * K], gh[K], gv[K];
    for (int x = 0; x < K; x++) {
        gh[x] = 2;
        gv[x] = 2;
        for (int y = 0; y < K; y++) sub[x * K + y] = x == y ? 0 : 5;
    }
    ga_costs cs{K, sub, gh, gv, 5, 5};
    std::vector<uint8_t> a(1000), b(800);
    uint64_t s = 99;
    for (auto& x : a) x = (uint8_t)(splitmix(s) % 4);
    for (auto& x : b) x = (uint8_t)(splitmix(s) % 4);
    ProblemShape ps;
    std::string err;
    CHECK(check_problem(a.data(), 1000, b.data(), 800, &cs, nullptr, nullptr, 0, 800, ps, err) == GA_OK, "valid: %s",
          err.c_str());
    CHECK(ps.big == 6 * 1000 && ps.CB == 1 && ps.qbytes == 1, "shape big %lld CB %d qbytes %d", (long long)ps.big, ps.CB,
          ps.qbytes);
    CHECK(check_problem(nullptr, 1000, b.data(), 800, &cs, nullptr, nullptr, 0, 800, ps, err) == GA_E_ARG, "null a");
    CHECK(check_problem(a.data(), 0, b.data(), 800, &cs, nullptr, nullptr, 0, 800, ps, err) == GA_E_ARG, "empty");
    CHECK(check_problem(a.data(), 1000, b.data(), 800, &cs, nullptr, nullptr, 10, 5, ps, err) == GA_E_ARG, "slab");
    a[17] = K;
    CHECK(check_problem(a.data(), 1000, b.data(), 800, &cs, nullptr, nullptr, 0, 800, ps, err) == GA_E_ARG, "code");
    a[17] = 0;
    ga_costs neg = cs;
    neg.gap_open = -1;
    CHECK(check_problem(a.data(), 1000, b.data(), 800, &neg, nullptr, nullptr, 0, 800, ps, err) == GA_E_ARG, "open < 0");
    ga_costs wide = cs;
    wide.gap_open = 200;  // o + 1 >= 128: 4-byte traceback words
    CHECK(check_problem(a.data(), 1000, b.data(), 800, &wide, nullptr, nullptr, 0, 800, ps, err) == GA_OK && ps.CB == 4,
          "open 200: CB %d", ps.CB);
    ga_costs huge = cs;
    huge.gap_open = 40000;
    CHECK(check_problem(a.data(), 1000, b.data(), 800, &huge, nullptr, nullptr, 0, 800, ps, err) == GA_E_RANGE,
          "open 40000 must not fit a traceback word");
    int32_t sub2[K * K];
    std::memcpy(sub2, sub, sizeof(sub));
    sub2[3] = 1 << 20;
    ga_costs big = cs;
    big.sub = sub2;
    big.max_cost = 1 << 20;
    CHECK(check_problem(a.data(), 1000, b.data(), 800, &big, nullptr, nullptr, 0, 800, ps, err) == GA_E_RANGE,
          "int32 range guard");
    // custom boundaries: both or neither
    std::vector<int32_t> row0(3 * 801, 0), col0(3 * 1001, 0);
    CHECK(check_problem(a.data(), 1000, b.data(), 800, &cs, row0.data(), nullptr, 0, 800, ps, err) == GA_E_ARG,
          "row0 without col0");
    CHECK(check_problem(a.data(), 1000, b.data(), 800, &cs, row0.data(), col0.data(), 0, 800, ps, err) == GA_OK,
          "custom boundaries: %s", err.c_str());
    row0[5] = 1 << 29;
    CHECK(check_problem(a.data(), 1000, b.data(), 800, &cs, row0.data(), col0.data(), 0, 800, ps, err) == GA_E_RANGE,
          "boundary values in the range guard");
    // the lean checkpoint store's 32-bit buffer: recompute checkpoints refused past it
    CHECK(rc_rows_fit(100000) && !rc_rows_fit((int64_t)1 << 28), "rc_rows_fit");
}

double ms_since(std::chrono::steady_clock::time_point t) {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t).count();
}

}  // namespace

int main(int argc, char** argv) {
    if (argc >= 3 && std::string(argv[1]) == "bench") {
        const int64_t steps = std::atoll(argv[2]);
        const auto st = random_state(1);
        for (int rep = 0; rep < 3; rep++) {
            RngTable R;
            auto t0 = std::chrono::steady_clock::now();
            build_rng(st.data(), steps, R);
            std::printf("table of %lld dispatches: %.3f ms\n", (long long)steps, ms_since(t0));
        }
        PyMT g;
        std::memcpy(g.mt, st.data(), sizeof(uint32_t) * MTN);
        auto t0 = std::chrono::steady_clock::now();
        const int64_t tw = steps * 32 / MTN + 1;
        for (int64_t t = 0; t < tw; t++) g.twist();
        std::printf("twists alone (%lld): %.3f ms (%u)\n", (long long)tw, ms_since(t0), g.mt[5]);
        return 0;
    }
    for (uint64_t seed = 1; seed <= 12; seed++) {
        const int64_t steps = seed <= 6 ? (int64_t)(seed * seed * 37) : (int64_t)(seed * 2111);
        test_table(seed, steps);
    }
    test_table(77, 0);
    test_table(78, 1);
    test_table(79, 50000);
    test_checks();
    if (failures) {
        std::fprintf(stderr, "%d check(s) failed\n", failures);
        return 1;
    }
    std::printf("ga_host_selftest: all checks passed\n");
    return 0;
}
