// ga_sync.h -- LDS / global-memory synchronisation helpers shared by the fill kernels
// (ga_kernels.hip, ga_lane.hip): counters, hand-off rows, bounded spins.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace ga {

#define RLX __ATOMIC_RELAXED
#define AGENT __HIP_MEMORY_SCOPE_AGENT
#define WGS __HIP_MEMORY_SCOPE_WORKGROUP
__device__ __forceinline__ unsigned lds_ld(unsigned* p) { return __hip_atomic_load(p, __ATOMIC_ACQUIRE, WGS); }
__device__ __forceinline__ unsigned sgpr_u(unsigned x) { return (unsigned)__builtin_amdgcn_readfirstlane((int)x); }
// wave-uniform counter read (scalar control flow): LDS executes a wave's operations in
// order, so a relaxed read of a counter published after its data is enough
__device__ __forceinline__ unsigned lds_ldu(unsigned* p) {
    return (unsigned)__builtin_amdgcn_readfirstlane((int)__hip_atomic_load(p, __ATOMIC_RELAXED, WGS));
}
__device__ __forceinline__ void lds_st(unsigned* p, unsigned v) { __hip_atomic_store(p, v, __ATOMIC_RELEASE, WGS); }
__device__ __forceinline__ unsigned g_ld(const unsigned* p) {
    return __hip_atomic_load(const_cast<unsigned*>(p), RLX, AGENT);
}
__device__ __forceinline__ void g_st(unsigned* p, unsigned v) { __hip_atomic_store(p, v, RLX, AGENT); }
__device__ __forceinline__ unsigned long long g_ld64(const int2* p) {
    return __hip_atomic_load(reinterpret_cast<unsigned long long*>(const_cast<int2*>(p)), RLX, AGENT);
}
__device__ __forceinline__ void g_st64(int2* p, int2 v) {
    unsigned long long x = (unsigned long long)(unsigned)v.x | ((unsigned long long)(unsigned)v.y << 32);
    __hip_atomic_store(reinterpret_cast<unsigned long long*>(p), x, RLX, AGENT);
}
__device__ __forceinline__ int2 unpack64(unsigned long long x) { return make_int2((int)(unsigned)x, (int)(x >> 32)); }
// A multi-GPU slab's halo and progress words: the left edge lands while the fill
// runs (written by an RCCL kernel into device memory, or by the host into pinned memory) and the
// right edge is read by the host / an RCCL kernel once its progress word covers it.  Both sides
// use system-scope accesses (written through / read past every GPU cache), and the data stores
// complete (s_waitcnt vmcnt(0)) before the progress word is stored.
__device__ __forceinline__ unsigned s_ld(const unsigned* p) {
    return __hip_atomic_load(const_cast<unsigned*>(p), RLX, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ unsigned long long s_ld64(const int2* p) {
    return __hip_atomic_load(reinterpret_cast<unsigned long long*>(const_cast<int2*>(p)), RLX,
                             __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void s_st64(int2* p, int2 v) {
    unsigned long long x = (unsigned long long)(unsigned)v.x | ((unsigned long long)(unsigned)v.y << 32);
    __hip_atomic_store(reinterpret_cast<unsigned long long*>(p), x, RLX, __HIP_MEMORY_SCOPE_SYSTEM);
}
// the progress word's value once its writer has aborted (never a row count)
constexpr unsigned PROG_ABORT = 0xffffffffu;
__device__ __forceinline__ void s_prog_abort(unsigned* p) {
    __hip_atomic_store(p, PROG_ABORT, RLX, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Bounded spin: returns false (and raises the abort word) after `limit` sleeps.
__device__ __forceinline__ bool spin_ok(unsigned& spins, unsigned limit, unsigned* abort_word) {
    __builtin_amdgcn_s_sleep(1);
    if (++spins >= limit) {
        g_st(abort_word, 1u);
        return false;
    }
    if ((spins & 1023u) == 0 && g_ld(abort_word)) return false;
    return true;
}

// Bounded spin for compute waves: LDS-only (no global memory op may appear in their
// loop, or the compiler's vmcnt bookkeeping turns the prefetch waits into vmcnt(0)).
__device__ __forceinline__ bool spin_ok_lds(unsigned& spins, unsigned limit, unsigned* abort_sh) {
    __builtin_amdgcn_s_sleep(1);
    if (++spins >= limit) {
        __hip_atomic_store(abort_sh, 1u, __ATOMIC_RELAXED, WGS);
        return false;
    }
    if ((spins & 255u) == 0 && lds_ldu(abort_sh)) return false;
    return true;
}

// LDS byte address of a __shared__ object (for hand-issued ds_read / ds_write)
template <typename T>
__device__ __forceinline__ unsigned lds_addr(T* p) {
    return (unsigned)(uintptr_t)(__attribute__((address_space(3))) T*)p;
}

}  // namespace ga
