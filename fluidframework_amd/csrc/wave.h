// wave.h — the wave-collective vocabulary the merge-tree engine is written in.
//
// The engine runs one 64-lane wavefront per document.  Control flow is
// wave-uniform ("scalar" code that every lane executes identically, so every
// lane holds the same value and may store it), and data-parallel sections are
// expressed with wave_map() over at most 64 items followed by collectives
// (ballot, first, exclusive scan, sum, broadcast).  On gfx950 a LaneArr<T> is
// the lane's own register and the collectives lower to ballot/DPP/ds_swizzle;
// the same source also compiles for the host (MT_WAVE_EMULATION, tests only),
// where a LaneArr<T> is a 64-element array.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define MT_HD __host__ __device__ __attribute__((always_inline))
#define MT_LAM __attribute__((always_inline))
#define MT_INLINE __host__ __device__ __forceinline__
#else
#define MT_HD inline
#define MT_LAM
#define MT_INLINE inline
#endif

#define MT_WAVE 64

// One lane copies n UTF-16 units with 8 independent loads in flight per step
// (a per-unit load->store chain would pay a full memory round trip per unit).
MT_INLINE void lane_copy16(uint16_t* dst, const uint16_t* src, int n) {
    int q = 0;
    for (; q + 8 <= n; q += 8) {
        uint16_t t[8];
#pragma unroll
        for (int j = 0; j < 8; j++) t[j] = src[q + j];
#pragma unroll
        for (int j = 0; j < 8; j++) dst[q + j] = t[j];
    }
    for (; q < n; q++) dst[q] = src[q];
}

#if defined(__HIP_DEVICE_COMPILE__)
// ---------------------------------------------------------------- device ----
template <class T> using LaneArr = T;
// Mark a wave-uniform 32-bit value as such (moves it to an SGPR).
__device__ __forceinline__ int uni(int x) { return __builtin_amdgcn_readfirstlane(x); }
__device__ __forceinline__ uint32_t uni(uint32_t x) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)x); }
__device__ __forceinline__ unsigned long long uni64(unsigned long long x) {
    return (unsigned long long)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)x) |
           ((unsigned long long)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(x >> 32)) << 32);
}

__device__ __forceinline__ int wave_lane() { return __lane_id(); }

template <class F>
__device__ __forceinline__ auto wave_map(int n, F f) -> decltype(f(0)) {
    using T = decltype(f(0));
    T v{};
    const int k = __lane_id();
    if (k < n) v = f(k);
    return v;
}
template <class F>
__device__ __forceinline__ void wave_for(int n, F f) {
    const int k = __lane_id();
    if (k < n) f(k);
}
template <class T> __device__ __forceinline__ T own(T a, int) { return a; }   // by value: no address-of, so no select-of-pointers
__device__ __forceinline__ int wave_at(int a, int j) { return __builtin_amdgcn_readlane(a, j); }
__device__ __forceinline__ uint32_t wave_at(uint32_t a, int j) { return (uint32_t)__builtin_amdgcn_readlane((int)a, j); }
__device__ __forceinline__ bool wave_at(bool a, int j) { return __builtin_amdgcn_readlane((int)a, j) != 0; }
__device__ __forceinline__ uint64_t wave_ballot(bool p) { return __ballot(p); }
__device__ __forceinline__ int wave_first(bool p) {
    uint64_t b = __ballot(p);
    return b ? __ffsll((unsigned long long)b) - 1 : -1;
}
__device__ __forceinline__ int wave_count(bool p) { return __popcll(__ballot(p)); }
// exclusive prefix count of p over lanes below this one
__device__ __forceinline__ int wave_rank(bool p) {
    uint64_t b = __ballot(p);
    return __popcll(b & ((1ull << __lane_id()) - 1ull));
}
// Scans and sums run on DPP (row_shr within 16-lane rows, then row_bcast:15/31
// across rows): VALU-latency chains instead of ds_bpermute round trips.
template <int CTRL, int ROWS = 0xf>
__device__ __forceinline__ int dpp0(int x) { return __builtin_amdgcn_update_dpp(0, x, CTRL, ROWS, 0xf, false); }
__device__ __forceinline__ int wave_incl_scan(int v) {
    int x = v;
    x += dpp0<0x111>(x);          // row_shr:1
    x += dpp0<0x112>(x);          // row_shr:2
    x += dpp0<0x114>(x);          // row_shr:4
    x += dpp0<0x118>(x);          // row_shr:8
    x += dpp0<0x142, 0xa>(x);     // row_bcast:15 -> rows 1, 3
    x += dpp0<0x143, 0xc>(x);     // row_bcast:31 -> rows 2, 3
    return x;
}
__device__ __forceinline__ int wave_sum(int v) { return __builtin_amdgcn_readlane(wave_incl_scan(v), 63); }
__device__ __forceinline__ int wave_excl_scan(int v) { return wave_incl_scan(v) - v; }
// Same for data held in lanes 0..7 (a block's children): three row shifts.
__device__ __forceinline__ int wave_incl_scan8(int v) {
    int x = v;
    x += dpp0<0x111>(x);
    x += dpp0<0x112>(x);
    x += dpp0<0x114>(x);
    return x;
}
__device__ __forceinline__ int wave_sum8(int v) { return __builtin_amdgcn_readlane(wave_incl_scan8(v), 7); }
__device__ __forceinline__ int wave_excl_scan8(int v) { return wave_incl_scan8(v) - v; }
// lane i receives a[i + off] (0 outside [0, 64)); call from uniform control flow
__device__ __forceinline__ int wave_from(int a, int off) {
    const int src = __lane_id() + off;
    const int v = __shfl(a, src & 63);
    return (src >= 0 && src < 64) ? v : 0;
}
// lanes 0..7 receive a[i + OFF] from within the first 16 lanes (DPP row shift)
template <int OFF> __device__ __forceinline__ int wave_from8(int a) {
    static_assert(OFF != 0 && OFF > -16 && OFF < 16, "row shift");
    if constexpr (OFF < 0) return dpp0<0x110 | (-OFF)>(a);
    else return dpp0<0x100 | OFF>(a);
}
// lane t receives a[t / 8] (one value per group of 8 lanes); call from uniform control flow
__device__ __forceinline__ int wave_gather8(int a) { return __shfl(a, __lane_id() >> 3); }
// lane t receives a[src(t)] (src in [0, 64)); call from uniform control flow
template <class F> __device__ __forceinline__ int wave_shfl(int a, F src) { return __shfl(a, src(__lane_id())); }
// lane k's value replaced by v (k uniform)
__device__ __forceinline__ int wave_set(int a, int k, int v) { return __lane_id() == k ? v : a; }
// per-lane add into wave-private LDS (conflicting lanes serialize in hardware)
__device__ __forceinline__ void lds_add(int* p, int v) { __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT); }
// keeps a loaded value alive (a prefetch whose result is otherwise unused)
__device__ __forceinline__ void mt_keep(int v) { __asm__ volatile("" ::"v"(v)); }
// the same value, opaque to the compiler: lane-index arithmetic behind it is not hoisted to the
// kernel's entry (where it would hold a VGPR, or a spill slot, across the whole replay loop)
__device__ __forceinline__ int mt_opaque(int v) { __asm__ volatile("" : "+v"(v)); return v; }
// per-lane compare-and-swap on LDS; returns the old value
__device__ __forceinline__ int lds_cas(int* p, int cmp, int v) {
    __hip_atomic_compare_exchange_strong(p, &cmp, v, __ATOMIC_RELAXED, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
    return cmp;
}
// Lane 0 takes the next slot of a global 64-bit cursor; every lane gets its index.
__device__ __forceinline__ unsigned long long wave_atomic_add(unsigned long long* p, unsigned long long d) {
    unsigned long long v = 0;
    if (__lane_id() == 0) v = __hip_atomic_fetch_add(p, d, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return (unsigned long long)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)v) |
           ((unsigned long long)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(v >> 32)) << 32);
}
__device__ __forceinline__ unsigned long long wave_atomic_next(unsigned long long* p) { return wave_atomic_add(p, 1ull); }
// 64-bit sum over all lanes (butterfly of 64-bit shuffles), wave-uniform result
__device__ __forceinline__ unsigned long long wave_sum64(unsigned long long v) {
    for (int off = 32; off >= 1; off >>= 1) v += (unsigned long long)__shfl_xor((long)v, off);
    return uni64(v);
}
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
}
#else
// ------------------------------------------------------ host emulation ----
#include <string.h>
template <class T> struct LaneArr {
    T v[MT_WAVE];
};
inline int wave_lane() { return 0; }
inline int uni(int x) { return x; }
inline uint32_t uni(uint32_t x) { return x; }
inline unsigned long long uni64(unsigned long long x) { return x; }

template <class F>
inline auto wave_map(int n, F f) -> LaneArr<decltype(f(0))> {
    LaneArr<decltype(f(0))> a;
    for (int k = 0; k < MT_WAVE; k++) a.v[k] = decltype(f(0)){};
    for (int k = 0; k < n && k < MT_WAVE; k++) a.v[k] = f(k);
    return a;
}
template <class F> inline void wave_for(int n, F f) {
    for (int k = 0; k < n && k < MT_WAVE; k++) f(k);
}
template <class T> inline T own(const LaneArr<T>& a, int k) { return a.v[k]; }
template <class T> inline T wave_at(const LaneArr<T>& a, int j) { return a.v[j]; }
inline uint64_t wave_ballot(const LaneArr<bool>& p) {
    uint64_t b = 0;
    for (int k = 0; k < MT_WAVE; k++) if (p.v[k]) b |= 1ull << k;
    return b;
}
inline int wave_first(const LaneArr<bool>& p) {
    for (int k = 0; k < MT_WAVE; k++) if (p.v[k]) return k;
    return -1;
}
inline int wave_count(const LaneArr<bool>& p) {
    int c = 0;
    for (int k = 0; k < MT_WAVE; k++) c += p.v[k] ? 1 : 0;
    return c;
}
inline LaneArr<int> wave_rank(const LaneArr<bool>& p) {
    LaneArr<int> r; int c = 0;
    for (int k = 0; k < MT_WAVE; k++) { r.v[k] = c; c += p.v[k] ? 1 : 0; }
    return r;
}
inline int wave_sum(const LaneArr<int>& a) {
    int s = 0;
    for (int k = 0; k < MT_WAVE; k++) s += a.v[k];
    return s;
}
inline LaneArr<int> wave_excl_scan(const LaneArr<int>& a) {
    LaneArr<int> r; int s = 0;
    for (int k = 0; k < MT_WAVE; k++) { r.v[k] = s; s += a.v[k]; }
    return r;
}
inline int wave_sum8(const LaneArr<int>& a) {
    int s = 0;
    for (int k = 0; k < 8; k++) s += a.v[k];
    return s;
}
inline LaneArr<int> wave_excl_scan8(const LaneArr<int>& a) { return wave_excl_scan(a); }
inline LaneArr<int> wave_from(const LaneArr<int>& a, int off) {
    LaneArr<int> r;
    for (int k = 0; k < MT_WAVE; k++) { const int s = k + off; r.v[k] = (s >= 0 && s < MT_WAVE) ? a.v[s] : 0; }
    return r;
}
template <int OFF> inline LaneArr<int> wave_from8(const LaneArr<int>& a) {
    LaneArr<int> r;
    for (int k = 0; k < MT_WAVE; k++) { const int s = (k & 15) + OFF; r.v[k] = (s >= 0 && s < 16) ? a.v[(k & ~15) + s] : 0; }
    return r;
}
inline LaneArr<int> wave_gather8(const LaneArr<int>& a) {
    LaneArr<int> r;
    for (int t = 0; t < MT_WAVE; t++) r.v[t] = a.v[t >> 3];
    return r;
}
template <class F> inline LaneArr<int> wave_shfl(const LaneArr<int>& a, F src) {
    LaneArr<int> r;
    for (int t = 0; t < MT_WAVE; t++) r.v[t] = a.v[src(t) & 63];
    return r;
}
inline LaneArr<int> wave_set(LaneArr<int> a, int k, int v) { if (k >= 0 && k < MT_WAVE) a.v[k] = v; return a; }
inline void lds_add(int* p, int v) { *p += v; }
inline int lds_cas(int* p, int cmp, int v) { const int o = *p; if (o == cmp) *p = v; return o; }
inline void mt_keep(int) {}
inline int mt_opaque(int v) { return v; }
inline unsigned long long wave_atomic_add(unsigned long long* p, unsigned long long d) { return __atomic_fetch_add(p, d, __ATOMIC_RELAXED); }
inline unsigned long long wave_atomic_next(unsigned long long* p) { return wave_atomic_add(p, 1ull); }
inline unsigned long long wave_sum64(const LaneArr<unsigned long long>& a) {
    unsigned long long s = 0;
    for (int k = 0; k < MT_WAVE; k++) s += a.v[k];
    return s;
}
inline void wave_sync() {}
#endif
