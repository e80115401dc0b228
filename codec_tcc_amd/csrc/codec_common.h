// codec_common.h -- helpers shared by the HIP translation units of libcodec_hip.so
// (error reporting, profiling hooks, wave/block scans, streaming vector loads/stores).
#pragma once
#include <hip/hip_runtime.h>

#include <atomic>
#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "codec_tcc.h"

typedef unsigned long long u64;

// ------------------------------------------------------------------ error reporting
extern thread_local char g_err[512];

static inline int set_err(int code, const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
    return code;
}

#define CODEC_EINVAL (-1000)
#define HIP_TRY(expr)                                                                     \
    do {                                                                                  \
        hipError_t e_ = (expr);                                                           \
        if (e_ != hipSuccess)                                                             \
            return set_err(-(int)e_, "%s: %s (%s:%d)", #expr, hipGetErrorString(e_),      \
                           __FILE__, __LINE__);                                           \
    } while (0)
#define LAUNCH_CHECK(name)                                                                \
    do {                                                                                  \
        hipError_t e_ = hipGetLastError();                                                \
        if (e_ != hipSuccess)                                                             \
            return set_err(-(int)e_, "launch %s: %s", name, hipGetErrorString(e_));       \
    } while (0)

// ------------------------------------------------------------------ profiling hooks
struct ProfWin {
    hipEvent_t* ev = nullptr;
    int32_t* tag = nullptr;
    int cap = 0, n = 0;
};
extern ProfWin g_prof;

struct ProfScope {   // records a start event now and the end event at scope exit
    hipStream_t st;
    int slot = -1;
    ProfScope(hipStream_t s, int tag) : st(s) {
        if (g_prof.ev && g_prof.n < g_prof.cap) {
            slot = g_prof.n++;
            g_prof.tag[slot] = tag;
            (void)hipEventRecord(g_prof.ev[2 * slot], st);   // profiling only: a failed record leaves a 0 time
        }
    }
    ~ProfScope() {
        if (slot >= 0) (void)hipEventRecord(g_prof.ev[2 * slot + 1], st);
    }
};

// ------------------------------------------------------------------ block primitives
// inclusive scan over the wave.  CODEC_WSCAN_DPP (default): each 16-lane row scanned by four
// DPP row_shr adds (lanes shifted in from outside the row read 0), the rows' totals then added
// from lanes 15 / 31 / 47 via readlane (scalars) -- no LDS round trip; 0: six __shfl_up
// (ds_bpermute) steps, the round-4 form
#ifndef CODEC_WSCAN_DPP
#define CODEC_WSCAN_DPP 1
#endif
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t x) {
    const int lane = threadIdx.x & 63;
#if CODEC_WSCAN_DPP
    int v = (int)x;
    v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xF, 0xF, true);   // row_shr:1
    v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xF, 0xF, true);   // row_shr:2
    v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xF, 0xF, true);   // row_shr:4
    v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xF, 0xF, true);   // row_shr:8
    const uint32_t r0 = (uint32_t)__builtin_amdgcn_readlane(v, 15);
    const uint32_t r1 = (uint32_t)__builtin_amdgcn_readlane(v, 31);
    const uint32_t r2 = (uint32_t)__builtin_amdgcn_readlane(v, 47);
    const int row = lane >> 4;
    uint32_t add = row >= 1 ? r0 : 0u;
    add += row >= 2 ? r1 : 0u;
    add += row >= 3 ? r2 : 0u;
    return (uint32_t)v + add;
#else
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    return x;
#endif
}

// ---- float64 across a wave without the LDS crossbar (DPP and gfx950's permlane swaps): a
// butterfly, so the order of additions is NOT numpy's -- for approximate sums only (the
// guard-banded decision's H(Y) and walk)
template <int CTRL, bool BC>
__device__ __forceinline__ double dpp_f64(double x) {
    const long long v = __double_as_longlong(x);
    const int lo = __builtin_amdgcn_update_dpp(0, (int)v, CTRL, 0xF, 0xF, BC);
    const int hi = __builtin_amdgcn_update_dpp(0, (int)(v >> 32), CTRL, 0xF, 0xF, BC);
    return __longlong_as_double(((long long)hi << 32) | (long long)(uint32_t)lo);
}
// x + (x of lane ^ 32) / (lane ^ 16), every lane (v_permlane32/16_swap of a register with itself)
__device__ __forceinline__ double xor32_sum_f64(double x) {
    const long long v = __double_as_longlong(x);
    const auto lo = __builtin_amdgcn_permlane32_swap((unsigned)v, (unsigned)v, false, false);
    const auto hi = __builtin_amdgcn_permlane32_swap((unsigned)(v >> 32), (unsigned)(v >> 32), false, false);
    return __longlong_as_double(((long long)hi[0] << 32) | (long long)lo[0]) +
           __longlong_as_double(((long long)hi[1] << 32) | (long long)lo[1]);
}
__device__ __forceinline__ double xor16_sum_f64(double x) {
    const long long v = __double_as_longlong(x);
    const auto lo = __builtin_amdgcn_permlane16_swap((unsigned)v, (unsigned)v, false, false);
    const auto hi = __builtin_amdgcn_permlane16_swap((unsigned)(v >> 32), (unsigned)(v >> 32), false, false);
    return __longlong_as_double(((long long)hi[0] << 32) | (long long)lo[0]) +
           __longlong_as_double(((long long)hi[1] << 32) | (long long)lo[1]);
}
// the wave's sum in every lane
__device__ __forceinline__ double wave_sum_f64(double x) {
    x = xor32_sum_f64(x);
    x = xor16_sum_f64(x);
    x += dpp_f64<0x128, false>(x);   // row_ror:8
    x += dpp_f64<0x124, false>(x);   // row_ror:4
    x += dpp_f64<0x4E, false>(x);    // quad_perm [2,3,0,1]
    x += dpp_f64<0xB1, false>(x);    // quad_perm [1,0,3,2]
    return x;
}
// inclusive scan inside each 16-lane row (row_shr with zero fill)
__device__ __forceinline__ double row_incl_scan_f64(double x) {
    x += dpp_f64<0x111, true>(x);
    x += dpp_f64<0x112, true>(x);
    x += dpp_f64<0x114, true>(x);
    x += dpp_f64<0x118, true>(x);
    return x;
}

// exclusive scan over the block (NT threads); sh needs NT/64+1 words
template <int NT>
__device__ uint32_t block_excl_scan(uint32_t x, uint32_t* sh, uint32_t* total) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint32_t inc = wave_incl_scan(x);
    if (lane == 63) sh[wv] = inc;
    __syncthreads();
    // every wave scans the NT/64 wave totals itself (no serial pass by one thread, one
    // barrier fewer)
    const uint32_t wt = lane < NT / 64 ? sh[lane] : 0u;
    const uint32_t wi = wave_incl_scan(wt);
    const uint32_t pre = wv ? (uint32_t)__shfl(wi, wv - 1, 64) : 0u;
    *total = (uint32_t)__shfl(wi, NT / 64 - 1, 64);
    __syncthreads();   // sh reusable
    return pre + inc - x;
}

// 64-bit variant (several packed 16-bit counters scanned at once); sh needs NT/64+1 words
template <int NT>
__device__ u64 block_excl_scan64(u64 x, u64* sh, u64* total) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    u64 inc = x;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const u64 y = __shfl_up(inc, o, 64);
        if (lane >= o) inc += y;
    }
    if (lane == 63) sh[wv] = inc;
    __syncthreads();
    if (threadIdx.x == 0) {
        u64 acc = 0;
        for (int w = 0; w < NT / 64; ++w) {
            const u64 tmp = sh[w];
            sh[w] = acc;
            acc += tmp;
        }
        sh[NT / 64] = acc;
    }
    __syncthreads();
    const u64 r = sh[wv] + inc - x;
    *total = sh[NT / 64];
    __syncthreads();
    return r;
}

// A barrier for LDS traffic only.  __syncthreads()'s workgroup fence makes hipcc wait
// vmcnt(0) first, i.e. for every outstanding global load AND store of the wave; kernels whose
// workgroups exchange data only through LDS use this instead, so stores drain and loads stay
// in flight across the barrier (cdna_hip_programming.md: raw s_barrier + lgkmcnt(0)).  The
// asm "memory" clobbers stop the compiler moving LDS accesses across it.
__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

// block_excl_scan with LDS-only barriers (see lds_barrier): global loads in flight (prefetches)
// stay in flight through it
template <int NT>
__device__ uint32_t block_excl_scan_lds(uint32_t x, uint32_t* sh, uint32_t* total) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint32_t inc = wave_incl_scan(x);
    if (lane == 63) sh[wv] = inc;
    lds_barrier();
    const uint32_t wt = lane < NT / 64 ? sh[lane] : 0u;
    const uint32_t wi = wave_incl_scan(wt);
    // the wave index is uniform: readlane instead of a bpermute round trip through the LDS crossbar
    const int wvs = __builtin_amdgcn_readfirstlane(wv);
    const uint32_t pre = wvs ? (uint32_t)__builtin_amdgcn_readlane((int)wi, wvs - 1) : 0u;
    *total = (uint32_t)__builtin_amdgcn_readlane((int)wi, NT / 64 - 1);
    lds_barrier();   // sh reusable
    return pre + inc - x;
}

// block_excl_scan64 / block_sum_u32 with LDS-only barriers (see lds_barrier)
template <int NT>
__device__ u64 block_excl_scan64_lds(u64 x, u64* sh, u64* total) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    u64 inc = x;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const u64 y = __shfl_up(inc, o, 64);
        if (lane >= o) inc += y;
    }
    if (lane == 63) sh[wv] = inc;
    lds_barrier();
    u64 base = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < NT / 64; ++w) {
        const u64 v = sh[w];
        tot += v;
        base += w < wv ? v : 0ull;
    }
    *total = tot;
    lds_barrier();   // sh is reused by the caller's next scan
    return base + inc - x;
}

template <int NT>
__device__ uint32_t block_sum_u32_lds(uint32_t x, uint32_t* sh) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) x += __shfl_xor(x, o, 64);
    if (lane == 0) sh[wv] = x;
    lds_barrier();
    uint32_t t = 0;
#pragma unroll
    for (int w = 0; w < NT / 64; ++w) t += sh[w];
    lds_barrier();
    return t;
}

template <int NT>
__device__ uint32_t block_sum_u32(uint32_t x, uint32_t* sh) {
    uint32_t tot;
    block_excl_scan<NT>(x, sh, &tot);
    return tot;
}

template <int NT>
__device__ int block_max_i32(int x, int* sh) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) x = max(x, __shfl_xor(x, o, 64));
    if (lane == 0) sh[wv] = x;
    __syncthreads();
    if (threadIdx.x == 0) {
        int m = sh[0];
        for (int w = 1; w < NT / 64; ++w) m = max(m, sh[w]);
        sh[NT / 64] = m;
    }
    __syncthreads();
    const int r = sh[NT / 64];
    __syncthreads();
    return r;
}

template <typename T> struct Vec8;
template <> struct Vec8<uint16_t> { typedef uint4 type; };
template <> struct Vec8<uint8_t> { typedef uint2 type; };

// streaming loads/stores; NT = non-temporal (measured: nt on BOTH the load and the store
// stream is what lifts a 2 GiB read+write pass from ~5.1 to ~5.9 TB/s, tools/ubench_stream.hip)
typedef unsigned int v4u __attribute__((ext_vector_type(4)));
typedef unsigned int v2u __attribute__((ext_vector_type(2)));
// cache-policy A/B (build-time, tools/r05/build_variant.sh): CODEC_PLAIN_LOADS / CODEC_PLAIN_STORES
// turn every non-temporal 16-B / 8-B vector load / store into a plain one
#ifndef CODEC_PLAIN_LOADS
#define CODEC_PLAIN_LOADS 0
#endif
#ifndef CODEC_PLAIN_STORES
#define CODEC_PLAIN_STORES 0
#endif
template <bool NT> __device__ __forceinline__ uint4 ldv(const uint4* p) {
    if constexpr (NT && !CODEC_PLAIN_LOADS) {
        const v4u x = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(p));
        return make_uint4(x.x, x.y, x.z, x.w);
    } else {
        return *p;
    }
}
template <bool NT> __device__ __forceinline__ uint2 ldv(const uint2* p) {
    if constexpr (NT && !CODEC_PLAIN_LOADS) {
        const v2u x = __builtin_nontemporal_load(reinterpret_cast<const v2u*>(p));
        return make_uint2(x.x, x.y);
    } else {
        return *p;
    }
}
// CODEC_ST_SC (A/B only): the non-temporal 16-B stores issued instead as write-through stores
// with cache-policy bits 1 = sc1, 3 = sc0 sc1 (they drop the line from the XCD's L2,
// MI355X_MICROARCH.md); inline asm, ended by s_nop 1 as the guide's store forms are.
// Measured slower on the headline (1.48 -> 1.52 ms) and the LSB scan, +-3 % on C3
// (profiles/r05/ab_store_sc.txt), so the default stays the compiler's non-temporal store.
#ifndef CODEC_ST_SC
#define CODEC_ST_SC 0
#endif
template <bool NT> __device__ __forceinline__ void stv(uint4* p, const uint4& v) {
    if constexpr (NT && CODEC_ST_SC == 1) {
        v4u x = {v.x, v.y, v.z, v.w};
        asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" ::"v"(p), "v"(x) : "memory");
    } else if constexpr (NT && CODEC_ST_SC == 3) {
        v4u x = {v.x, v.y, v.z, v.w};
        asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1\n\ts_nop 1" ::"v"(p), "v"(x) : "memory");
    } else if constexpr (NT && !CODEC_PLAIN_STORES) {
        v4u x = {v.x, v.y, v.z, v.w};
        __builtin_nontemporal_store(x, reinterpret_cast<v4u*>(p));
    } else {
        *p = v;
    }
}
template <bool NT> __device__ __forceinline__ void stv(uint2* p, const uint2& v) {
    if constexpr (NT && !CODEC_PLAIN_STORES) {
        v2u x = {v.x, v.y};
        __builtin_nontemporal_store(x, reinterpret_cast<v2u*>(p));
    } else {
        *p = v;
    }
}

__device__ __forceinline__ uint32_t vor_of(const uint4& v) { return v.x | v.y | v.z | v.w; }
__device__ __forceinline__ uint32_t vor_of(const uint2& v) { return v.x | v.y; }

__device__ __forceinline__ uint32_t lsb_count(const uint4& v) {
    return __popc(v.x & 0x00010001u) + __popc(v.y & 0x00010001u) + __popc(v.z & 0x00010001u) +
           __popc(v.w & 0x00010001u);
}
__device__ __forceinline__ uint32_t lsb_count(const uint2& v) {
    return __popc(v.x & 0x01010101u) + __popc(v.y & 0x01010101u);
}

static inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

// launch-shape knobs (the defaults are the measured best on MI355X).  An environment override
// is honoured only while the tuning switch is on: CODEC_TUNING=1 in the
// environment when the library is loaded (read once, at load), or codec_set_tuning(1) (A/B
// tools, the test suite).  With the switch off -- the product default -- every knob is its
// default and no launch reads the environment, so a stray CODEC_* variable cannot change which
// kernels run and getenv never races a setenv in another thread.
extern std::atomic<int> g_tuning;
static inline bool tuning_on() { return g_tuning.load(std::memory_order_relaxed) != 0; }
static long long knob(const char* name, long long dflt) {
    if (!tuning_on()) return dflt;
    const char* v = getenv(name);
    return (v && *v) ? atoll(v) : dflt;
}

// fault-injection and spin-bound knobs (tests only): live only under the tuning switch AND
// either a -DCODEC_DEBUG_KNOBS build or the master switch CODEC_DEBUG=1, so a leaked
// CODEC_PEE_DEBUG_SKIP cannot make a production launch skip a publish
static inline bool debug_knobs_enabled() {
#ifdef CODEC_DEBUG_KNOBS
    return tuning_on();
#else
    if (!tuning_on()) return false;
    const char* v = getenv("CODEC_DEBUG");
    return v && v[0] == '1' && v[1] == 0;
#endif
}
static long long debug_knob(const char* name, long long dflt) {
    return debug_knobs_enabled() ? knob(name, dflt) : dflt;
}

static inline size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

// CUs of the current device (cached per device): slice-serial dispatch decisions
static inline int device_cu_count() {
    static int cached[64] = {0};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
    if (!cached[dev]) {
        int n = 0;
        if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
        cached[dev] = n;
    }
    return cached[dev];
}
