// Cost of the decision's numpy-order float64 sums (np_sum_wave and friends) in isolation:
// one workgroup, `nact` waves each summing the same m terms from LDS (m ~ 3 300 for a ct12
// 512^2 slice), stamps (s_memtime, shader clocks) around the leaf phase and the tree combine.
// Variants must return the bit pattern np_sum_wave returns (a bit check over 644 sizes runs
// first).  Variants: 8 lanes per leaf (lane q = numpy's r[q]), with shuffles (wave8), with DPP
// and two passes in flight (wave8b), branch-free (wave8c), per half-tree for the decision's
// paired MI round (pairs8, pairs8c), and the current one-lane-per-slot layout with branch-free
// node sizes (wave_bf, pairs bf).  Results: profiles/r05/ubench_npsum.txt; the kernels' A/B:
// profiles/r05/ab_npsum.txt (nothing adopted).
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -Iinclude -Icodec_tcc_amd/csrc \
//         tools/ubench_npsum.hip -o tools/bin/ubench_npsum
#include "codec_hip.hip"

#include <math.h>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

// variant 1: np_sum_wave with the stamps split (leaves | combine)
template <class F>
__device__ double npw_stamped(const F& f, int m, long long* t1) {
    const int lane = threadIdx.x & 63;
    double res = -0.0;
    for (int cs = 0; cs < m; cs += NP_CHUNK) {
        const int r = min(NP_CHUNK, m - cs);
        int aA, aB;
        const int nA = np_node_size(r, 7, lane, &aA);
        const int nB = np_node_size(r, 7, lane + 64, &aB);
        const double vA = nA > 0 ? np_leaf(f, cs + aA, nA) : 0.0;
        const double vB = nB > 0 ? np_leaf(f, cs + aB, nB) : 0.0;
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        *t1 = __builtin_amdgcn_s_memtime();
        res += np_combine_wave(vA, vB, r);
    }
    return res;
}


// k-th (0-based) set bit of the 128-bit mask (lo, hi); k < popc
__device__ __forceinline__ int select128(u64 lo, u64 hi, int k) {
    const int cl = __popcll(lo);
    u64 m = k < cl ? lo : hi;
    int pos = k < cl ? 0 : 64;
    k = k < cl ? k : k - cl;
#pragma unroll
    for (int w = 32; w >= 1; w >>= 1) {
        const u64 low = m & ((1ull << w) - 1ull);
        const int c = __popcll(low);
        const bool up = k >= c;
        k = up ? k - c : k;
        m = up ? (m >> w) : low;
        pos += up ? w : 0;
    }
    return pos;
}

// variant 2: 8 lanes per leaf (lane q = numpy's accumulator r[q]), the 128 slots' leaves taken
// 8 at a time in slot order, their sums routed back to the slot lanes for np_combine_wave
template <class F>
__device__ double np_sum_wave8(const F& f, int m) {
    const int lane = threadIdx.x & 63, g = lane >> 3, q = lane & 7;
    double res = -0.0;
    for (int cs = 0; cs < m; cs += NP_CHUNK) {
        const int r = min(NP_CHUNK, m - cs);
        int aA, aB;
        const int nA = np_node_size(r, 7, lane, &aA);
        const int nB = np_node_size(r, 7, lane + 64, &aB);
        const u64 MA = __ballot(nA > 0), MB = __ballot(nB > 0);
        const int nl = __popcll(MA) + __popcll(MB);
        const int kA = (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(MA >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)MA, 0u));
        const int kB = __popcll(MA) + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(MB >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)MB, 0u));
        double vA = 0.0, vB = 0.0;
        for (int k0 = 0; k0 < nl; k0 += 8) {
            const int k = k0 + g;
            const int slot = k < nl ? select128(MA, MB, k) : 0;
            const int xa = __shfl(aA, slot & 63, 64), xb = __shfl(aB, slot & 63, 64);
            const int ya = __shfl(nA, slot & 63, 64), yb = __shfl(nB, slot & 63, 64);
            const int a = cs + (slot < 64 ? xa : xb);
            const int n = k < nl ? (slot < 64 ? ya : yb) : 0;
            const int lim = n >= 8 ? n - (n % 8) : 0;
            double tv[NP_LEAF / 8];
#pragma unroll
            for (int u = 0; u < NP_LEAF / 8; ++u) tv[u] = (8 * u < lim) ? f(a + 8 * u + q) : 0.0;
            double acc = tv[0];
#pragma unroll
            for (int u = 1; u < NP_LEAF / 8; ++u)
                if (8 * u < lim) acc += tv[u];
            const double s2 = acc + __shfl_xor(acc, 1, 64);
            const double s4 = s2 + __shfl_xor(s2, 2, 64);
            double s8 = s4 + __shfl_xor(s4, 4, 64);
            if (q == 0 && n > 0) {
                if (n >= 8) {
                    for (int i = lim; i < n; ++i) s8 += f(a + i);
                } else {
                    s8 = -0.0;
                    for (int i = 0; i < n; ++i) s8 += f(a + i);
                }
            }
            const double gA = __shfl(s8, 8 * (kA & 7), 64), gB = __shfl(s8, 8 * (kB & 7), 64);
            if (nA > 0 && (kA >> 3) == (k0 >> 3)) vA = gA;
            if (nB > 0 && (kB >> 3) == (k0 >> 3)) vB = gB;
        }
        res += np_combine_wave(vA, vB, r);
    }
    return res;
}

template <int C>
__device__ __forceinline__ double dppd(double x) {
    const long long b = __double_as_longlong(x);
    const int lo = __builtin_amdgcn_update_dpp(0, (int)b, C, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), C, 0xF, 0xF, false);
    return __longlong_as_double(((long long)hi << 32) | (long long)(uint32_t)lo);
}

// k-th (0-based) set bit of a 64-bit mask
__device__ __forceinline__ int select64(u64 m, int k) {
    int pos = 0;
#pragma unroll
    for (int w = 32; w >= 1; w >>= 1) {
        const u64 low = m & ((1ull << w) - 1ull);
        const int c = __popcll(low);
        const bool up = k >= c;
        k = up ? k - c : k;
        m = up ? (m >> w) : low;
        pos += up ? w : 0;
    }
    return pos;
}

// one pass of 8 leaves, 8 lanes each (lane q = numpy's r[q]); the leaf's sum in lane q == 0
template <class F>
__device__ __forceinline__ double leaf8_sum(const F& f, int a, int n, int q, const double (&tv)[NP_LEAF / 8]) {
    const int lim = n >= 8 ? n - (n % 8) : 0;
    double acc = tv[0];
#pragma unroll
    for (int u = 1; u < NP_LEAF / 8; ++u)
        if (8 * u < lim) acc += tv[u];
    const double s2 = acc + dppd<0xB1>(acc);     // quad_perm [1,0,3,2]: r0+r1, r2+r3, ...
    const double s4 = s2 + dppd<0x4E>(s2);       // quad_perm [2,3,0,1]: (r0+r1)+(r2+r3)
    double s8 = s4 + dppd<0x141>(s4);            // row_half_mirror: lane 0 gets lane 7's (r6+r7)+(r4+r5)
    if (q == 0 && n > 0) {
        if (n >= 8) {
            for (int i = lim; i < n; ++i) s8 += f(a + i);
        } else {
            s8 = -0.0;
            for (int i = 0; i < n; ++i) s8 += f(a + i);
        }
    }
    return s8;
}

template <class F>
__device__ __forceinline__ void leaf8_load(const F& f, int a, int n, int q, double (&tv)[NP_LEAF / 8]) {
    const int lim = n >= 8 ? n - (n % 8) : 0;
#pragma unroll
    for (int u = 0; u < NP_LEAF / 8; ++u) tv[u] = (8 * u < lim) ? f(a + 8 * u + q) : 0.0;
}

// slot values of the 64 slots [base, base + 64) of a chunk tree (r elements at cs): lane l
// returns slot base + l's leaf sum (0 if the slot holds no leaf)
template <class F>
__device__ __forceinline__ double ub_slots8(const F& f, int cs, int r, int base) {
    const int lane = threadIdx.x & 63, g = lane >> 3, q = lane & 7;
    int aS;
    const int nS = np_node_size(r, 7, lane + base, &aS);
    const u64 M = __ballot(nS > 0);
    const int nl = __popcll(M);
    const int kS = (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(M >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)M, 0u));
    double v = 0.0;
    for (int k0 = 0; k0 < nl; k0 += 16) {      // two passes of 8 leaves, loads of both first
        const int k1 = k0 + g, k2 = k0 + 8 + g;
        const int s1 = k1 < nl ? select64(M, k1) : 0, s2 = k2 < nl ? select64(M, k2) : 0;
        const int a1 = cs + __shfl(aS, s1, 64), a2 = cs + __shfl(aS, s2, 64);
        // shuffles outside the conditionals: a bpermute only reads lanes active in it
        const int m1 = __shfl(nS, s1, 64), m2 = __shfl(nS, s2, 64);
        const int n1 = k1 < nl ? m1 : 0, n2 = k2 < nl ? m2 : 0;
        double t1[NP_LEAF / 8], t2[NP_LEAF / 8];
        leaf8_load(f, a1, n1, q, t1);
        leaf8_load(f, a2, n2, q, t2);
        const double r1 = leaf8_sum(f, a1, n1, q, t1);
        const double r2 = leaf8_sum(f, a2, n2, q, t2);
        const double g1 = __shfl(r1, 8 * (kS & 7), 64), g2 = __shfl(r2, 8 * (kS & 7), 64);
        if (nS > 0 && (kS >> 3) == (k0 >> 3)) v = g1;
        if (nS > 0 && (kS >> 3) == (k0 >> 3) + 1) v = g2;
    }
    return v;
}

template <class F>
__device__ __forceinline__ double ub_slots8_st(const F& f, int cs, int r, int base, long long* st) {
    const int lane = threadIdx.x & 63, g = lane >> 3, q = lane & 7;
    int aS;
    const int nS = np_node_size(r, 7, lane + base, &aS);
    const u64 M = __ballot(nS > 0);
    const int nl = __popcll(M);
    const int kS = (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(M >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)M, 0u));
    double v = 0.0;
    int si = 0;
#define STMP() do { asm volatile("s_waitcnt lgkmcnt(0) vmcnt(0)" ::: "memory"); if (si < 30) st[si++] = __builtin_amdgcn_s_memtime(); } while (0)
    STMP();
    for (int k0 = 0; k0 < nl; k0 += 16) {      // two passes of 8 leaves, loads of both first
        const int k1 = k0 + g, k2 = k0 + 8 + g;
        const int s1 = k1 < nl ? select64(M, k1) : 0, s2 = k2 < nl ? select64(M, k2) : 0;
        const int a1 = cs + __shfl(aS, s1, 64), a2 = cs + __shfl(aS, s2, 64);
        // shuffles outside the conditionals: a bpermute only reads lanes active in it
        const int m1 = __shfl(nS, s1, 64), m2 = __shfl(nS, s2, 64);
        const int n1 = k1 < nl ? m1 : 0, n2 = k2 < nl ? m2 : 0;
        STMP();
        double t1[NP_LEAF / 8], t2[NP_LEAF / 8];
        leaf8_load(f, a1, n1, q, t1);
        leaf8_load(f, a2, n2, q, t2);
        STMP();
        const double r1 = leaf8_sum(f, a1, n1, q, t1);
        const double r2 = leaf8_sum(f, a2, n2, q, t2);
        STMP();
        const double g1 = __shfl(r1, 8 * (kS & 7), 64), g2 = __shfl(r2, 8 * (kS & 7), 64);
        if (nS > 0 && (kS >> 3) == (k0 >> 3)) v = g1;
        if (nS > 0 && (kS >> 3) == (k0 >> 3) + 1) v = g2;
    }
    STMP();
#undef STMP
    return v;
}

template <class F>
__device__ double np_sum_wave8b(const F& f, int m) {
    double res = -0.0;
    for (int cs = 0; cs < m; cs += NP_CHUNK) {
        const int r = min(NP_CHUNK, m - cs);
        const double vA = ub_slots8(f, cs, r, 0);
        const double vB = ub_slots8(f, cs, r, 64);
        res += np_combine_wave(vA, vB, r);
    }
    return res;
}

// ---- branch-free variants (v3)
// node (D, j)'s size and start in a chunk tree of r elements, straight-line selects
template <int D>
__device__ __forceinline__ int nns_bf(int r, int j, int* start) {
    int a = 0, n = r;
#pragma unroll
    for (int l = D - 1; l >= 0; --l) {
        const bool bit = (j >> l) & 1;
        const bool big = n > NP_LEAF;
        const int n2 = (n >> 1) & ~7;
        a += (big && bit) ? n2 : 0;
        n = big ? (bit ? n - n2 : n2) : (bit ? 0 : n);
    }
    *start = a;
    return n;
}

__device__ __forceinline__ double np_combine_wave_bf(double vA, double vB, int r) {
    const int lane = threadIdx.x & 63;
    const int s0 = (2 * lane) & 63;
    const double lA = __shfl(vA, s0, 64), rA = __shfl(vA, s0 + 1, 64);
    const double lB = __shfl(vB, s0, 64), rB = __shfl(vB, s0 + 1, 64);
    int a6;
    const int n6 = nns_bf<6>(r, lane, &a6);
    const double L6 = lane < 32 ? lA : lB, R6 = lane < 32 ? rA : rB;
    double v = n6 > NP_LEAF ? L6 + R6 : L6;
    int ad;
#define NPC_LEVEL(D)                                                    \
    {                                                                   \
        const double L = __shfl(v, (2 * lane) & 63, 64);                \
        const double R = __shfl(v, (2 * lane + 1) & 63, 64);            \
        const int nd = nns_bf<D>(r, lane, &ad);                         \
        v = nd > NP_LEAF ? L + R : L;                                   \
    }
    NPC_LEVEL(5) NPC_LEVEL(4) NPC_LEVEL(3) NPC_LEVEL(2) NPC_LEVEL(1) NPC_LEVEL(0)
#undef NPC_LEVEL
    return __shfl(v, 0, 64);
}

// one pass of 8 leaves (8 lanes each), branch-free: every lane issues its 16 loads and its
// tail load (clamped in-bounds addresses, masked values), the accumulators add -0.0 (an exact
// identity) past the leaf's end, the tail is brought to lane q = 0 by DPP row shifts
template <class F>
__device__ __forceinline__ void leafc_load(const F& f, int a, int n, int q, int mmax, double (&tv)[NP_LEAF / 8], double& tq) {
    const int lim = n >= 8 ? n - (n % 8) : 0;
#pragma unroll
    for (int u = 0; u < NP_LEAF / 8; ++u) {
        const int i = min(a + 8 * u + q, mmax);
        const double x = f(i);
        tv[u] = (8 * u < lim) ? x : -0.0;
    }
    const int it = min(a + lim + q, mmax);
    const double xt = f(it);
    tq = (lim + q < n) ? xt : -0.0;
}

template <class F>
__device__ __forceinline__ double leafc_sum(int n, const double (&tv)[NP_LEAF / 8], double tq) {
    double acc = tv[0];
#pragma unroll
    for (int u = 1; u < NP_LEAF / 8; ++u) acc += tv[u];
    const double s2 = acc + dppd<0xB1>(acc);
    const double s4 = s2 + dppd<0x4E>(s2);
    double s8 = s4 + dppd<0x141>(s4);
    // tail elements lim .. n-1 sit in lanes q = 0 .. n%8-1 (tq); lane q = 0 adds them in order
    const double t1 = dppd<0x101>(tq), t2 = dppd<0x102>(tq), t3 = dppd<0x103>(tq);
    const double t4 = dppd<0x104>(tq), t5 = dppd<0x105>(tq), t6 = dppd<0x106>(tq);
    if (n < 8) s8 = -0.0;     // numpy's n < 8 loop starts from -0.0 and adds every element
    s8 += tq; s8 += t1; s8 += t2; s8 += t3; s8 += t4; s8 += t5; s8 += t6;
    return s8;
}

template <class F>
__device__ __forceinline__ double np_slots8c(const F& f, int cs, int r, int base, int mmax) {
    const int lane = threadIdx.x & 63, g = lane >> 3, q = lane & 7;
    int aS;
    const int nS = nns_bf<7>(r, lane + base, &aS);
    const u64 M = __ballot(nS > 0);
    const int nl = __popcll(M);
    const int kS = (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(M >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)M, 0u));
    double v = 0.0;
    for (int k0 = 0; k0 < nl; k0 += 16) {
        const int k1 = k0 + g, k2 = k0 + 8 + g;
        const int s1 = select64(M, min(k1, nl - 1)), s2 = select64(M, min(k2, nl - 1));
        const int a1 = cs + __shfl(aS, s1, 64), a2 = cs + __shfl(aS, s2, 64);
        const int m1 = __shfl(nS, s1, 64), m2 = __shfl(nS, s2, 64);
        const int n1 = k1 < nl ? m1 : 0, n2 = k2 < nl ? m2 : 0;
        double t1[NP_LEAF / 8], t2[NP_LEAF / 8], q1, q2;
        leafc_load(f, a1, n1, q, mmax, t1, q1);
        leafc_load(f, a2, n2, q, mmax, t2, q2);
        const double r1 = leafc_sum<F>(n1, t1, q1);
        const double r2 = leafc_sum<F>(n2, t2, q2);
        const double g1 = __shfl(r1, 8 * (kS & 7), 64), g2 = __shfl(r2, 8 * (kS & 7), 64);
        v = (nS > 0 && (kS >> 3) == (k0 >> 3)) ? g1 : v;
        v = (nS > 0 && (kS >> 3) == (k0 >> 3) + 1) ? g2 : v;
    }
    return v;
}

template <class F>
__device__ double np_sum_wave8c(const F& f, int m) {
    double res = -0.0;
    for (int cs = 0; cs < m; cs += NP_CHUNK) {
        const int r = min(NP_CHUNK, m - cs);
        const double vA = np_slots8c(f, cs, r, 0, m - 1);
        const double vB = np_slots8c(f, cs, r, 64, m - 1);
        res += np_combine_wave_bf(vA, vB, r);
    }
    return res;
}

// old leaf layout (one lane per slot) with the branch-free node sizes and combine
template <class F>
__device__ double np_sum_wave_bf(const F& f, int m) {
    const int lane = threadIdx.x & 63;
    double res = -0.0;
    for (int cs = 0; cs < m; cs += NP_CHUNK) {
        const int r = min(NP_CHUNK, m - cs);
        int aA, aB;
        const int nA = nns_bf<7>(r, lane, &aA);
        const int nB = nns_bf<7>(r, lane + 64, &aB);
        const double vA = nA > 0 ? np_leaf(f, cs + aA, nA) : 0.0;
        const double vB = nB > 0 ? np_leaf(f, cs + aB, nB) : 0.0;
        res += np_combine_wave_bf(vA, vB, r);
    }
    return res;
}

__global__ __launch_bounds__(1024) void k_npsum(const double* __restrict__ g, const uint16_t* __restrict__ glist, int m,
                                                int mode, int nact, long long* __restrict__ ts, double* __restrict__ out) {
    __shared__ double tl[8192];
    __shared__ uint16_t L[8192];
    __shared__ double xb[8][64];
    __shared__ int flag[8];
    for (int i = threadIdx.x; i < m; i += 1024) { tl[i] = g[i]; L[i] = glist[i]; }
    if (threadIdx.x < 8) flag[threadIdx.x] = 0;
    __syncthreads();
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if (wv >= nact) return;
    long long t0 = __builtin_amdgcn_s_memtime(), t1 = 0;
    const long long r0 = wall_clock64();
    double h;
    if (mode == 0) h = np_sum_wave(RankTerm{tl}, m);
    else if (mode == 1) h = npw_stamped(RankTerm{tl}, m, &t1);
    else if (mode == 2) h = np_sum_wave(ListTerm{tl, L}, m);
    else if (mode == 3) h = npw_stamped(ListTerm{tl, L}, m, &t1);
    else if (mode == 4) h = np_sum_wave8(RankTerm{tl}, m);
    else if (mode == 5) h = np_sum_wave8(ListTerm{tl, L}, m);
    else if (mode == 6) h = np_sum_wave8b(RankTerm{tl}, m);
    else if (mode == 7) h = np_sum_wave8b(ListTerm{tl, L}, m);
    else if (mode == 10) h = np_sum_wave8c(RankTerm{tl}, m);
    else if (mode == 11) h = np_sum_wave8c(ListTerm{tl, L}, m);
    else if (mode == 12) {   // pairs, branch-free halves
        const int h2 = wv & 1, k = wv >> 1;
        const double v = np_slots8c(ListTerm{tl, L}, 0, m, 64 * h2, m - 1);
        if (h2) {
            xb[k][lane] = v;
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            if (lane == 0) atomicAdd(&flag[k], 1);
            h = 0.0;
        } else {
            for (int it = 0; it < (1 << 20) && __hip_atomic_load(&flag[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < 1; ++it) __builtin_amdgcn_s_sleep(1);
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
            h = -0.0;
            h += np_combine_wave_bf(v, xb[k][lane], m);
        }
    }
    else if (mode == 13 || mode == 16) {   // pairs, the decision's current layout (np_leaf per slot lane)
        const int h2 = wv & 1, k = wv >> 1;
        int a = 0;
        const int n = mode == 13 ? np_node_size(m, 7, lane + 64 * h2, &a) : nns_bf<7>(m, lane + 64 * h2, &a);
        const double v = n > 0 ? np_leaf(ListTerm{tl, L}, a, n) : 0.0;
        if (h2) {
            xb[k][lane] = v;
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            if (lane == 0) atomicAdd(&flag[k], 1);
            h = 0.0;
        } else {
            for (int it = 0; it < (1 << 20) && __hip_atomic_load(&flag[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < 1; ++it) __builtin_amdgcn_s_sleep(1);
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
            h = -0.0;
            h += mode == 13 ? np_combine_wave(v, xb[k][lane], m) : np_combine_wave_bf(v, xb[k][lane], m);
        }
    }
    else if (mode == 14) h = np_sum_wave_bf(RankTerm{tl}, m);
    else if (mode == 15) h = np_sum_wave_bf(ListTerm{tl, L}, m);
    else if (mode == 9) {   // one wave, stamped halves (rank order)
        __shared__ long long stt[64];
        if (wv == 0) {
            const double vA = ub_slots8_st(RankTerm{tl}, 0, m, 0, stt);
            const double vB = ub_slots8_st(RankTerm{tl}, 0, m, 64, stt + 30);
            h = -0.0;
            h += np_combine_wave(vA, vB, m);
            if (lane < 60) ts[lane] = stt[lane];
        } else h = 0.0;
        if (lane == 0 && wv == 0) out[0] = h;
        return;
    }
    else {   // mode 8: pairs of waves, one half each (the decision's paired round), list order
        const int h2 = wv & 1, k = wv >> 1;
        const double v = ub_slots8(ListTerm{tl, L}, 0, m, 64 * h2);
        if (h2) {
            xb[k][lane] = v;
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            if (lane == 0) atomicAdd(&flag[k], 1);
            h = 0.0;
        } else {
            for (int it = 0; it < (1 << 20) && __hip_atomic_load(&flag[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < 1; ++it) __builtin_amdgcn_s_sleep(1);
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
            h = -0.0;
            h += np_combine_wave(v, xb[k][lane], m);
        }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    long long t2 = __builtin_amdgcn_s_memtime();
    const long long r1 = wall_clock64();
    if (lane == 0 && wv == 0) { ts[46] = t2 - t0; ts[47] = r1 - r0; }
    if (lane == 0) {
        out[wv] = h;
        ts[3 * wv] = t0; ts[3 * wv + 1] = t1; ts[3 * wv + 2] = t2;
    }
}

// bit check: wave 0/1 = old/new over the identity order, waves 2/3 over the list
__global__ __launch_bounds__(512) void k_npcheck(const double* __restrict__ g, const uint16_t* __restrict__ glist, int m,
                                                 double* __restrict__ out) {
    __shared__ double tl[8192];
    __shared__ uint16_t L[8192];
    for (int i = threadIdx.x; i < m; i += blockDim.x) { tl[i] = g[i]; L[i] = glist[i]; }
    __syncthreads();
    const int wv = threadIdx.x >> 6;
    double h;
    if (wv == 0) h = np_sum_wave(RankTerm{tl}, m);
    else if (wv == 1) h = np_sum_wave8(RankTerm{tl}, m);
    else if (wv == 2) h = np_sum_wave(ListTerm{tl, L}, m);
    else if (wv == 3) h = np_sum_wave8(ListTerm{tl, L}, m);
    else if (wv == 4) h = np_sum_wave8b(RankTerm{tl}, m);
    else if (wv == 5) h = np_sum_wave8b(ListTerm{tl, L}, m);
    else if (wv == 6) h = np_sum_wave8c(RankTerm{tl}, m);
    else h = np_sum_wave8c(ListTerm{tl, L}, m);
    if ((threadIdx.x & 63) == 0) out[wv] = h;
}

int main() {
    // terms of a ct12-like 512^2 slice: counts of a smooth field + noise, p*log2(p)
    const int H = 512, W = 512;
    std::vector<uint32_t> hist(4096, 0);
    srand(1);
    for (int y = 0; y < H; ++y)
        for (int x = 0; x < W; ++x) {
            double base = (sin(x / 97.0 + 1) + cos(y / 61.0) + 2.0) / 4.0 * 4095.0 * 0.8;
            double u1 = (rand() + 1.0) / (RAND_MAX + 2.0), u2 = (rand() + 1.0) / (RAND_MAX + 2.0);
            double n = sqrt(-2 * log(u1)) * cos(2 * M_PI * u2) * 16.0;
            int v = (int)lrint(base + n);
            v = v < 0 ? 0 : v > 4095 ? 4095 : v;
            hist[v]++;
        }
    std::vector<double> terms;
    std::vector<int> vals;
    for (int v = 0; v < 4096; ++v)
        if (hist[v]) { double p = hist[v] / (double)(H * W); terms.push_back(p * log2(p)); vals.push_back(v); }
    const int m = (int)terms.size();
    std::vector<uint16_t> list;   // plane-2 joint order
    for (int q = 0; q < 2; ++q)
        for (int r = 0; r < m; ++r)
            if (((vals[r] >> 2) & 1) == q) list.push_back((uint16_t)r);
    printf("m = %d\n", m);
    double *dg, *dout;
    uint16_t* dl;
    long long* dts;
    CK(hipMalloc(&dg, 8192 * 8));
    CK(hipMalloc(&dl, 8192 * 2));
    CK(hipMalloc(&dout, 16 * 8));
    CK(hipMalloc(&dts, 64 * 8)); CK(hipMemset(dts, 0, 64 * 8));
    CK(hipMemcpy(dg, terms.data(), m * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(dl, list.data(), m * 2, hipMemcpyHostToDevice));
    {   // bit check over many m, random terms of mixed magnitude and a random permutation
        std::vector<double> rt(8192);
        std::vector<uint16_t> perm(8192);
        int bad = 0, nm = 0;
        for (int mm = 1; mm <= 8192; mm += (mm < 300 ? 1 : mm < 2000 ? 7 : 61)) {
            for (int i = 0; i < mm; ++i) rt[i] = -ldexp((rand() + 1.0) / RAND_MAX, -(rand() % 30));
            for (int i = 0; i < mm; ++i) perm[i] = (uint16_t)i;
            for (int i = mm - 1; i > 0; --i) std::swap(perm[i], perm[rand() % (i + 1)]);
            CK(hipMemcpy(dg, rt.data(), mm * 8, hipMemcpyHostToDevice));
            CK(hipMemcpy(dl, perm.data(), mm * 2, hipMemcpyHostToDevice));
            hipLaunchKernelGGL(k_npcheck, dim3(1), dim3(512), 0, 0, dg, dl, mm, dout);
            double o[8];
            CK(hipMemcpy(o, dout, 64, hipMemcpyDeviceToHost));
            ++nm;
            if (memcmp(&o[0], &o[1], 8) || memcmp(&o[2], &o[3], 8) || memcmp(&o[0], &o[4], 8) || memcmp(&o[2], &o[5], 8) || memcmp(&o[0], &o[6], 8) || memcmp(&o[2], &o[7], 8)) {
                if (bad < 10) printf("MISMATCH m=%d: %.17g %.17g %.17g %.17g | %.17g %.17g %.17g %.17g\n", mm, o[0], o[1], o[4], o[6], o[2], o[3], o[5], o[7]);
                ++bad;
            }
        }
        printf("bit check: %d of %d sizes differ\n", bad, nm);
        CK(hipMemcpy(dg, terms.data(), m * 8, hipMemcpyHostToDevice));
        CK(hipMemcpy(dl, list.data(), m * 2, hipMemcpyHostToDevice));
    }
    {
        hipLaunchKernelGGL(k_npsum, dim3(1), dim3(1024), 0, 0, dg, dl, m, 9, 1, dts, dout);
        CK(hipDeviceSynchronize());
        long long st[60];
        CK(hipMemcpy(st, dts, sizeof(st), hipMemcpyDeviceToHost));
        for (int hh = 0; hh < 2; ++hh) {
            printf("half %d stamps (clk from start):", hh);
            for (int i = 1; i < 30 && st[30 * hh + i] > 0 && st[30 * hh + i] - st[30 * hh] < 1000000; ++i) printf(" %lld", st[30 * hh + i] - st[30 * hh]);
            printf("\n");
        }
    }
    const char* names[] = {"rank np_sum_wave", "rank stamped", "list np_sum_wave", "list stamped", "rank wave8", "list wave8", "rank wave8b", "list wave8b", "list pairs8", "stamps", "rank wave8c", "list wave8c", "list pairs8c", "list pairs (cur)", "rank wave_bf", "list wave_bf", "list pairs bf"};
    for (int mode = 0; mode < 17; ++mode)
        for (int nact0 : {1, 4, 8, 12, 16}) {
            if (mode == 9) continue;
            const int nact = ((mode == 8 || mode == 12 || mode == 13 || mode == 16) && nact0 == 1) ? 2 : nact0;
            long long best = 1LL << 60, bl = 0;
            double h = 0;
            for (int rep = 0; rep < 20; ++rep) {
                hipLaunchKernelGGL(k_npsum, dim3(1), dim3(1024), 0, 0, dg, dl, m, mode, nact, dts, dout);
                CK(hipDeviceSynchronize());
                long long ts[48];
                CK(hipMemcpy(ts, dts, sizeof(ts), hipMemcpyDeviceToHost));
                CK(hipMemcpy(&h, dout, 8, hipMemcpyDeviceToHost));
                long long mx = 0, ml = 0;
                for (int w = 0; w < nact; ++w) {
                    mx = std::max(mx, ts[3 * w + 2] - ts[3 * w]);
                    if (ts[3 * w + 1]) ml = std::max(ml, ts[3 * w + 1] - ts[3 * w]);
                }
                if (mx < best) { best = mx; bl = ml; }
            }
            unsigned long long hb;
            memcpy(&hb, &h, 8);
            long long cal[2];
            CK(hipMemcpy(cal, dts + 46, 16, hipMemcpyDeviceToHost));
            printf("%-18s waves %2d: %6lld clk total (leaves %6lld)  sum %.17g (%016llx)  [memtime/realtime(100MHz) %.1f]\n", names[mode], nact, best, bl, h, hb,
                   cal[1] ? (double)cal[0] / cal[1] : 0.0);
        }
    return 0;
}
