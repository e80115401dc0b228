// codec_hip.hip -- CDNA4 (gfx950 / MI355X) kernels and the C ABI for the LSB bit-plane
// embed/extract path of wesleyfn/codec-tcc (reference: src/codec.py).  See DESIGN.md.
//
// Pipeline per batch of B slices ([B][H][W] uint8/uint16 in HBM):
//   k_scan_fast / k_scan_generic : ONE streaming read of the cover -> value histogram
//                                  (LDS-privatised), full-block LSB popcounts -> packed
//                                  argmax key, and the cover->stego copy.
//   k_block_exact                : numpy-exact np.var for partial / non-power-of-two blocks.
//   k_decide                     : per slice (one workgroup): bit-exact numpy entropy and
//                                  mutual information (8192-chunked pairwise sums emulated,
//                                  log2 from a numpy-built table), the s decision, the start
//                                  offset and the segment windows -> codec_slice_meta.
//   k_embed                      : one thread per embedded bit: window write + packed
//                                  location map via wave ballot.
//   k_restore + k_gather         : extraction: stream stego->cover with the map XOR-ed back,
//                                  and the payload bits (ballot-packed).
// Numerics: this file MUST be compiled with -ffp-contract=off (no FMA contraction) so the
// float64 sums reproduce numpy's bit for bit.
#include "codec_common.h"

#include <algorithm>

thread_local char g_err[512] = "";
ProfWin g_prof;
// the A/B knobs' tuning switch (codec_common.h): CODEC_TUNING=1 at load, or codec_set_tuning
static int tuning_from_env() {
    const char* v = getenv("CODEC_TUNING");
    return (v && v[0] == '1' && v[1] == 0) ? 1 : 0;
}
std::atomic<int> g_tuning{tuning_from_env()};

// ------------------------------------------------------------------ numpy float emulation
// numpy's add.reduce over a contiguous float64 array (np.sum) walks it in buffers of
// 8192 elements, each summed by pairwise_sum (<8: serial; <=128: 8 accumulators;
// else split at n/2 rounded down to a multiple of 8), and adds the buffer sums
// serially.  Verified against numpy 2.2 on lengths 0..200000 (tests/test_numpy_semantics).
#define NP_CHUNK 8192
#define NP_LEAF 128

template <class F>
__device__ __forceinline__ double np_leaf(const F& f, int a, int n) {
    if (n < 8) {
        double r = -0.0;
        for (int i = 0; i < n; ++i) r += f(a + i);
        return r;
    }
    double r0 = f(a + 0), r1 = f(a + 1), r2 = f(a + 2), r3 = f(a + 3);
    double r4 = f(a + 4), r5 = f(a + 5), r6 = f(a + 6), r7 = f(a + 7);
    int i = 8;
    const int lim = n - (n % 8);
    // two of numpy's 8-wide steps per iteration: all 16 (possibly indirect) loads are issued
    // before the adds, which keep numpy's per-accumulator order (r_k += x_k, then x_{8+k})
    for (; i + 8 < lim; i += 16) {
        double x[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) x[k] = f(a + i + k);
        r0 += x[0]; r1 += x[1]; r2 += x[2]; r3 += x[3]; r4 += x[4]; r5 += x[5]; r6 += x[6]; r7 += x[7];
        r0 += x[8]; r1 += x[9]; r2 += x[10]; r3 += x[11]; r4 += x[12]; r5 += x[13]; r6 += x[14]; r7 += x[15];
    }
    for (; i < lim; i += 8) {
        r0 += f(a + i + 0); r1 += f(a + i + 1); r2 += f(a + i + 2); r3 += f(a + i + 3);
        r4 += f(a + i + 4); r5 += f(a + i + 5); r6 += f(a + i + 6); r7 += f(a + i + 7);
    }
    double res = ((r0 + r1) + (r2 + r3)) + ((r4 + r5) + (r6 + r7));
    for (; i < n; ++i) res += f(a + i);
    return res;
}

// serial pairwise_sum over [a, a+n), n <= NP_CHUNK, explicit stack (depth <= 8)
template <class F>
__device__ double np_pairwise_serial(const F& f, int a, int n) {
    if (n <= NP_LEAF) return np_leaf(f, a, n);
    int sa[12], sn[12], st[12];
    double sv[12];
    int sp = 0, vp = 0;
    sa[0] = a; sn[0] = n; st[0] = 0; sp = 1;
    while (sp > 0) {
        int k = sp - 1;
        int na = sa[k], nn = sn[k];
        if (nn <= NP_LEAF) {
            sv[vp++] = np_leaf(f, na, nn);
            --sp;
            continue;
        }
        int n2 = (nn >> 1) & ~7;
        if (st[k] == 0) {
            st[k] = 1;
            sa[sp] = na; sn[sp] = n2; st[sp] = 0; ++sp;
        } else if (st[k] == 1) {
            st[k] = 2;
            sa[sp] = na + n2; sn[sp] = nn - n2; st[sp] = 0; ++sp;
        } else {
            double r = sv[--vp];
            double l = sv[--vp];
            sv[vp++] = l + r;
            --sp;
        }
    }
    return sv[0];
}

// np.sum semantics, serial (small n: partial-block variance)
template <class F>
__device__ double np_sum_serial(const F& f, int n) {
    double res = -0.0;
    for (int a = 0; a < n; a += NP_CHUNK) {
        int len = min(NP_CHUNK, n - a);
        res += np_pairwise_serial(f, a, len);
    }
    return res;
}

// size of node (d, j) of the chunk tree of a chunk holding r elements
__device__ __forceinline__ int np_node_size(int r, int d, int j, int* start) {
    int a = 0, n = r;
    for (int l = d - 1; l >= 0; --l) {
        const int bit = (j >> l) & 1;
        if (n > NP_LEAF) {
            const int n2 = (n >> 1) & ~7;
            if (bit) { a += n2; n -= n2; } else { n = n2; }
        } else if (bit) {
            n = 0;
        }
    }
    *start = a;
    return n;
}

// one chunk tree's internal nodes from its depth-7 slot sums (slot lane in vA, slot
// lane + 64 in vB), bottom-up in numpy's order with shuffles; the chunk sum, in every lane
__device__ __forceinline__ double np_combine_wave(double vA, double vB, int r) {
    const int lane = threadIdx.x & 63;
    // level 6: node j (lane j) = slots 2j, 2j+1 (lanes 2j, 2j+1 of vA for j < 32, of vB above)
    const int s0 = (2 * lane) & 63;
    const double lA = __shfl(vA, s0, 64), rA = __shfl(vA, s0 + 1, 64);
    const double lB = __shfl(vB, s0, 64), rB = __shfl(vB, s0 + 1, 64);
    int a6;
    const int n6 = np_node_size(r, 6, lane, &a6);
    const double L6 = lane < 32 ? lA : lB, R6 = lane < 32 ? rA : rB;
    double v = n6 > NP_LEAF ? L6 + R6 : L6;
    for (int d = 5; d >= 0; --d) {
        const double L = __shfl(v, (2 * lane) & 63, 64);
        const double R = __shfl(v, (2 * lane + 1) & 63, 64);
        int ad;
        const int nd = np_node_size(r, d, lane, &ad);
        v = nd > NP_LEAF ? L + R : L;
    }
    return __shfl(v, 0, 64);
}

// np.sum semantics over any m, computed by ONE wave (no block barrier), so that 16 waves
// can sum 16 different orders at once.  Per 8192-element buffer: the chunk's depth-7 tree
// has 128 bottom slots, two per lane (slots lane and lane+64); a slot's leaf (numpy's
// 8-accumulator loop) is summed serially by its lane, then internal nodes are re-added
// bottom-up with shuffles (node (d, j) lives in lane j).  Buffer sums are added serially.
// Result valid in every lane.
template <class F>
__device__ __forceinline__ double np_sum_wave(const F& f, int m) {
    const int lane = threadIdx.x & 63;
    double res = -0.0;
    for (int cs = 0; cs < m; cs += NP_CHUNK) {
        const int r = min(NP_CHUNK, m - cs);
        int aA, aB;
        const int nA = np_node_size(r, 7, lane, &aA);
        const int nB = np_node_size(r, 7, lane + 64, &aB);
        const double vA = nA > 0 ? np_leaf(f, cs + aA, nA) : 0.0;
        const double vB = nB > 0 ? np_leaf(f, cs + aB, nB) : 0.0;
        res += np_combine_wave(vA, vB, r);
    }
    return res;
}

// The chunk trees' internal nodes, bottom-up in numpy's order, from the depth-7 slot sums
// vals[chunk * 128 + slot] (1024 threads, m <= 8 chunks); the chunk sums are then added
// serially.  Returns the sum to all threads.
__device__ double np_tree_combine1024(int m, double* vals) {
    const int t = threadIdx.x;
    const int c = t >> 7, j = t & 127;
    const int r = min(NP_CHUNK, max(0, m - c * NP_CHUNK));
    for (int d = 6; d >= 0; --d) {
        const bool act = (r > 0) && (j < (1 << d));
        double nv = 0.0;
        if (act) {
            int a;
            const int n = np_node_size(r, d, j, &a);
            const double L = vals[c * 128 + 2 * j];
            const double R = vals[c * 128 + 2 * j + 1];
            nv = (n > NP_LEAF) ? (L + R) : L;
        }
        __syncthreads();
        if (act) vals[c * 128 + j] = nv;
        __syncthreads();
    }
    double res = -0.0;
    const int nchunks = (m + NP_CHUNK - 1) / NP_CHUNK;
    for (int k = 0; k < nchunks; ++k) res += vals[k * 128];
    __syncthreads();
    return res;
}

// np.sum semantics over m <= 65536 elements, computed by a 1024-thread block.
// Slot t = (chunk t/128, bottom slot t%128 of that chunk's depth-7 tree); leaves reached
// above depth 7 are carried down the left spine.  Leaves are summed wave-cooperatively:
// 8 lanes per leaf, lane q holding numpy's accumulator r[q] (so one load instruction
// touches 8 contiguous 64-byte segments), combined as ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7)).
// Internal nodes are then re-added bottom-up in numpy's order.  Returns the sum to all.
template <class F>
__device__ double np_sum_block1024(const F& f, int m, double* vals /*[1024]*/) {
    const int t = threadIdx.x;
    {
        const int lane = t & 63, wv = t >> 6, q = lane & 7;
        const int nchunks_ = (m + NP_CHUNK - 1) / NP_CHUNK;
        for (int rnd = 0; rnd < nchunks_; ++rnd) {          // one numpy buffer per round
            const int slot = rnd * 128 + wv * 8 + (lane >> 3);
            const int cs = rnd * NP_CHUNK;
            const int rr = min(NP_CHUNK, max(0, m - cs));
            int a = 0, n = 0;
            if (rr > 0) n = np_node_size(rr, 7, slot & 127, &a);
            a += cs;
            const int lim = n - (n % 8);
            // all of this lane's (<= 16) loads are issued before the dependent adds
            double tv[NP_LEAF / 8];
#pragma unroll
            for (int u = 0; u < NP_LEAF / 8; ++u) tv[u] = (8 * u < lim) ? f(a + 8 * u + q) : 0.0;
            double acc = 0.0;
            if (n >= 8) {
                acc = tv[0];
#pragma unroll
                for (int u = 1; u < NP_LEAF / 8; ++u)
                    if (8 * u < lim) acc += tv[u];
            }
            const double s2 = acc + __shfl_xor(acc, 1, 64);
            const double s4 = s2 + __shfl_xor(s2, 2, 64);
            const double s8 = s4 + __shfl_xor(s4, 4, 64);
            if (q == 0) {
                double res;
                if (n >= 8) {
                    res = s8;
                    for (int i = lim; i < n; ++i) res += f(a + i);
                } else {
                    res = -0.0;
                    for (int i = 0; i < n; ++i) res += f(a + i);
                }
                vals[slot] = n > 0 ? res : 0.0;
            }
        }
    }
    __syncthreads();
    return np_tree_combine1024(m, vals);
}

// np_sum_block1024's leaves alone (no barrier): slot sums into vals[chunk * 128 + slot]
template <class F>
__device__ __forceinline__ void np_leaves_block1024(const F& f, int m, double* vals, int wrot = 0) {
    const int t = threadIdx.x;
    const int lane = t & 63, wv = ((t >> 6) + wrot) & 15, q = lane & 7;   // wave w takes slots of (w + wrot) % 16
    const int nchunks_ = (m + NP_CHUNK - 1) / NP_CHUNK;
    for (int rnd = 0; rnd < nchunks_; ++rnd) {
        const int slot = rnd * 128 + wv * 8 + (lane >> 3);
        const int cs = rnd * NP_CHUNK;
        const int rr = min(NP_CHUNK, max(0, m - cs));
        int a = 0, n = 0;
        if (rr > 0) n = np_node_size(rr, 7, slot & 127, &a);
        a += cs;
        const int lim = n - (n % 8);
        double tv[NP_LEAF / 8];
#pragma unroll
        for (int u = 0; u < NP_LEAF / 8; ++u) tv[u] = (8 * u < lim) ? f(a + 8 * u + q) : 0.0;
        double acc = 0.0;
        if (n >= 8) {
            acc = tv[0];
#pragma unroll
            for (int u = 1; u < NP_LEAF / 8; ++u)
                if (8 * u < lim) acc += tv[u];
        }
        const double s2 = acc + __shfl_xor(acc, 1, 64);
        const double s4 = s2 + __shfl_xor(s2, 2, 64);
        const double s8 = s4 + __shfl_xor(s4, 4, 64);
        if (q == 0) {
            double res;
            if (n >= 8) {
                res = s8;
                for (int i = lim; i < n; ++i) res += f(a + i);
            } else {
                res = -0.0;
                for (int i = 0; i < n; ++i) res += f(a + i);
            }
            vals[slot] = n > 0 ? res : 0.0;
        }
    }
}

// the chunk trees over np_leaves_block1024's slot sums, re-added by ONE wave with shuffles
// (after a barrier that orders the slot stores); the sum, valid in that wave
__device__ __forceinline__ double np_combine_slots_wave(int m, const double* vals) {
    const int lane = threadIdx.x & 63;
    double res = -0.0;
    for (int cs = 0; cs < m; cs += NP_CHUNK) {
        const int c = cs / NP_CHUNK;
        res += np_combine_wave(vals[c * 128 + lane], vals[c * 128 + 64 + lane], min(NP_CHUNK, m - cs));
    }
    return res;
}

// np_sum_block1024's leaves, then wave 0 alone re-adds the chunk trees with shuffles (no
// block barriers: 14 fewer than np_tree_combine1024).  The sum is valid in wave 0 only.
template <class F>
__device__ double np_sum_block1024_w0(const F& f, int m, double* vals /*[1024]*/) {
    np_leaves_block1024(f, m, vals);
    __syncthreads();
    return threadIdx.x < 64 ? np_combine_slots_wave(m, vals) : -0.0;
}

// ---- wide slices (k_decide's walk path): the non-zero bins of a slice are kept as 64-bin
// group masks nz[g] (bin v = 64 g + e) and per-bin count codes cv[v] (the count if below
// kTermCodes, else kBigCode); a term is tc[code] (p * log2 p of that count, computed once
// per slice) or, for big counts, computed from the histogram.  The k-th element of a
// plane's joint order (codec.py:546-551: bit-clear bins ascending, then bit-set bins) is
// reached by walking the group masks, so neither a rank list nor a term array is stored.
constexpr int kTermCodes = 512;
constexpr uint16_t kBigCode = 0xFFFF;
// LDS slot of bin v's code: bits 1..6 XOR-swizzled with bits 7..12, so that the leaves'
// walkers (128 positions apart) read different banks
__device__ __forceinline__ int cv_slot(int v) { return v ^ (((v >> 7) & 63) << 1); }

struct JointWalk {
    const u64* nz;
    const uint16_t* cv;
    const double* tc;
    const uint32_t* hist;
    const double* lut;
    double N;
    int plane;      // -1: identity order (all bins in half 0)
    int ng;         // groups
    u64 lm;         // plane < 6: the lanes e of a group whose bit `plane` is set
    int h, g;
    u64 mk;         // bins of (h, g) still to visit
    __device__ void init(int pl) {
        plane = pl;
        lm = 0;
        if (pl >= 0 && pl < 6)
            for (int e = 0; e < 64; ++e) lm |= (u64)((e >> pl) & 1) << e;
    }
    __device__ __forceinline__ u64 mask(int hh, int gg) const {
        const u64 w = nz[gg];
        if (plane < 0) return hh ? 0ull : w;
        if (plane >= 6) return ((((gg << 6) >> plane) & 1) == hh) ? w : 0ull;
        return hh ? (w & lm) : (w & ~lm);
    }
    // the next bin of the order (-1 past the end: never for a valid leaf)
    __device__ __forceinline__ int nextv() {
        while (!mk) {
            if (++g == ng) {
                g = 0;
                if (++h > 1) return -1;
            }
            mk = mask(h, g);
        }
        const int e = __ffsll((long long)mk) - 1;
        mk &= mk - 1;
        return (g << 6) + e;
    }
    __device__ __forceinline__ double term(int v, uint16_t c) const {
        if (v < 0) return 0.0;
        if (c != kBigCode) return tc[c];
        const uint32_t n = hist[v];
        const double p = (double)n / N;
        return p * lut[n - 1];
    }
    // the next 8 terms: bins, then their codes, then the table terms (loads batched), big
    // counts patched afterwards (rare)
    __device__ __forceinline__ void next8(double* tv) {
        int v[8];
        uint32_t c[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) v[q] = nextv();
#pragma unroll
        for (int q = 0; q < 8; ++q) c[q] = cv[cv_slot(v[q] & 0xFFFF)];
#pragma unroll
        for (int q = 0; q < 8; ++q) tv[q] = tc[c[q] & (kTermCodes - 1)];
        bool big = false;
#pragma unroll
        for (int q = 0; q < 8; ++q) big |= c[q] == kBigCode || v[q] < 0;
        if (big) {
#pragma unroll
            for (int q = 0; q < 8; ++q)
                if (c[q] == kBigCode || v[q] < 0) tv[q] = term(v[q], (uint16_t)c[q]);
        }
    }
    __device__ __forceinline__ double next() {
        const int v = nextv();
        return term(v, v >= 0 ? cv[cv_slot(v)] : (uint16_t)0);
    }
};

// numpy's pairwise leaf over n elements of a walk (8 accumulators, then the tail)
__device__ __forceinline__ double np_leaf_walk(JointWalk& wk, int n) {
    double res = 0.0;
    if (n >= 8) {
        double acc[8];
        wk.next8(acc);
        const int lim = n - (n % 8);
        for (int i = 8; i < lim; i += 8) {
            double tv[8];
            wk.next8(tv);
#pragma unroll
            for (int q = 0; q < 8; ++q) acc[q] += tv[q];
        }
        res = ((acc[0] + acc[1]) + (acc[2] + acc[3])) + ((acc[4] + acc[5]) + (acc[6] + acc[7]));
        for (int i = lim; i < n; ++i) res += wk.next();
    } else if (n > 0) {
        res = -0.0;
        for (int i = 0; i < n; ++i) res += wk.next();
    }
    return res;
}

// np.sum of TWO orders at once (a plane's joint order, or the identity order) over the
// m0 / m1 non-zero bins of a wide slice (m = 0: order not summed), 1024 threads, order o
// on threads 512 o .. 512 o + 511.  The group counts of both halves of both orders are
// scanned (packed, one 64-bit scan per half) into start positions, kept in `vals` as u16
// deficits 64 g - prefix (a prefix never exceeds 64 g); each thread then seeks its two
// depth-7 slots (even j, then odd j: a full chunk's leaves are its even slots) by binary
// search, walks the leaves and the chunk trees are combined per order.  vals: 2048 doubles.
#ifdef DECIDE_TS
#define WTS(k) do { if (threadIdx.x == 0 && wts) wts[k] = wall_clock64(); } while (0)
#else
#define WTS(k) do { } while (0)
#endif
__device__ __forceinline__ void np_sum_walk2(JointWalk wk, int pl0, int m0, int pl1, int m1, double* vals,
                                             u64* sh64, double* out, long long* wts) {
    const int t = threadIdx.x;
    const int ng = wk.ng;
    u64 xz = 0, xo = 0;
    if (t < ng) {
        wk.init(pl0);
        if (m0) { xz |= (u64)__popcll(wk.mask(0, t)); xo |= (u64)__popcll(wk.mask(1, t)); }
        wk.init(pl1);
        if (m1) { xz |= (u64)__popcll(wk.mask(0, t)) << 32; xo |= (u64)__popcll(wk.mask(1, t)) << 32; }
    }
    u64 tz, tone;
    const u64 pz = block_excl_scan64<1024>(xz, sh64, &tz);
    const u64 po = block_excl_scan64<1024>(xo, sh64, &tone);
    uint16_t* D = reinterpret_cast<uint16_t*>(vals);          // [order][half][1024]
    if (t < ng) {
        const uint32_t base = 64u * (uint32_t)t;
        D[t] = (uint16_t)(base - (uint32_t)pz);
        D[1024 + t] = (uint16_t)(base - (uint32_t)po);
        D[2048 + t] = (uint16_t)(base - (uint32_t)(pz >> 32));
        D[3072 + t] = (uint16_t)(base - (uint32_t)(po >> 32));
    }
    __syncthreads();
    WTS(0);
    const int o = t >> 9, tt = t & 511;
    wk.init(o ? pl1 : pl0);
    const int m = o ? m1 : m0;
    const uint32_t z = o ? (uint32_t)(tz >> 32) : (uint32_t)tz;
    int cs[2], js[2], ns[2], hs[2] = {0, 0}, gs[2] = {0, 0};
    u64 mks[2] = {0ull, 0ull};
#pragma unroll
    for (int sl = 0; sl < 2; ++sl) {
        const int c = tt >> 6, j = 2 * (tt & 63) + sl;
        const int r = min(NP_CHUNK, max(0, m - c * NP_CHUNK));
        int a = 0, n = 0;
        if (r > 0) n = np_node_size(r, 7, j, &a);
        a += c * NP_CHUNK;
        cs[sl] = c; js[sl] = j; ns[sl] = n;
        if (n > 0) {                              // seek position a
            const int hh = (uint32_t)a >= z ? 1 : 0;
            const uint16_t* Dp = D + o * 2048 + hh * 1024;
            const uint32_t base = hh ? z : 0u;
            int lo = 0, hi = ng - 1;              // last group starting at or before a
            while (lo < hi) {
                const int mid = (lo + hi + 1) >> 1;
                if (base + 64u * (uint32_t)mid - Dp[mid] <= (uint32_t)a) lo = mid; else hi = mid - 1;
            }
            u64 mk = wk.mask(hh, lo);
            for (uint32_t k = (uint32_t)a - (base + 64u * (uint32_t)lo - Dp[lo]); k > 0; --k) mk &= mk - 1;
            hs[sl] = hh; gs[sl] = lo; mks[sl] = mk;
        }
    }
    __syncthreads();                              // deficits read; vals free again
    WTS(1);
    double* vo = vals + o * 1024;
#pragma unroll
    for (int sl = 0; sl < 2; ++sl) {
        double res = 0.0;
        if (ns[sl] > 0) {
            wk.h = hs[sl]; wk.g = gs[sl]; wk.mk = mks[sl];
            res = np_leaf_walk(wk, ns[sl]);
        }
        vo[cs[sl] * 128 + js[sl]] = ns[sl] > 0 ? res : 0.0;
    }
    __syncthreads();
    WTS(2);
    {   // both orders' chunk trees (np_tree_combine1024's order), 64 threads per chunk
        const int c = (t >> 6) & 7, j = t & 63;
        const int r = min(NP_CHUNK, max(0, m - c * NP_CHUNK));
        for (int d = 6; d >= 0; --d) {
            const bool act = (r > 0) && (j < (1 << d));
            double nv = 0.0;
            if (act) {
                int a;
                const int n = np_node_size(r, d, j, &a);
                const double L = vo[c * 128 + 2 * j];
                const double R = vo[c * 128 + 2 * j + 1];
                nv = (n > NP_LEAF) ? (L + R) : L;
            }
            __syncthreads();
            if (act) vo[c * 128 + j] = nv;
            __syncthreads();
        }
    }
#pragma unroll
    for (int q = 0; q < 2; ++q) {
        const int mq = q ? m1 : m0;
        double res = -0.0;
        for (int k = 0; k < (mq + NP_CHUNK - 1) / NP_CHUNK; ++k) res += vals[q * 1024 + k * 128];
        out[q] = res;
    }
    __syncthreads();
    WTS(3);
}

// ------------------------------------------------------------------ histogram helpers
// uint16 covers: 65536 bins kept as 16-bit halves of 32768 LDS words (128 KiB).  An add
// whose returned old value shows a half wrapping is rare; its exact effect on the two
// fields is recorded in the global histogram, so the per-workgroup pixel count is
// unbounded (final bin = LDS field + recorded adjustments, modulo 2^32).
__device__ __forceinline__ void hist16_add(uint32_t* lds, uint32_t* ghist, uint32_t v, uint32_t cnt) {
    const uint32_t w = v >> 1;
    if (v & 1u) {
        const uint32_t old = atomicAdd(&lds[w], cnt << 16);
        if ((old >> 16) + cnt > 0xFFFFu) atomicAdd(&ghist[v], 0x10000u);
    } else {
        const uint32_t old = atomicAdd(&lds[w], cnt);
        if ((old & 0xFFFFu) + cnt > 0xFFFFu) {
            atomicAdd(&ghist[v], 0x10000u);
            uint32_t adj = 0xFFFFFFFFu;                     // -1: spurious carry into v+1
            if ((old >> 16) == 0xFFFFu) adj += 0x10000u;    // ...which wrapped that field
            atomicAdd(&ghist[v + 1], adj);
        }
    }
}

template <typename T> struct HistCfg;
template <> struct HistCfg<uint16_t> {
    static constexpr int kBins = 65536;
    static constexpr int kLdsWords = 32768;
};
template <> struct HistCfg<uint8_t> {
    static constexpr int kBins = 256;
    static constexpr int kLdsWords = 16 * 256;   // one private copy per wave (16 waves)
};

template <typename T>
__device__ __forceinline__ void hist_add(uint32_t* lds, uint32_t* ghist, uint32_t v, uint32_t cnt);
template <>
__device__ __forceinline__ void hist_add<uint16_t>(uint32_t* lds, uint32_t* ghist, uint32_t v, uint32_t cnt) {
    hist16_add(lds, ghist, v, cnt);
}
template <>
__device__ __forceinline__ void hist_add<uint8_t>(uint32_t* lds, uint32_t*, uint32_t v, uint32_t cnt) {
    atomicAdd(&lds[((threadIdx.x >> 6) << 8) + v], cnt);
}

// `vmax` bounds every value the workgroup counted (its OR of pixels: a value's bits are a
// subset of it), so LDS words past vmax / 2 are zero and are not read (ct12: 2 048 of 32 768)
template <typename T>
__device__ void hist_flush(uint32_t* lds, uint32_t* ghist, uint32_t vmax = 0xFFFFu);
template <>
__device__ void hist_flush<uint16_t>(uint32_t* lds, uint32_t* ghist, uint32_t vmax) {
    u64* g64 = reinterpret_cast<u64*>(ghist);
    const int nw = (int)min((vmax & 0xFFFFu) >> 1, 32767u) + 1;
    for (int w = threadIdx.x; w < nw; w += blockDim.x) {
        const uint32_t x = lds[w];
        if (x) atomicAdd(&g64[w], (u64)(x & 0xFFFFu) | ((u64)(x >> 16) << 32));
    }
}
template <>
__device__ void hist_flush<uint8_t>(uint32_t* lds, uint32_t* ghist, uint32_t) {
    for (int v = threadIdx.x; v < 256; v += blockDim.x) {
        uint32_t acc = 0;
        for (int c = 0; c < 16; ++c) acc += lds[(c << 8) + v];
        if (acc) atomicAdd(&ghist[v], acc);
    }
}

// exact bookkeeping after an LDS add of `cnt` to value v's 16-bit field returned `old`
// (only called when a field wrapped; see hist16_add)
__device__ __noinline__ void hist16_fix(uint32_t* ghist, uint32_t v, uint32_t cnt, uint32_t old) {
    if (v & 1u) {
        if ((old >> 16) + cnt > 0xFFFFu) atomicAdd(&ghist[v], 0x10000u);
    } else if ((old & 0xFFFFu) + cnt > 0xFFFFu) {
        atomicAdd(&ghist[v], 0x10000u);
        uint32_t adj = 0xFFFFFFFFu;
        if ((old >> 16) == 0xFFFFu) adj += 0x10000u;
        atomicAdd(&ghist[v + 1], adj);
    }
}

// 8 consecutive pixels of a vector (16 B of uint16 / 8 B of uint8): equal neighbours are
// merged into one add (constant regions), the 8 LDS atomics are issued back to back and
// their returned values are checked for 16-bit wraps only afterwards, so the adds
// pipeline instead of each waiting for its return.
// NORET: the workgroup counts fewer than 65 536 pixels, so no 16-bit field can wrap and the
// adds need no return (ds_add_u32 instead of ds_add_rtn_u32)
template <typename T, typename V, bool NORET = false>
__device__ __forceinline__ void hist_add8(uint32_t* lds, uint32_t* ghist, const V& vec, uint32_t* wrapf = nullptr) {
    uint32_t px[8];
    if constexpr (sizeof(T) == 2) {
        px[0] = vec.x & 0xFFFFu; px[1] = vec.x >> 16; px[2] = vec.y & 0xFFFFu; px[3] = vec.y >> 16;
        px[4] = vec.z & 0xFFFFu; px[5] = vec.z >> 16; px[6] = vec.w & 0xFFFFu; px[7] = vec.w >> 16;
    } else {
#pragma unroll
        for (int k = 0; k < 4; ++k) { px[k] = (vec.x >> (8 * k)) & 0xFFu; px[4 + k] = (vec.y >> (8 * k)) & 0xFFu; }
    }
    uint32_t cnt[8];
    uint32_t run = 1;
#pragma unroll
    for (int k = 0; k < 7; ++k) {
        const bool eq = px[k + 1] == px[k];
        cnt[k] = eq ? 0u : run;
        run = eq ? run + 1u : 1u;
    }
    cnt[7] = run;
    if constexpr (sizeof(T) == 2 && NORET) {
#pragma unroll
        for (int k = 0; k < 8; ++k)
            if (cnt[k]) atomicAdd(&lds[px[k] >> 1], (px[k] & 1u) ? (cnt[k] << 16) : cnt[k]);
    } else if constexpr (sizeof(T) == 2) {
        uint32_t old[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            old[k] = 0;
            if (cnt[k]) old[k] = atomicAdd(&lds[px[k] >> 1], (px[k] & 1u) ? (cnt[k] << 16) : cnt[k]);
        }
        bool wrap = false;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const uint32_t field = (px[k] & 1u) ? (old[k] >> 16) : (old[k] & 0xFFFFu);
            wrap |= (field + cnt[k]) > 0xFFFFu;
        }
        if (wrap) {
            if (wrapf) *wrapf = 1u;   // fused scan: the slice's counts are no longer all in LDS
#pragma unroll
            for (int k = 0; k < 8; ++k)
                if (cnt[k]) hist16_fix(ghist, px[k], cnt[k], old[k]);
        }
    } else {
        const uint32_t base = (threadIdx.x >> 6) << 8;
#pragma unroll
        for (int k = 0; k < 8; ++k)
            if (cnt[k]) atomicAdd(&lds[base + px[k]], cnt[k]);
    }
}


// ------------------------------------------------------------------ K1: scan + copy (fast)
// Requirements (checked on the host): W % 8 == 0, SB in {8,16,32,64}, stego dtype ==
// cover dtype with every bit kept, 16-B (u16) / 8-B (u8) aligned buffers.
// Work item = (band of SB rows, 8-pixel column chunk); a wave covers 64 consecutive
// chunks of one band, so every load instruction reads 1 KiB (u16) contiguously; the
// SB/8 lanes of one block column combine their LSB counts with shuffles.
template <typename T, int SB, bool NT, bool HIST, bool NORET = false>
__device__ __forceinline__ void scan_fast_body(const T* __restrict__ cover, T* __restrict__ stego,
                                               int H, int W, int bands_per_wg,
                                               uint32_t* __restrict__ ghist_all,
                                               u64* __restrict__ gkey, uint32_t* __restrict__ gor, int csplit) {
    typedef typename Vec8<T>::type V;
    constexpr int G = SB / 8;
    constexpr uint32_t NPB = (uint32_t)SB * SB;
    __shared__ uint32_t lds[HistCfg<T>::kLdsWords];
    __shared__ u64 wkey;
    __shared__ uint32_t wor;
    const int b = blockIdx.y;
    const size_t npx = (size_t)H * W;
    const T* src = cover + (size_t)b * npx;
    T* dst = stego ? stego + (size_t)b * npx : nullptr;
    uint32_t* ghist = ghist_all + (size_t)b * HistCfg<T>::kBins;

    for (int i = threadIdx.x; i < HistCfg<T>::kLdsWords; i += 1024) lds[i] = 0;
    if (threadIdx.x == 0) { wkey = 0; wor = 0; }
    __syncthreads();

    const int nbands = (H + SB - 1) / SB;
    // csplit > 1 (small batches: fewer bands than CUs): workgroup x takes column segment
    // x % csplit of the bands of group x / csplit; segments are whole block columns (G chunks)
    const int band0 = (int)(blockIdx.x / (unsigned)csplit) * bands_per_wg;
    const int band1 = min(nbands, band0 + bands_per_wg);
    const int CR = W / 8;
    const int CRp = (CR + G - 1) / G * G;
    const int seg = (int)(blockIdx.x % (unsigned)csplit);
    const int CRs = (CRp / G + csplit - 1) / csplit * G;   // chunks per segment, a multiple of G
    const int c0 = min(CRp, seg * CRs), CRw = min(CRp, c0 + CRs) - c0;
    const int nbx = (W + SB - 1) / SB;
    const int fullbx = W / SB, fullby = H / SB;
    const int nitems = max(0, band1 - band0) * CRw;
    const int lane = threadIdx.x & 63;
    u64 best = 0;
    uint32_t vor = 0;   // OR of every pixel: bounds the histogram range the decision scans

    for (int base = (threadIdx.x & ~63); base < nitems; base += 1024) {
        const int it = base + lane;
        const bool valid = it < nitems;
        const int band = band0 + (valid ? it / CRw : 0);
        const int c = valid ? c0 + it % CRw : CRp;
        const bool inrow = valid && c < CR;
        uint32_t ones = 0;
        if (inrow) {
            const int rows = min(SB, H - band * SB);
            const size_t rowpix = (size_t)band * SB * W + (size_t)c * 8;
            const V* s = reinterpret_cast<const V*>(src + rowpix);
            V* d = dst ? reinterpret_cast<V*>(dst + rowpix) : nullptr;
            const int stride = W / 8;   // vectors per row
            int r = 0;
            // RB rows in flight per lane (the whole 16-row block column): a small batch has
            // few busy waves (one band = W/8 lanes), so each lane's serial load rounds were its
            // time (1 x 2048^2: 4 rounds of 4 rows, 18 us; the workgroup holds the CU's LDS
            // alone, so the 64 data VGPRs cost no occupancy)
            constexpr int RB = SB < 16 ? SB : 16;
            for (; r + RB <= rows; r += RB) {
                V v[RB];
#pragma unroll
                for (int k = 0; k < RB; ++k) v[k] = ldv<NT>(s + (size_t)(r + k) * stride);
                if (d) {
#pragma unroll
                    for (int k = 0; k < RB; ++k) stv<NT>(d + (size_t)(r + k) * stride, v[k]);
                }
#pragma unroll
                for (int k = 0; k < RB; ++k) {
                    ones += lsb_count(v[k]);
                    vor |= vor_of(v[k]);
                    if constexpr (HIST) hist_add8<T, typename Vec8<T>::type, NORET>(lds, ghist, v[k]);
                }
            }
            for (; r < rows; ++r) {
                V v0 = ldv<NT>(s + (size_t)r * stride);
                if (d) stv<NT>(d + (size_t)r * stride, v0);
                ones += lsb_count(v0);
                vor |= vor_of(v0);
                if constexpr (HIST) hist_add8<T, typename Vec8<T>::type, NORET>(lds, ghist, v0);
            }
        }
#pragma unroll
        for (int o = 1; o < G; o <<= 1) ones += __shfl_xor(ones, o, 64);
        const bool full = inrow && band < fullby && (c / G) < fullbx && (lane % G) == 0;
        if (full) {
            const uint32_t score = ones * (NPB - ones);
            const uint32_t idx = (uint32_t)band * nbx + (uint32_t)(c / G);
            const u64 key = ((u64)score << 32) | (u64)(0xFFFFFFFFu - idx);
            best = best > key ? best : key;
        }
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
        const u64 other = __shfl_xor(best, o, 64);
        best = best > other ? best : other;
    }
    if (lane == 0 && best) atomicMax(&wkey, best);
    if constexpr (sizeof(T) == 2) vor = (vor | (vor >> 16)) & 0xFFFFu;
    else vor = (vor | (vor >> 8) | (vor >> 16) | (vor >> 24)) & 0xFFu;
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) vor |= __shfl_xor(vor, o, 64);
    // one global OR per workgroup (a same-address global atomic per wave serialised)
    if (lane == 0 && vor) atomicOr(&wor, vor);
    __syncthreads();
    hist_flush<T>(lds, ghist, wor);
    if (threadIdx.x == 0) {
        if (wkey) atomicMax(&gkey[b], wkey);
        if (wor) atomicOr(&gor[b], wor);
    }
}

template <typename T, int SB, bool NT, bool HIST = true, bool NORET = false>
__global__ __launch_bounds__(1024) void k_scan_fast(const T* __restrict__ cover, T* __restrict__ stego,
                                                    int H, int W, int bands_per_wg,
                                                    uint32_t* __restrict__ ghist_all,
                                                    u64* __restrict__ gkey, uint32_t* __restrict__ gor, int csplit) {
    scan_fast_body<T, SB, NT, HIST, NORET>(cover, stego, H, W, bands_per_wg, ghist_all, gkey, gor, csplit);
}

// read-only variant (plan only, or in place where the stego copy is the cover itself); a
// separate symbol so profiles never average it with the copying pass
template <typename T, int SB>
__global__ __launch_bounds__(1024) void k_scan_read(const T* __restrict__ cover, int H, int W, int bands_per_wg,
                                                    uint32_t* __restrict__ ghist_all,
                                                    u64* __restrict__ gkey, uint32_t* __restrict__ gor, int csplit) {
    scan_fast_body<T, SB, true, true>(cover, nullptr, H, W, bands_per_wg, ghist_all, gkey, gor, csplit);
}

// ------------------------------------------------------------------ K1 (row-major): scan + copy
// Same outputs as k_scan_fast, different sweep: a workgroup owns whole SB-row bands of one
// slice (one contiguous region) and streams it in flat order, 4096 16-B vectors (64 KiB of
// uint16) per iteration, vector u*1024+t of the iteration to thread t.  Measured on the
// MI355X (tools/ubench_stagger.hip): this flat per-region order copies at 6.2 TB/s where
// the column-band order of k_scan_fast tops out at 5.8 TB/s.  Block LSB counts no longer
// stay in one thread's registers, so they go to packed 16-bit LDS counters (one per full
// block of the region, pre-combined across the SB/8 lanes of a block row when W % SB == 0)
// and are turned into argmax keys once the region is done.
#define SCAN_ROWS_CNT_WORDS 7168   // 28 KiB of LDS = 14 336 block counters per workgroup
// the region's first loads go out before the LDS zeroing (build-time A/B knob; 256 x 2048^2
// k_scan_rows 0.7944 -> 0.7874 ms, profiles/r03/lockstep_ab.log).  A barrier per iteration
// (waves in lockstep, as the restore wants) made the sweep slower: 0.79 -> 0.89 ms.
#ifndef SCAN_EARLY_LOAD
#define SCAN_EARLY_LOAD 1
#endif
// DIAG (timing diagnostics only, decisions are wrong): 1 = no histogram adds, 4 = copy with
// the sweep's bookkeeping only, 5 = bare region copy (tools/ubench_stagger.hip's loop).
// Measured in one process at 256 x 2048^2 (profiles/r01/ubench/scan_rows_diag.txt): full
// kernel 0.800 ms, no histogram 0.762, bare region copy 0.757 -- the histogram, block
// counts and key costs 5 % over the copy in this order.  U (vectors per thread per
// iteration) = 4; U = 2 or 8 (pipelined or not) measured 0.83-0.84 ms.
// k_scan_rows' LDS (a struct so that k_scan_decide can overlay k_decide's on it); `wor` and
// `wrap` serve the fused kernel only: the workgroup's OR of pixels and "a 16-bit field wrapped"
template <typename T>
struct ScanRowsSmem {
    uint32_t lds[HistCfg<T>::kLdsWords];
    uint32_t cnt[SCAN_ROWS_CNT_WORDS];
    u64 wkey;
    uint32_t wor, wrap;
};

// FUSED (k_scan_decide: the workgroup is its slice's only one): no histogram flush, and the
// OR word and block key stay in LDS for the decision that follows in the same workgroup
template <typename T, int SB, bool NT, bool STORE, int DIAG = 0, bool PIPE = true, int U = 4, bool FUSED = false>
__device__ __forceinline__ void scan_rows_body(ScanRowsSmem<T>& SS, const T* __restrict__ cover, T* __restrict__ stego,
                                               int H, int W, int bands_per_wg,
                                               uint32_t* __restrict__ ghist_all,
                                               u64* __restrict__ gkey, uint32_t* __restrict__ gor) {
    typedef typename Vec8<T>::type V;
    constexpr int G = SB / 8;                 // lanes (vectors) per block row segment
    constexpr int LG = G == 1 ? 0 : G == 2 ? 1 : G == 4 ? 2 : 3;
    constexpr int LSB_ = SB == 8 ? 3 : SB == 16 ? 4 : SB == 32 ? 5 : 6;
    constexpr uint32_t NPB = (uint32_t)SB * SB;
    constexpr int NT_ = 1024;
    uint32_t* lds = SS.lds;
    uint32_t* cnt = SS.cnt;
    u64& wkey = SS.wkey;
    const int b = blockIdx.y;
    const size_t npx = (size_t)H * W;
    const T* src = cover + (size_t)b * npx;
    T* dst = STORE ? stego + (size_t)b * npx : nullptr;
    uint32_t* ghist = ghist_all + (size_t)b * HistCfg<T>::kBins;

    const int CR = W / 8;                                   // vectors per row
    const int band0 = blockIdx.x * bands_per_wg;
    const int row0 = band0 * SB;
    const int row1 = min(H, row0 + bands_per_wg * SB);
    const int fullbx = W / SB, fullby = H / SB, nbx = (W + SB - 1) / SB;
    // full blocks of this region: bands [band0, min(band1, fullby)) x [0, fullbx)
    const int fb1 = min(fullby, band0 + bands_per_wg);
    const int nfull = max(0, fb1 - band0) * fullbx;        // host guarantees nfull <= 2*CNT_WORDS
    const long long nvec = (long long)max(0, row1 - row0) * CR;
    const V* s = reinterpret_cast<const V*>(src + (size_t)row0 * W);
    V* d = STORE ? reinterpret_cast<V*>(dst + (size_t)row0 * W) : nullptr;
    const long long step = (long long)NT_ * U;
    const long long nwhole = nvec / step * step;   // iterations with every vector in range
    V v[U], vn[U];
#if SCAN_EARLY_LOAD
    // the region's first loads go out before the LDS zeroing (they touch no LDS), and the
    // barrier after it is LDS-only (__syncthreads' fence would wait for them)
    if (PIPE && DIAG != 5 && nwhole > 0) {
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = ldv<NT>(s + (long long)u * NT_ + threadIdx.x);
    }
#endif
    for (int i = threadIdx.x; i < HistCfg<T>::kLdsWords; i += NT_) lds[i] = 0;
    for (int i = threadIdx.x; i < (nfull + 1) / 2; i += NT_) cnt[i] = 0;
    if (threadIdx.x == 0) { wkey = 0; SS.wor = 0u; SS.wrap = 0u; }
#if SCAN_EARLY_LOAD
    lds_barrier();
#else
    __syncthreads();
#endif
    const int lane = threadIdx.x & 63;
    const bool grouped = (CR % G) == 0;                     // G-lane groups share a block row
    // (row, column-vector) of this thread's first vector, advanced incrementally
    const int dq = NT_ / CR, dr = NT_ % CR;                 // one u step = 1024 vectors
    int r = threadIdx.x / CR, c = threadIdx.x % CR;
    uint32_t vor = 0;
    if constexpr (DIAG == 5) {   // the bare region copy of tools/ubench_stagger.hip
        unsigned acc = 0;
        for (long long base = threadIdx.x; base + 3 * NT_ < nvec; base += (long long)NT_ * U) {
            V w[U];
#pragma unroll
            for (int u = 0; u < U; ++u) w[u] = ldv<NT>(s + base + u * NT_);
#pragma unroll
            for (int u = 0; u < U; ++u) { stv<NT>(d + base + u * NT_, w[u]); acc += w[u].x & 1u; }
        }
        if (acc == 0xFFFFFFFFu) gor[b] = acc;
        return;
    }
    // one iteration's stores, block counts and histogram adds on 4 loaded vectors
    auto process = [&](long long base, const V* v, bool whole) {
        int rr[U], cc[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            rr[u] = r; cc[u] = c;
            c += dr; r += dq;
            if (c >= CR) { c -= CR; ++r; }
        }
        if constexpr (STORE) {
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const long long i = base + (long long)u * NT_ + threadIdx.x;
                if (whole || i < nvec) stv<NT>(d + i, v[u]);
            }
        }
        // block LSB counts: a lane's U vectors often sit in one block (W = 2048: rows q,
        // q+4, q+8, q+12 of one band, same column pair), so a count is carried while the next
        // vector's block is the same and one LDS add is issued per block change
        int kk[U];
        bool fl[U];
        uint32_t on[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const long long i = base + (long long)u * NT_ + threadIdx.x;
            const bool ok = whole || i < nvec;
            uint32_t ones = ok ? lsb_count(v[u]) : 0u;
            if (ok) vor |= vor_of(v[u]);
            const int by = rr[u] >> LSB_, bx = cc[u] >> LG;
            fl[u] = ok && (band0 + by) < fullby && bx < fullbx;
            kk[u] = by * fullbx + bx;
            if (grouped) {
#pragma unroll
                for (int o = 1; o < G; o <<= 1) ones += __shfl_xor(ones, o, 64);
                fl[u] = fl[u] && (lane & (G - 1)) == 0;
            }
            on[u] = ones;
        }
        if (DIAG != 4) {
            uint32_t carry = 0;
#pragma unroll
            for (int u = 0; u < U; ++u) {
                if (!fl[u]) continue;
                carry += on[u];
                const bool same_next = (u + 1 < U) && fl[u + 1] && kk[u + 1] == kk[u];
                if (!same_next && carry) {
                    atomicAdd(&cnt[kk[u] >> 1], carry << ((kk[u] & 1) * 16));
                    carry = 0;
                } else if (!same_next) {
                    carry = 0;
                }
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const long long i = base + (long long)u * NT_ + threadIdx.x;
            const bool ok = whole || i < nvec;
            if (DIAG == 4) { vor ^= v[u].x; continue; }
            if (DIAG == 0)
                if (ok) hist_add8<T>(lds, ghist, v[u], FUSED ? &SS.wrap : nullptr);
        }
    };
    if constexpr (PIPE) {
        // software pipelined: the next iteration's loads are issued before this iteration's
        // stores and histogram adds
#if !SCAN_EARLY_LOAD
        if (nwhole > 0) {
#pragma unroll
            for (int u = 0; u < U; ++u) v[u] = ldv<NT>(s + (long long)u * NT_ + threadIdx.x);
        }
#endif
        for (long long base = 0; base < nwhole; base += step) {
            if (base + step < nwhole) {
#pragma unroll
                for (int u = 0; u < U; ++u) vn[u] = ldv<NT>(s + base + step + (long long)u * NT_ + threadIdx.x);
            }
            process(base, v, true);
#pragma unroll
            for (int u = 0; u < U; ++u) v[u] = vn[u];
        }
    } else {
        for (long long base = 0; base < nwhole; base += step) {
            V v[U];
#pragma unroll
            for (int u = 0; u < U; ++u) v[u] = ldv<NT>(s + base + (long long)u * NT_ + threadIdx.x);
            process(base, v, true);
        }
    }
    if (nwhole < nvec) {   // ragged last iteration
        V v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const long long i = nwhole + (long long)u * NT_ + threadIdx.x;
            if (i < nvec) v[u] = ldv<NT>(s + i);
        }
        process(nwhole, v, false);
    }
    if constexpr (sizeof(T) == 2) vor = (vor | (vor >> 16)) & 0xFFFFu;
    else vor = (vor | (vor >> 8) | (vor >> 16) | (vor >> 24)) & 0xFFu;
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) vor |= __shfl_xor(vor, o, 64);
    if (lane == 0 && vor) atomicOr(&SS.wor, vor);   // the workgroup's OR (bounds the flush)
    // fused (k_scan_decide): LDS-only -- the copy's last stores drain during the decision
    // instead (the fused embed, which rewrites window pixels, waits for them with a full barrier)
    if constexpr (FUSED) lds_barrier(); else __syncthreads();
    // block keys: score c(n-c) (exact variance numerator of a full pow2 block), first
    // maximal block in raster order wins (~index in the low word)
    u64 best = 0;
    for (int k = threadIdx.x; k < nfull; k += NT_) {
        const uint32_t ones = (cnt[k >> 1] >> ((k & 1) * 16)) & 0xFFFFu;
        const uint32_t score = ones * (NPB - ones);
        const int by = k / fullbx, bx = k - by * fullbx;
        const uint32_t idx = (uint32_t)(band0 + by) * nbx + (uint32_t)bx;
        const u64 key = ((u64)score << 32) | (u64)(0xFFFFFFFFu - idx);
        best = best > key ? best : key;
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
        const u64 other = __shfl_xor(best, o, 64);
        best = best > other ? best : other;
    }
    if (lane == 0 && best) atomicMax(&wkey, best);
    if (DIAG == 0 && !FUSED) hist_flush<T>(lds, ghist, SS.wor);
    if constexpr (FUSED) lds_barrier(); else __syncthreads();
    if (!FUSED && threadIdx.x == 0 && wkey) atomicMax(&gkey[b], wkey);
    if (!FUSED && threadIdx.x == 0 && SS.wor) atomicOr(&gor[b], SS.wor);
}

template <typename T, int SB, bool NT, bool STORE, int DIAG = 0, bool PIPE = true, int U = 4>
__global__ __launch_bounds__(1024) void k_scan_rows(const T* __restrict__ cover, T* __restrict__ stego,
                                                    int H, int W, int bands_per_wg,
                                                    uint32_t* __restrict__ ghist_all,
                                                    u64* __restrict__ gkey, uint32_t* __restrict__ gor) {
    __shared__ ScanRowsSmem<T> SS;
    scan_rows_body<T, SB, NT, STORE, DIAG, PIPE, U>(SS, cover, stego, H, W, bands_per_wg, ghist_all, gkey, gor);
}

// ------------------------------------------------------------------ K1': scan + copy (generic)
// Any W, any block size, dtype conversion / plane masking (nbits != dtype bits).
template <typename Tin, typename Tout>
__global__ __launch_bounds__(1024) void k_scan_generic(const Tin* __restrict__ cover, Tout* __restrict__ stego,
                                                       long long npx, long long px_per_wg, uint32_t keep,
                                                       uint32_t* __restrict__ ghist_all, uint32_t* __restrict__ gor) {
    __shared__ uint32_t lds[HistCfg<Tin>::kLdsWords];
    const int b = blockIdx.y;
    const Tin* src = cover + (size_t)b * npx;
    Tout* dst = stego ? stego + (size_t)b * npx : nullptr;
    uint32_t* ghist = ghist_all + (size_t)b * HistCfg<Tin>::kBins;
    for (int i = threadIdx.x; i < HistCfg<Tin>::kLdsWords; i += 1024) lds[i] = 0;
    __syncthreads();
    const long long q0 = (long long)blockIdx.x * px_per_wg;
    const long long q1 = min(npx, q0 + px_per_wg);
    uint32_t vor = 0;
    for (long long q = q0 + threadIdx.x; q < q1; q += 1024) {
        const uint32_t v = src[q];
        if (dst) dst[q] = (Tout)(v & keep);
        vor |= v;
        hist_add<Tin>(lds, ghist, v, 1u);
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) vor |= __shfl_xor(vor, o, 64);
    if ((threadIdx.x & 63) == 0 && vor) atomicOr(&gor[blockIdx.y], vor);
    __syncthreads();
    hist_flush<Tin>(lds, ghist);
}

// ------------------------------------------------------------------ K2: exact block variance
__device__ __forceinline__ int exact_count(int H, int W, int sb, int edge_only) {
    const int nby = (H + sb - 1) / sb, nbx = (W + sb - 1) / sb;
    if (!edge_only) return nby * nbx;
    const int ncol = (W % sb) ? nby : 0;
    const int nrow = (H % sb) ? (nbx - ((W % sb) ? 1 : 0)) : 0;
    return ncol + nrow;
}

__device__ __forceinline__ void exact_block(int e, int H, int W, int sb, int edge_only, int* by, int* bx) {
    const int nby = (H + sb - 1) / sb, nbx = (W + sb - 1) / sb;
    if (!edge_only) { *by = e / nbx; *bx = e % nbx; return; }
    const int ncol = (W % sb) ? nby : 0;
    if (e < ncol) { *by = e; *bx = nbx - 1; return; }
    *by = nby - 1;
    *bx = e - ncol;
}

// float(np.var(plane0[y:y1, x:x1])) exactly as numpy computes it (codec.py:446):
// mean = c/n; x - mean per element; squares; np.sum (pairwise, row-major); / n.
template <typename T>
__global__ __launch_bounds__(256) void k_block_exact(const T* __restrict__ img, int H, int W, int sb, int edge_only,
                                                     double* __restrict__ scores, int cap) {
    const int b = blockIdx.y;
    const int e = blockIdx.x * 256 + threadIdx.x;
    const int cnt = exact_count(H, W, sb, edge_only);
    if (e >= cnt) return;
    int by, bx;
    exact_block(e, H, W, sb, edge_only, &by, &bx);
    const int y0 = by * sb, x0 = bx * sb;
    const int bh = min(sb, H - y0), bw = min(sb, W - x0);
    const int n = bh * bw;
    const T* base = img + (size_t)b * H * W + (size_t)y0 * W + x0;
    int c = 0;
    for (int y = 0; y < bh; ++y)
        for (int x = 0; x < bw; ++x) c += base[(size_t)y * W + x] & 1;
    const double mean = (double)c / (double)n;
    const double a0 = (0.0 - mean) * (0.0 - mean);
    const double a1 = (1.0 - mean) * (1.0 - mean);
    auto elem = [&](int k) -> double {
        const int y = k / bw, x = k - y * bw;
        return (base[(size_t)y * W + x] & 1) ? a1 : a0;
    };
    const double sum = np_sum_serial(elem, n);
    scores[(size_t)b * cap + e] = sum / (double)n;
}

// ------------------------------------------------------------------ block-adaptive writes
// lsb_embed_block_adaptive (codec.py:372-404): run r = {plane, first pixel, length, first
// segment bit}; LSB := bit, bitmap := old ^ new (both as uint8, codec.py:395-399).  Runs
// never overlap (distinct blocks of one plane), so every pixel has one writer.
template <typename T>
__global__ __launch_bounds__(256) void k_lsb_runs(T* __restrict__ planes, uint8_t* __restrict__ bitmaps, long long npx,
                                                  const uint8_t* __restrict__ bits, long long bits_stride,
                                                  const long long* __restrict__ runs) {
    const long long* r = runs + 4 * (size_t)blockIdx.x;
    const long long p = r[0], off = r[1], len = r[2], src = r[3];
    T* px = planes + p * npx + off;
    uint8_t* bm = bitmaps + p * npx + off;
    const uint8_t* b = bits + p * bits_stride + src;
    for (long long i = threadIdx.x; i < len; i += 256) {
        const uint8_t old = (uint8_t)px[i];
        const uint8_t nw = (uint8_t)((old & 0xFE) | (b[i] & 1));
        px[i] = (T)nw;
        bm[i] = old ^ nw;
    }
}

// ------------------------------------------------------------------ per-slice window cache
struct SliceWin {
    int s, tot, npix;
    uint32_t flags;
    int perm[16], off[16], n[16], cat[16], src[16], sizes[16];
};

__device__ __forceinline__ void load_win(const codec_slice_meta* M, SliceWin* W) {
    const int i = threadIdx.x;   // 16 threads, one plane each (independent loads, one round trip)
    if (i < 16) {
        W->perm[i] = M->perm[i]; W->off[i] = M->off[i]; W->n[i] = M->n[i];
        W->cat[i] = M->cat[i]; W->src[i] = M->src[i]; W->sizes[i] = M->sizes[i];
        if (i == 0) { W->s = M->s; W->tot = M->total_used; W->npix = M->npix; W->flags = M->flags; }
    }
    __syncthreads();
}

// the windows in perm order for per-bit lookups: bit j lies in segment k = #(ends <= j),
// plane seg_p[k], pixel seg_q0[k] + j (mod npx) -- 16 register-held ends and two
// independent LDS reads per bit instead of plane_of's dependent search
__device__ __forceinline__ void win_segments(const SliceWin& W, int* seg_p, int* seg_q0, int (&ends)[16]) {
    const int k = threadIdx.x;
    if (k < 16 && k < W.s) {
        const int p = W.perm[k];
        seg_p[k] = p;
        seg_q0[k] = W.off[p] - W.cat[p];
    }
#pragma unroll
    for (int kk = 0; kk < 16; ++kk) ends[kk] = kk < W.s ? W.cat[W.perm[kk]] + W.n[W.perm[kk]] : 0x7FFFFFFF;
    __syncthreads();
}

// plane owning location-map bit j (segments are concatenated in perm order)
__device__ __forceinline__ int plane_of(const SliceWin& W, int j) {
    for (int k = 0; k < W.s; ++k) {
        const int p = W.perm[k];
        if (j < W.cat[p] + W.n[p]) return p;
    }
    return -1;
}

// ------------------------------------------------------------------ K3: decide
// identity order: element k is the k-th non-zero bin's term p*log2(p)
struct RankTerm {
    const double* terms;
    __device__ __forceinline__ double operator()(int k) const { return terms[k]; }
};
// permuted order: list[k] is the identity rank of the k-th element
struct ListTerm {
    const double* terms;
    const uint16_t* list;
    __device__ __forceinline__ double operator()(int k) const { return terms[list[k]]; }
};

#ifndef DECIDE_RP
// planes per round of the wave-parallel decision: 7 plane waves + the H(Y) wave = 2 waves
// per SIMD (8 put three on one SIMD: 33.4 -> 32.0 us per slice, tools/decide_phases.py)
#define DECIDE_RP 7
#endif
#ifndef DECIDE_RP2
// planes per round when each plane takes two waves: 5 (the usual s on 12-bit CT data) on waves
// 0-9 + the H(Y) wave = 1.5 plane-units per SIMD; a slice needing more planes runs another round
#define DECIDE_RP2 5
#endif
// split decision: a plane workgroup's "no value" (a NaN bit pattern, never a real H(X,Y))
#define PLANE_NONE 0x7FF8DEAD00000001ull
// a split decision's main workgroup that stopped waiting for a plane slot marks it ABANDONED
// (CAS 0 -> ABANDONED); the late plane workgroup's CAS then fails and it clears the slot
// itself, so no value of this launch can be read by the next one
#define PLANE_ABANDONED 0x7FF8DEAD00000002ull
// a plane workgroup whose slice the guard-banded decision settled (no joint sum needed)
#define PLANE_FAST 0x7FF8DEAD00000003ull
#ifdef DECIDE_TS   // diagnostic build only (tools/decide_phases.py): phase timestamps into the term scratch
// (b, role: decide_body's slice and workgroup role -- k_decide's blockIdx.x / .y; k_scan_decide
// runs slice blockIdx.y as role 0)
#define DTS(k) do { if (threadIdx.x == 0 && role == 0) reinterpret_cast<long long*>(gterms + (size_t)b * HistCfg<T>::kBins)[HistCfg<T>::kBins - 16 + (k)] = wall_clock64(); } while (0)
// plane workgroups of the split decision: 4 stamps each below the main's 16
#define PTS(k) do { if (threadIdx.x == 0) reinterpret_cast<long long*>(gterms + (size_t)b * HistCfg<T>::kBins)[HistCfg<T>::kBins - 80 + 4 * (role - 1) + (k)] = wall_clock64(); } while (0)
// wave path: lane 0 of wave k stamps the end of its first round's work (slot R - 80 + k)
#define WVTS(k) do { if ((threadIdx.x & 63) == 0 && role == 0) reinterpret_cast<long long*>(gterms + (size_t)b * HistCfg<T>::kBins)[HistCfg<T>::kBins - 80 + (k)] = wall_clock64(); } while (0)
// every wave's lane 0 stamps phase boundary `ph` (0: pass 1 done, 1: terms done) into its own slot
#define WPH(ph) do { if ((threadIdx.x & 63) == 0 && role == 0) reinterpret_cast<long long*>(gterms + (size_t)b * HistCfg<T>::kBins)[HistCfg<T>::kBins - 112 + 16 * (ph) + (threadIdx.x >> 6)] = wall_clock64(); } while (0)
#else
#define DTS(k) do { } while (0)
#define PTS(k) do { } while (0)
#define WVTS(k) do { } while (0)
#define WPH(ph) do { } while (0)
#endif
// CODEC_DECIDE_WAVES=0 (host env, passed in codec_params.reserved bit 0) forces the
// block-sequential decision path (A/B and tests)
__device__ __forceinline__ bool knob_dev_decide_fast(const codec_params& P) { return !(P.reserved & 1); }

__device__ __forceinline__ double plogp(const double* lut, uint32_t c, double N) {
    const double p = (double)c / N;       // counts[counts > 0] / size   (codec.py:498)
    return p * lut[c - 1];                // probabilities * np.log2(probabilities)  (:501)
}

// The order of the joint bincount of calculate_mutual_information (codec.py:546-551):
// index = bit * (max_val+1) + value, so the non-zero joint bins are the image's non-zero
// bins with bit `plane` = 0 (ascending value) followed by those with bit 1.  Each thread
// owns `bpt` consecutive bins (non-zero ones flagged in `nzmask`, identity ranks from
// `rank0`); `list` receives identity ranks in joint order.
__device__ void build_joint_order(u64 nzmask, int v0, uint32_t rank0, int plane, uint16_t* list, uint32_t* sh) {
    uint32_t oc = 0;
    for (u64 msk = nzmask; msk; msk &= msk - 1) oc += ((v0 + __ffsll((long long)msk) - 1) >> plane) & 1;
    const uint32_t zc = (uint32_t)__popcll(nzmask) - oc;
    uint32_t ztot, otot;
    uint32_t zp = block_excl_scan<1024>(zc, sh, &ztot);
    uint32_t op = block_excl_scan<1024>(oc, sh, &otot) + ztot;
    uint32_t r = rank0;
    for (u64 msk = nzmask; msk; msk &= msk - 1, ++r) {
        const int v = v0 + __ffsll((long long)msk) - 1;
        if ((v >> plane) & 1) list[op++] = (uint16_t)r; else list[zp++] = (uint16_t)r;
    }
    __syncthreads();
}

// build_joint_order with one packed scan (zero counts low, one counts high): m < 65536
__device__ void build_joint_order_m16(u64 nzmask, int v0, uint32_t rank0, int plane, uint16_t* list, uint32_t* sh) {
    uint32_t oc = 0;
    for (u64 msk = nzmask; msk; msk &= msk - 1) oc += ((v0 + __ffsll((long long)msk) - 1) >> plane) & 1;
    const uint32_t zc = (uint32_t)__popcll(nzmask) - oc;
    uint32_t tot;
    const uint32_t ex = block_excl_scan<1024>(zc | (oc << 16), sh, &tot);
    uint32_t zp = ex & 0xFFFFu, op = (ex >> 16) + (tot & 0xFFFFu);
    uint32_t r = rank0;
    for (u64 msk = nzmask; msk; msk &= msk - 1, ++r) {
        const int v = v0 + __ffsll((long long)msk) - 1;
        if ((v >> plane) & 1) list[op++] = (uint16_t)r; else list[zp++] = (uint16_t)r;
    }
    __syncthreads();
}

// EMBED: codec_encode's fused path -- after thread 0 has written the slice's windows, the
// workgroup embeds the slice's payload itself (k_embed's work, without its launch)
struct EmbedArgs {
    const void* cover;
    void* stego;
    const u64* payload;
    u64* maps;
    int pw, mw;
    uint32_t keep;
};

// k_decide's LDS, one struct so that the fused scan + decision kernel (k_scan_decide) can
// overlay it on the scan's (a union: `list` over the histogram, `vals` over the block counters)
template <typename T, bool EMBED>
struct DecideSmem {
    static constexpr int R = HistCfg<T>::kBins;
    static constexpr bool kWideT = sizeof(T) == 2;
    // `list` doubles as the wave-parallel path's arena: terms (8m B), rank -> value (2m B),
    // one joint-order list per plane in flight (2m B each)
    __align__(16) uint16_t list[R];
    double vals[sizeof(T) == 2 ? 2048 : 1024];   // 2048: the walk path's two orders
    uint32_t sh[20];
    u64 sh64[17];
    uint32_t pops_sh[16];
    double mis_sh[16];
    double best_sc[16];
    int best_ix[16];
    double hxy_sh[16], hx_sh[16], hy_sh;
    int ctl_sh[4];
    // walk path (wide 16-bit slices): non-zero masks per 64-bin group, terms by count
    u64 nzs[kWideT ? R / 64 : 1];
    double tcs[kWideT ? kTermCodes : 1];
    u64 pay_sh[EMBED ? 256 : 1];
    u64 slot_sh[16];
    int slot_to;
    int32_t lay_sh[sizeof(codec_layout) / 4];
    SliceWin Wsh;
    int seg_end[16], seg_p[16], seg_q0[16], seg_s0[16];
};

// what the fused kernel hands the decision: the slice's OR word and block key, and -- when the
// slice's counts fit (no 16-bit field wrapped, values < 4096) -- its histogram in the scan's
// LDS (16-bit halves), read by pass 1 instead of the global histogram
struct FusedScan {
    const uint32_t* lds;
    uint32_t orv;
    u64 key;
    bool lds_ok;
    // the decision's global inputs, loaded before the scan (their latency hides under it):
    // the slice's layout class, this thread's int of the class's 16 layouts, its payload word
    int cls;
    int32_t lay_v;
    u64 pay_v;
};

// FUSEDK: the fused scan + decision kernel (k_scan_decide).  LEAN (the fused kernel, and
// k_decide wherever the guard-banded decision applies: no all_mi, no forced split): the
// wave-parallel exact MI rounds and the walk path are compiled out -- a slice the guard band
// sends to the exact sums runs the block-sequential sums instead (over the LDS terms on the
// wave path) -- so the kernel carries the register pressure of the fast decision only
template <typename T, bool EMBED, bool FUSEDK = false, bool LEAN = FUSEDK>
__device__ __forceinline__ void decide_body(DecideSmem<T, EMBED>& S, const FusedScan* fz, const int b, const int role,
                                            codec_params P,
                                            uint32_t* __restrict__ ghist_all, uint32_t* __restrict__ gor,
                                            double* __restrict__ gterms, u64* __restrict__ gkey,
                                            const double* __restrict__ exact, int exact_cap, int exact_edge_only,
                                            int fast_blocks, const double* __restrict__ lut, long long lut_len,
                                            const codec_layout* __restrict__ table,
                                            const int32_t* __restrict__ slice_class,
                                            codec_slice_meta* __restrict__ meta_all, EmbedArgs E,
                                            u64* __restrict__ plane_slots, int nsplit, uint32_t spin_max,
                                            int dbg_late) {
    constexpr int R = HistCfg<T>::kBins;
    auto& list = S.list;
    auto& vals = S.vals;
    auto& sh = S.sh;
    auto& sh64 = S.sh64;
    auto& pops_sh = S.pops_sh;
    auto& mis_sh = S.mis_sh;
    auto& best_sc = S.best_sc;
    auto& best_ix = S.best_ix;
    auto& hxy_sh = S.hxy_sh;
    auto& hx_sh = S.hx_sh;
    double& hy_sh = S.hy_sh;
    auto& ctl_sh = S.ctl_sh;
    constexpr bool kWideT = sizeof(T) == 2;
    auto& nzs = S.nzs;
    auto& tcs = S.tcs;

    const int t = threadIdx.x;
    // split decision (small batches, nsplit > 0): blockIdx.y = 0 is the slice's main
    // workgroup; blockIdx.y = 1 + i computes plane i's joint entropy on its own CU and
    // publishes it in plane_slots[16 b + i] (see the plane branch below)
    const uint32_t* hist = ghist_all + (size_t)b * R;
    double* terms = gterms + (size_t)b * R;
    const long long npx = (long long)P.H * P.W;
    const double Nd = (double)npx;
    codec_slice_meta* M = meta_all + b;

    DTS(0);
    if (role > 0) PTS(0);
    // the scan's block key, loaded now (used by the offset argmax after the decision)
    // (thread 0, and lane 0 of waves 2 and 13: the fast decision / the paired MI round find the
    // offset on those idle waves)
    const bool keyed = (t == 0 || t == 128 || t == 832) && role == 0 && fast_blocks && P.fixed_offset < 0 && P.mode == CODEC_MODE_HYBRID;
    const u64 key0 = keyed ? (fz ? fz->key : gkey[b]) : 0ull;
    // the slice's layout class (its layout for s is loaded once s is known)
    constexpr int kLayW = (int)(sizeof(codec_layout) / 4);
    static_assert(16 * kLayW <= 1024, "one int of the class's layouts per thread");
    const int cls = fz ? fz->cls : role == 0 ? slice_class[b] : 0;
    const int32_t* lay_all = reinterpret_cast<const int32_t*>(table + (size_t)cls * 16);
    // fused embed: the slice's payload words (<= 2 KiB) go to LDS now, read by the embed
    // loop after the decision instead of one dependent global load per bit
    constexpr int kPaySh = EMBED ? 256 : 1;
    auto& pay_sh = S.pay_sh;
    const bool pay_in_lds = EMBED && E.pw <= kPaySh;
    static_assert(kPaySh <= 1024, "one payload word per thread");
    // requested now, parked in LDS just before the windows: a store here would hold the
    // workgroup until the load returns (one global round trip ahead of pass 1)
    const u64 pay_v = fz ? fz->pay_v : (EMBED && pay_in_lds && role == 0 && t < E.pw) ? E.payload[(size_t)b * E.pw + t] : 0ull;
    // 16-bit slices whose values stay below 4096 (12-bit CT): each thread's 4 bins [4t, 4t + 4)
    // of the global histogram are requested together with the OR word instead of one round
    // trip after it (bins at or above the range read as zero: the workspace is kept clean)
    constexpr bool kSpec = sizeof(T) == 2;
    uint4 spec = make_uint4(0u, 0u, 0u, 0u);
    if (kSpec && !fz) spec = reinterpret_cast<const uint4*>(hist)[t];
    // ---- bins that can be non-zero: [0, Rp), Rp = next power of two above OR(pixels)
    const uint32_t orv = fz ? fz->orv : gor[b];
    int Rp = orv ? (1 << (32 - __clz((int)orv))) : 1;
    // fused (k_scan_decide): pass 1 reads the counts from the scan's LDS histogram
    const uint32_t* flds = (fz && fz->lds_ok) ? fz->lds : nullptr;
    if (Rp > R) Rp = R;
    // <= 64 bins per thread; 16-bit slices below 4096 take 4 per thread (threads past the range
    // hold none), the speculative load's layout
    const int bpt = Rp > 4096 ? Rp / 1024 : kSpec ? 4 : Rp > 1024 ? Rp / 1024 : 1;
    const int v0 = t * bpt;
    const bool use_spec = kSpec && !fz && bpt == 4;

    // ---- pass 1: non-zero bins (bitmask), per-plane popcounts (the planes of codec.py:571)
    u64 nzmask = 0;
    uint32_t pop[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) pop[i] = 0;
    // wide slices (>= 16384 possible values): coalesced pass, one 64-bin group per wave
    // step, writing the group masks and the count codes (into the `list` arena) as well
    const bool wide = kWideT && Rp >= 16384 && !(P.reserved & 3);
    if (wide) {
        const int lane = t & 63, wv = t >> 6;
        // bin v = 64 g + lane, g = wv + 16 k: plane bits 0..5 are the lane's, 6..9 the
        // wave's, 10..15 those of k; only the lane total and the 6 k-bit sums are kept
        uint32_t tot = 0, pk[6] = {0, 0, 0, 0, 0, 0};
        const int ng = Rp / 64;
        for (int k0 = 0; wv + 16 * k0 < ng; k0 += 16) {       // 16 group loads in flight
            uint32_t cc[16];
#pragma unroll
            for (int u = 0; u < 16; ++u) {
                const int g = wv + 16 * (k0 + u);
                cc[u] = g < ng ? hist[(g << 6) + lane] : 0u;
            }
#pragma unroll
            for (int u = 0; u < 16; ++u) {
                const int k = k0 + u, g = wv + 16 * k;
                if (g >= ng) break;                               // uniform
                const uint32_t c = cc[u];
                list[cv_slot((g << 6) + lane)] = c < (uint32_t)kTermCodes ? (uint16_t)c : kBigCode;
                const u64 bm = __ballot(c != 0u);
                if (lane == 0) nzs[g] = bm;
                tot += c;
#pragma unroll
                for (int q = 0; q < 6; ++q) pk[q] += ((k >> q) & 1) ? c : 0u;
            }
        }
#pragma unroll
        for (int i = 0; i < 6; ++i) pop[i] = ((lane >> i) & 1) ? tot : 0u;
#pragma unroll
        for (int i = 6; i < 10; ++i) pop[i] = ((wv >> (i - 6)) & 1) ? tot : 0u;
#pragma unroll
        for (int i = 10; i < 16; ++i) pop[i] = pk[i - 10];
        for (int c = t; c < kTermCodes; c += 1024)
            tcs[c] = (c >= 1 && (long long)c <= npx && lut_len >= c) ? plogp(lut, (uint32_t)c, Nd) : 0.0;
        __syncthreads();
        const u64 w = nzs[v0 >> 6];
        nzmask = bpt == 64 ? w : (w >> (v0 & 63)) & ((1ull << bpt) - 1);
    }
    // small value ranges (every 12-bit slice): the non-zero counts are kept in LDS (`vals`,
    // free until the sums) for the terms pass, instead of a second histogram round trip
    uint32_t* cnt_sh = reinterpret_cast<uint32_t*>(vals);
    const bool cnt_lds = !wide && Rp <= (int)(sizeof(vals) / 4);
    // <= 8 bins per thread (Rp <= 8192: every 12-bit slice): the counts stay in registers and
    // their log2 table entries are requested at once, so that the table round trip runs under
    // the rank scan instead of after it
    const bool lut_pre = !wide && bpt <= 8 && lut_len >= npx;
    uint32_t c8[8];
    double l8[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) { c8[u] = 0u; l8[u] = 0.0; }
    for (int k0 = 0; k0 < bpt && !wide; k0 += 16) {
        uint32_t cc[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) {            // 16 loads in flight, then the adds
            const int v = v0 + k0 + u;
            if (use_spec && u < 4)
                cc[u] = v < Rp ? (u == 0 ? spec.x : u == 1 ? spec.y : u == 2 ? spec.z : spec.w) : 0u;
            else
                cc[u] = (k0 + u < bpt && v < Rp) ? (flds ? (flds[v >> 1] >> (16 * (v & 1))) & 0xFFFFu : hist[v]) : 0u;
        }
        if (lut_pre) {
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                c8[u] = cc[u];
                if (cc[u]) l8[u] = lut[cc[u] - 1];
            }
        }
#pragma unroll
        for (int u = 0; u < 16; ++u) {
            const int v = v0 + k0 + u;
            if (cc[u]) {
                if (cnt_lds) cnt_sh[v] = cc[u];
                nzmask |= 1ull << (k0 + u);
                if (bpt != 4) {
#pragma unroll
                    for (int i = 0; i < 16; ++i) pop[i] += ((v >> i) & 1) ? cc[u] : 0u;
                }
            }
        }
        if (bpt == 4) {   // bins 4t .. 4t + 3: planes 0 and 1 differ inside, planes >= 2 are bits of t
            const uint32_t tot = cc[0] + cc[1] + cc[2] + cc[3];
            pop[0] = cc[1] + cc[3];
            pop[1] = cc[2] + cc[3];
#pragma unroll
            for (int i = 2; i < 16; ++i) pop[i] = ((t >> (i - 2)) & 1) ? tot : 0u;
        }
    }
    DTS(12);
    WPH(0);
    // the entry prefetches are consumed here, with pass 1's loads (issued before them, so
    // no extra wait): left to themselves they sink to their first use after the decision
    if (!fz) asm volatile("" ::"v"((uint32_t)key0), "v"((uint32_t)(key0 >> 32)), "s"(cls));
    // the class's 16 layouts (one int per thread), requested now, stored into LDS after the terms
    const int32_t lay_v = fz ? fz->lay_v : (role == 0 && t < 16 * kLayW) ? lay_all[t] : 0;
    if (t < 16) pops_sh[t] = 0;
    uint32_t m;
    // LDS-only barriers from here to the embed (lds_barrier): a __syncthreads would also wait
    // for every global access in flight -- the log2-table prefetch above, the meta stores of
    // the windows phase -- where only LDS needs ordering
    const uint32_t rank0 = block_excl_scan_lds<1024>((uint32_t)__popcll(nzmask), sh, &m);
    DTS(13);
    {   // the 16 per-plane sums of the wave as one reduce-scatter: 8 + 4 + 2 + 1 shuffles leave
        // lane l with plane l >> 2 summed over 16 lanes, two more finish it (17 instead of 96)
        // (lane ^ 32 and ^ 16 by gfx950's permlane swaps, ^ 8 by a DPP row rotation, ^ 4 by a
        // swizzle, ^ 2 and ^ 1 by quad permutes: no bpermute round trip through the LDS crossbar)
        const int lane = t & 63;
        uint32_t a[8], b4[4], c2[2];
        const bool h3 = (lane >> 3) & 1, h2 = (lane >> 2) & 1;
#pragma unroll
        for (int j = 0; j < 8; ++j) {   // lanes < 32 keep plane j, lanes >= 32 plane 8 + j
            const auto sw = __builtin_amdgcn_permlane32_swap(pop[j], pop[8 + j], false, false);
            a[j] = sw[0] + sw[1];
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {   // lanes with bit 4 clear keep a[j], the others a[4 + j]
            const auto sw = __builtin_amdgcn_permlane16_swap(a[j], a[4 + j], false, false);
            b4[j] = sw[0] + sw[1];
        }
#pragma unroll
        for (int j = 0; j < 2; ++j)     // row_ror:8 inside a 16-lane row is lane ^ 8
            c2[j] = (h3 ? b4[2 + j] : b4[j]) +
                    (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(h3 ? b4[j] : b4[2 + j]), 0x128, 0xF, 0xF, false);
        uint32_t x = (h2 ? c2[1] : c2[0]) +
                     (uint32_t)__builtin_amdgcn_ds_swizzle((int)(h2 ? c2[0] : c2[1]), 0x101F);   // lane ^ 4
        x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x4E, 0xF, 0xF, false);   // quad_perm [2,3,0,1]
        x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0xB1, 0xF, 0xF, false);   // quad_perm [1,0,3,2]
        if ((lane & 3) == 0 && x) atomicAdd(&pops_sh[lane >> 2], x);
    }
    DTS(1);
    const bool lut_ok = lut_len >= npx;
    // wave-parallel path (m small enough that terms + per-plane joint orders fit in LDS):
    // each wave sums one plane's H(X,Y) with np_sum_wave, no block barriers inside a sum
    // arena: terms (8m B) | rank -> value (2m B) | per 64-rank group, the 16 bit-plane
    // ballots of its values (128 B) | one joint-order list per plane in flight (2m B)
    const size_t arena = sizeof(list);
    const int ngrp = (int)((m + 63) / 64);
    const size_t off_pm = (10 * (size_t)m + 15) / 16 * 16;
    const size_t off_jl = off_pm + (size_t)ngrp * 128;
    const int wplanes = (m > 1 && off_jl + 2 * (size_t)m <= arena) ? (int)min((size_t)16, (arena - off_jl) / (2 * (size_t)m)) : 0;
    const bool wfast = lut_ok && wplanes >= 1 && knob_dev_decide_fast(P);
    // (compiled out of the fused kernel: a wide slice there sums its terms from global memory
    // on the block path -- with the guard band that is H(Y) alone for nearly every slice)
    const bool walk = !LEAN && wide && lut_ok && !wfast && m > 1;
    double* tl = reinterpret_cast<double*>(list);
    uint16_t* rv = reinterpret_cast<uint16_t*>(tl + (wfast ? m : 0));
    u64* pm = reinterpret_cast<u64*>(reinterpret_cast<char*>(list) + off_pm);
    uint16_t* jl = reinterpret_cast<uint16_t*>(reinterpret_cast<char*>(list) + off_jl);
    if (wfast) terms = tl;
    // the guard-banded decision (below) needs H(Y) only to ~1e-13: this thread's terms summed
    // in any order
    const bool try_fast = P.fixed_s <= 0 && !P.all_mi && lut_ok && !(P.reserved & 8);
    double hy_part = 0.0;
    // terms of the non-zero bins in ascending value order, computed once
    if (lut_ok && !walk && lut_pre) {   // from pass 1's registers: bin v0 + u has rank rank0 + (set bits below u)
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            if ((nzmask >> u) & 1ull) {
                const uint32_t r = rank0 + (uint32_t)__popcll(nzmask & ((1ull << u) - 1ull));
                const double tt = ((double)c8[u] / Nd) * l8[u];      // plogp: p * log2(p)
                terms[r] = tt;
                hy_part += tt;
                if (wfast) rv[r] = (uint16_t)(v0 + u);
            }
        }
    } else if (lut_ok && !walk) {
        uint32_t r = rank0;
        u64 msk = nzmask;
        while (msk) {
            int vv[8];
            uint32_t cc[8];
            int k = 0;
#pragma unroll
            for (int u = 0; u < 8; ++u) {         // up to 8 independent hist->lut chains
                vv[u] = -1;
                if (msk) { vv[u] = v0 + __ffsll((long long)msk) - 1; msk &= msk - 1; ++k; }
            }
#pragma unroll
            for (int u = 0; u < 8; ++u) cc[u] = vv[u] >= 0 ? (cnt_lds ? cnt_sh[vv[u]] : hist[vv[u]]) : 1u;
            double tt[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) tt[u] = plogp(lut, cc[u], Nd);
#pragma unroll
            for (int u = 0; u < 8; ++u)
                if (u < k) { terms[r + u] = tt[u]; hy_part += tt[u]; }
            if (wfast) {
#pragma unroll
                for (int u = 0; u < 8; ++u)
                    if (u < k) rv[r + u] = (uint16_t)vv[u];
            }
            r += k;
        }
    }
    if (try_fast) DTS(8);
    WPH(1);
    if (try_fast && walk) {   // wide slices: no term array -- the count codes of pass 1, a wave per group
        const int lane = t & 63, wv = t >> 6, ng = Rp / 64;
        for (int g0 = wv; g0 < ng; g0 += 16 * 8) {
            uint16_t cc[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int g = g0 + 16 * u;
                cc[u] = g < ng ? list[cv_slot((g << 6) + lane)] : (uint16_t)0;
            }
#pragma unroll
            for (int u = 0; u < 8; ++u)
                hy_part += cc[u] != kBigCode ? tcs[cc[u]] : plogp(lut, hist[((g0 + 16 * u) << 6) + lane], Nd);
        }
    }
    if (t < 16) mis_sh[t] = 0.0;
    if (wfast) lds_barrier();   // the terms are in LDS (uniform)
    else __syncthreads();       // the terms went to global memory

    // ---- the s decision, guard-banded.  X = f(Y), so I(X;Y) = H(X) exactly: the
    // reference's MI (codec.py:554, h_x + h_y - h_xy from two numpy-order sums) differs from
    // H(X) only by the rounding of its sums, |d| <= ~1e-13 per plane (a pairwise sum of terms
    // totalling <= 16 bits; measured <= 3.6e-14 on 48 slices).  So s is decided from the
    // cumulative H(X) against beta * H(Y) with H(Y) summed in any order, unless a prefix of
    // that walk lies within kDecideGuard of its target: then -- or when all_mi asks for every
    // exact value, or fixed_s skips the decision -- the numpy-order joint sums below decide as
    // before.  A slice decided here records CODEC_FLAG_INFO_FAST (mi[] = H(X) of the planes
    // the loop evaluated, cum_info their sum); one that fell back, CODEC_FLAG_GUARD_FALLBACK.
    constexpr double kDecideGuard = 1e-9;
    int fs = 0;               // uniform: s of the fast decision, 0 = the exact path decides
    bool guard_fb = false;    // uniform: the guard band sent the slice to the exact path
    double fast_cum = 0.0;    // thread 0
    // the start offset (codec.py:441-453; independent of s): find_offset below, or one wave's
    // shuffles (wave_offset) where a wave is idle meanwhile
    const int sb = P.block;
    const int nbx = (P.W + sb - 1) / sb;
    double bsc = -1.0;
    int bix = 0x7FFFFFFF;
    bool offset_done = false;
    const bool need_offset = P.fixed_offset < 0 && P.mode == CODEC_MODE_HYBRID;
    // first maximal float(np.var) block in raster order: the exact scores of the partial /
    // non-power-of-two blocks and the scan's packed key (lane 0 holds it), reduced by the calling
    // wave alone (score desc, raster index asc) into best_sc[0] / best_ix[0]
    auto wave_offset = [&]() {
        const int lane = t & 63;
        double ws = -1.0;
        int wi = 0x7FFFFFFF;
        const int cnt = exact_count(P.H, P.W, sb, exact_edge_only);
        for (int e = lane; e < cnt; e += 64) {
            int by, bx;
            exact_block(e, P.H, P.W, sb, exact_edge_only, &by, &bx);
            const double sc = exact[(size_t)b * exact_cap + e];
            const int ix = by * nbx + bx;
            if (sc > ws || (sc == ws && ix < wi)) { ws = sc; wi = ix; }
        }
        if (lane == 0 && fast_blocks && key0) {
            const uint32_t score = (uint32_t)(key0 >> 32);
            const int ix = (int)(0xFFFFFFFFu - (uint32_t)(key0 & 0xFFFFFFFFu));
            const double sc = (double)score / ((double)sb * sb * (double)sb * sb);
            if (sc > ws || (sc == ws && ix < wi)) { ws = sc; wi = ix; }
        }
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) {
            const double os = __shfl_xor(ws, o, 64);
            const int oi = __shfl_xor(wi, o, 64);
            if (os > ws || (os == ws && oi < wi)) { ws = os; wi = oi; }
        }
        if (lane == 0) { best_sc[0] = ws; best_ix[0] = wi; }
    };
    // the record's exact H(Y) (numpy's order, 8 lanes per leaf over the whole workgroup, slot
    // sums in vals[512..], clear of the layouts) and the offset ride along with the fast
    // decision on the wave path, so a settled slice goes straight to its windows
    const bool pre = try_fast && wfast && role == 0;
    if (try_fast) {
        const int lane = t & 63, wv = t >> 6;
        if (pre) {
            if (t < 16 * kLayW) reinterpret_cast<int32_t*>(vals)[t] = lay_v;   // the class's 16 layouts (one per s)
            np_leaves_block1024(RankTerm{tl}, (int)m, vals + 512, 8);   // waves 8.. (clear of waves 0-2)
        }
        const double hp = wave_sum_f64(hy_part);  // any order: the fast H(Y)
        if (lane == 0) hxy_sh[wv] = hp;           // scratch until the exact rounds
        const int nb = min(P.nbits, 16);
        double hx = 0.0;                          // wave 1, lane i: H(X) of plane i
        if (wv == 1 && lane < nb) {   // codec.py:530-532; log2 on the device (no table round trip)
            const uint32_t pp = pops_sh[lane];
            const double p1 = (double)pp / Nd, p0 = (double)(npx - pp) / Nd;
            hx = (pp != 0 && (long long)pp != npx) ? -(p0 * log2(p0) + p1 * log2(p1)) : 0.0;
        }
        DTS(6);
        lds_barrier();
        DTS(7);
        if (wv == 1) {   // the walk, lane-parallel: prefix sums of H(X) against beta * H(Y)
            const double tg = P.beta * -wave_sum_f64(lane < 16 ? hxy_sh[lane] : 0.0);
            const double c = row_incl_scan_f64(hx);   // lanes 0..15; 0 for a constant plane (codec.py:520-523)
            const u64 reach = __ballot(lane < nb && c >= tg);
            const int sf = reach ? __ffsll((long long)reach) : 1;   // codec.py:591-593; s = 1 if never
            const int nev = reach ? sf : nb;                         // planes the loop evaluates
            // every evaluated prefix more than the guard from its target (a NaN fails it too)
            const bool clear = __ballot(lane < nev && !(fabs(c - tg) > kDecideGuard)) == 0ull;
            const double cum = __longlong_as_double(
                ((long long)__builtin_amdgcn_readlane((int)(__double_as_longlong(c) >> 32), nev - 1) << 32) |
                (long long)(uint32_t)__builtin_amdgcn_readlane((int)__double_as_longlong(c), nev - 1));
            if (clear && lane < nev) mis_sh[lane] = hx;
            if (lane == 0) { ctl_sh[2] = clear ? sf : 0; hxy_sh[0] = cum; }   // after the wave's reads
            WVTS(1);
        }
        if (pre && wv == 8) {
            const double h = np_combine_slots_wave((int)m, vals + 512);
            if (lane == 0) hy_sh = -h;
            WVTS(0);
        }
        if (pre && wv == 2 && need_offset) { wave_offset(); WVTS(2); }
        lds_barrier();
        DTS(9);
        fs = ctl_sh[2];
        guard_fb = fs == 0;
        if (t == 0) fast_cum = hxy_sh[0];
    }

    if (role > 0 && fs) {   // split decision, decided without the joint sums: nothing to compute
        if (t == 0) {
            u64* sp = plane_slots + 16 * (size_t)b + (role - 1);
            u64 expect = 0ull;
            if (!__hip_atomic_compare_exchange_strong(sp, &expect, PLANE_FAST, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                      __HIP_MEMORY_SCOPE_AGENT) && expect == PLANE_ABANDONED)
                __hip_atomic_store(sp, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        return;
    }
    if (role > 0) {
        // ---- a plane workgroup: H(X,Y) of plane i over the whole CU -- the joint order by
        // a block scan, numpy's pairwise sum by np_sum_block1024 (the same tree as the wave
        // path's np_sum_wave, so the value is bit-identical) -- published as its bit pattern
        // (never 0: the main workgroup polls for non-zero).  Planes the main workgroup will
        // not read (constant plane, slice off the wave path) publish PLANE_NONE.
        const int i = role - 1;
        u64 pub = PLANE_NONE;
        const uint32_t pp = pops_sh[i];
        PTS(1);
        if (wfast && i < min(P.nbits, 16) && pp != 0 && (long long)pp != npx) {
            build_joint_order_m16(nzmask, v0, rank0, i, jl, sh);   // wave path: m < 65536
            PTS(2);
            const double h = -np_sum_block1024_w0(ListTerm{tl, jl}, (int)m, vals);
            PTS(3);
            pub = (u64)__double_as_longlong(h);
            if (pub == 0ull) pub = 0x8000000000000000ull;   // +0.0 -> -0.0: same MI
        }
        if (t == 0) {
            u64* sp = plane_slots + 16 * (size_t)b + i;
            if (b == 0 && i == dbg_late) {
                // CODEC_DECIDE_DEBUG_LATE (tests only): this plane publishes only after the main
                // workgroup has given up on it -- the late-publication path, made deterministic
                for (uint32_t k = 0; k < (1u << 20); ++k) {   // bounded (~0.2 s)
                    if (__hip_atomic_load(sp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) break;
                    __builtin_amdgcn_s_sleep(8);
                }
            }
            u64 expect = 0ull;
            if (!__hip_atomic_compare_exchange_strong(sp, &expect, pub, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                      __HIP_MEMORY_SCOPE_AGENT) && expect == PLANE_ABANDONED)
                __hip_atomic_store(sp, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);   // nobody reads it: clear
        }
        return;
    }
    // main workgroup of a split decision: wait for every plane workgroup's value (they read
    // the histogram this workgroup clears at the end); the slots are cleared for the next
    // call at the end, with the histogram (a store here would be waited for by the next
    // vmcnt wait of the wave, ~2 us)
    auto& slot_sh = S.slot_sh;
    int& slot_to = S.slot_to;
    bool collected = false;
    bool abandoned = false;   // thread t < nsplit: slot t was given up (the late writer clears it)
    auto collect = [&]() {
        if (t == 0) slot_to = 0;
        __syncthreads();
        if (t < nsplit) {
            u64* sp = plane_slots + 16 * (size_t)b + t;
            u64 v = 0;
            for (uint32_t k = 0; k < spin_max; ++k) {   // bounded: co-resident by construction
                v = __hip_atomic_load(sp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (v) break;
                __builtin_amdgcn_s_sleep(2);
            }
            if (!v) {   // give up -- unless the value lands between the last poll and the mark
                u64 expect = 0ull;
                if (__hip_atomic_compare_exchange_strong(sp, &expect, PLANE_ABANDONED, __ATOMIC_RELAXED,
                                                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
                    v = PLANE_NONE;
                    slot_to = 1;
                    abandoned = true;
                } else {
                    v = expect;
                }
            }
            // a plane workgroup that took the guard-banded route while this one did not (the
            // two evaluate the same test on the same histogram, so never): an error, not a value
            if (v == PLANE_FAST && !fs) slot_to = 1;
            slot_sh[t] = v;
        }
        __syncthreads();
        collected = true;
    };

    // ---- start offset: first maximal float(np.var) block in raster order (codec.py:441-453);
    // independent of s, so the split decision finds it while its plane workgroups work
    auto find_offset = [&]() {
        offset_done = true;
        if (!(P.fixed_offset < 0 && P.mode == CODEC_MODE_HYBRID)) return;
        const int cnt = exact_count(P.H, P.W, sb, exact_edge_only);
        for (int e = t; e < cnt; e += 1024) {
            int by, bx;
            exact_block(e, P.H, P.W, sb, exact_edge_only, &by, &bx);
            const double sc = exact[(size_t)b * exact_cap + e];
            const int ix = by * nbx + bx;
            if (sc > bsc || (sc == bsc && ix < bix)) { bsc = sc; bix = ix; }
        }
        if (t == 0 && fast_blocks) {
            const u64 key = key0;
            if (key) {
                const uint32_t score = (uint32_t)(key >> 32);
                const int ix = (int)(0xFFFFFFFFu - (uint32_t)(key & 0xFFFFFFFFu));
                const double n2 = (double)sb * sb * (double)sb * sb;
                const double sc = (double)score / n2;
                if (sc > bsc || (sc == bsc && ix < bix)) { bsc = sc; bix = ix; }
            }
        }
        // block argmax (score desc, raster index asc)
        const int lane = t & 63, wv = t >> 6;
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) {
            const double os = __shfl_xor(bsc, o, 64);
            const int oi = __shfl_xor(bix, o, 64);
            if (os > bsc || (os == bsc && oi < bix)) { bsc = os; bix = oi; }
        }
        if (lane == 0) { best_sc[wv] = bsc; best_ix[wv] = bix; }
        __syncthreads();
        if (t == 0) {
            for (int w = 1; w < 16; ++w)
                if (best_sc[w] > bsc || (best_sc[w] == bsc && best_ix[w] < bix)) { bsc = best_sc[w]; bix = best_ix[w]; }
        }
    };

    DTS(2);
    // ---- calculate_entropy (codec.py:489-502) = H(Y) inside calculate_mutual_information
    double Hy = 0.0;
    int s = 1;
    bool decided = false;
    double cum = 0.0;
    if (fs) { s = fs; decided = true; cum = fast_cum; }   // the exact loops below stop at once
    const bool need_decision = (P.fixed_s <= 0);
    if (!LEAN && wfast && nsplit > 0 && !fs) {
        // split decision: H(Y) here (wave 15) while the plane workgroups sum their orders,
        // then thread 0 takes the planes in order exactly like the sequential loop
        const int wv = t >> 6, lane = t & 63;
        if (wv == 15) {
            const double h = -np_sum_wave(RankTerm{tl}, (int)m);
            if (lane == 0) hy_sh = h;
        }
        // H(X) of every plane meanwhile (its two table loads off thread 0's walk)
        if (wv == 1 && lane < min(P.nbits, 16)) {
            const uint32_t pp = pops_sh[lane];
            hx_sh[lane] = (pp != 0 && (long long)pp != npx) ? -(plogp(lut, (uint32_t)(npx - pp), Nd) + plogp(lut, pp, Nd)) : 0.0;
        }
        // the class's 16 layouts (one per s) into LDS meanwhile (`vals` is free here)
        if (t < 16 * kLayW) reinterpret_cast<int32_t*>(vals)[t] = lay_v;
        find_offset();   // meanwhile (its barrier also orders hx_sh / hy_sh)
        DTS(8);
        collect();
        DTS(14);
        Hy = hy_sh;
        if (t == 0) {
            const double target0 = P.beta * Hy;
            const int nb = min(P.nbits, 16);
            for (int ii = 0; ii < nb; ++ii) {
                if (!(need_decision && !decided) && !P.all_mi) break;
                const uint32_t pp = pops_sh[ii];
                double mi = 0.0;
                if (pp != 0 && (long long)pp != npx) {                // codec.py:520-523
                    const double hx = hx_sh[ii];
                    const double hxy = __longlong_as_double((long long)slot_sh[ii]);
                    mi = (hx + Hy) - hxy;                               // codec.py:554
                    if (!(mi > 0.0)) mi = 0.0;
                }
                mis_sh[ii] = mi;
                if (need_decision && !decided) {
                    cum += mi;
                    if (cum >= target0) { s = ii + 1; decided = true; }
                }
            }
        }
    } else if (wfast && fs) {
        // settled by the guard band: the record's exact H(Y), the start offset and the layouts
        // came with it
        Hy = hy_sh;
        if (t == 0 && need_offset) { bsc = best_sc[0]; bix = best_ix[0]; }
        offset_done = true;
    } else if (!LEAN && wfast) {
        // H(Y) by wave 0; then rounds of `wplanes` planes, plane i0+w on wave w: its joint
        // bincount order (bit-i-clear bins ascending, then bit-i-set bins, codec.py:546-551)
        // is written to its own list and summed with np_sum_wave.  Thread 0 then walks the
        // round's planes in order exactly like the sequential loop (same early exit).
        const int wv = t >> 6, lane = t & 63;
        // the class's 16 layouts (one per s) into LDS now (`vals` is free until the windows):
        // loaded after the decision they were one dependent global round trip (~2 us)
        if (t < 16 * kLayW) reinterpret_cast<int32_t*>(vals)[t] = lay_v;
        // paired planes (one buffer of m <= 8192 ranks): each plane's list build and leaf sums
        // go to two waves (2k, 2k + 1: different SIMDs), DECIDE_RP2 planes per round -- the round
        // is VALU-issue bound, and two planes on one SIMD were its critical path.
        // vals: the layouts (ints [0, 1024)), then the pairs' slot exchange and sync counters
        const bool pair = !(P.reserved & 4) && m <= NP_CHUNK && ngrp >= 2 && wplanes >= 1;
        int* pcnt = reinterpret_cast<int*>(vals + 896);
        if (pair && t < 8) pcnt[t] = 0;                  // ordered by the barrier after the masks
        const u64 lt = lane ? (~0ull >> (64 - lane)) : 0ull;
        for (int g = wv; g < ngrp; g += 16) {             // bit-plane ballots per rank group
            const int r = g * 64 + lane;
            const uint32_t v = r < (int)m ? rv[r] : 0u;
            uint32_t lo = 0, hi = 0;                       // lane i < 16 collects plane i's ballot
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const u64 bm = __ballot((v >> i) & 1u);
                lo = lane == i ? (uint32_t)bm : lo;
                hi = lane == i ? (uint32_t)(bm >> 32) : hi;
            }
            if (lane < 16) pm[g * 16 + lane] = (u64)lo | ((u64)hi << 32);
        }
        __syncthreads();
        DTS(8);
        // planes per round: enough for the usual s (5 on 12-bit data, 7 on uniform 16-bit),
        // few enough that the round's waves are not sharing SIMDs 4 to 1 (each list build and
        // sum is VALU-issue bound); H(Y) runs on the last wave meanwhile
        const int rp = min(wplanes, DECIDE_RP);
        if (wv == 15) {
            const double h = -np_sum_wave(RankTerm{tl}, (int)m);
            if (lane == 0) hy_sh = h;
            WVTS(15);
        }
        const int nb = min(P.nbits, 16);
        if (t == 0) ctl_sh[0] = 0;
        if (pair) {
            const int rp2 = min(wplanes, DECIDE_RP2);
            const int k = wv >> 1, h = wv & 1;
            double* xbuf = vals + 512 + 64 * k;                        // wave 2k+1's slot sums (k < 5)
            const int gh = (ngrp + 1) / 2;                             // groups of the first half
            // the start offset meanwhile (it does not depend on s), on idle wave 13 with wave
            // shuffles only -- find_offset's block barriers and cross-wave pass stay off the
            // path after the round (C3: ~2.9 us there); thread 0 picks it up after the rounds
            if (wv == 13 && need_offset) wave_offset();
            offset_done = true;   // every thread (uniform): find_offset is not called below
            // H(X) of every plane meanwhile, on an idle wave (its two table loads stay off the
            // pairs' critical path); read by thread 0's walk after the round's barrier
            if (wv == 14 && lane < nb) {
                const uint32_t pp = pops_sh[lane];
                hx_sh[lane] = (pp != 0 && (long long)pp != npx) ? -(plogp(lut, (uint32_t)(npx - pp), Nd) + plogp(lut, pp, Nd)) : 0.0;
            }
            int base = 0;
            for (int i0 = 0; i0 < nb; i0 += rp2) {
                const int i = i0 + k;
                if (wv < 2 * rp2 && i < nb) {
                    const uint32_t pp = pops_sh[i];
                    const bool run = pp != 0 && (long long)pp != npx;
                    uint16_t* L = jl + (size_t)k * m;
                    if (run) {
                        uint32_t ones = 0, onesA = 0;
                        for (int g = lane; g < ngrp; g += 64) {
                            const uint32_t c = (uint32_t)__popcll(pm[g * 16 + i]);
                            ones += c;
                            onesA += g < gh ? c : 0u;
                        }
#pragma unroll
                        for (int o = 32; o >= 1; o >>= 1) {
                            ones += __shfl_xor(ones, o, 64);
                            onesA += __shfl_xor(onesA, o, 64);
                        }
                        // half h: groups [g0, g1); the first half's groups are full (64 ranks)
                        const int g0 = h ? gh : 0, g1 = h ? ngrp : gh;
                        uint32_t zbase = h ? (uint32_t)gh * 64u - onesA : 0u;
                        uint32_t obase = (uint32_t)m - ones + (h ? onesA : 0u);
                        for (int blk = g0; blk < g1; blk += 64) {
                            const int gl = blk + lane;
                            const u64 mkl = gl < g1 ? pm[gl * 16 + i] : 0ull;
                            const int ng = min(64, g1 - blk);
                            for (int gg = 0; gg < ng; ++gg) {
                                const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)mkl, gg);
                                const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(mkl >> 32), gg);
                                const u64 mk = (u64)lo | ((u64)hi << 32);
                                const int g = blk + gg;
                                const int nr = min(64, (int)m - g * 64);
                                const u64 valid = nr >= 64 ? ~0ull : ((1ull << nr) - 1ull);
                                const u64 zm = ~mk & valid;
                                const bool one = (mk >> lane) & 1ull;
                                const uint32_t below = __builtin_amdgcn_mbcnt_hi((uint32_t)((one ? mk : zm) >> 32),
                                                       __builtin_amdgcn_mbcnt_lo((uint32_t)(one ? mk : zm), 0u));
                                if (lane < nr) L[(one ? obase : zbase) + below] = (uint16_t)(g * 64 + lane);
                                obase += (uint32_t)__popcll(mk);
                                zbase += (uint32_t)__popcll(zm);
                            }
                        }
                    }
                    // sync 1: both halves of the list are written
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                    if (lane == 0) atomicAdd(&pcnt[k], 1);
                    if (run) {
                        while (__hip_atomic_load(&pcnt[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < base + 2)
                            __builtin_amdgcn_s_sleep(1);
                        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
                    }
                    // the chunk tree's bottom slots: wave 2k lane l takes slot l, wave 2k+1 slot l + 64
                    double v = 0.0;
                    if (run) {
                        int a = 0;
                        const int n = np_node_size((int)m, 7, lane + 64 * h, &a);
                        v = n > 0 ? np_leaf(ListTerm{tl, L}, a, n) : 0.0;
                    }
                    if (h) {   // sync 2: hand the upper slots to wave 2k
                        if (run) xbuf[lane] = v;
                        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                        if (lane == 0) atomicAdd(&pcnt[k], 1);
                    } else {
                        double hxy = 0.0;
                        if (run) {
                            while (__hip_atomic_load(&pcnt[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < base + 3)
                                __builtin_amdgcn_s_sleep(1);
                            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
                            double res = -0.0;                         // np_sum_wave's buffer sum
                            res += np_combine_wave(v, xbuf[lane], (int)m);
                            hxy = -res;
                            if (i0 == 0) WVTS(wv);
                        }
                        if (lane == 0) hxy_sh[k] = hxy;
                    }
                    base += 3;
                }
                __syncthreads();
                if (t == 0) {
                    Hy = hy_sh;
                    const double target0 = P.beta * Hy;
                    int stop = 0;
                    for (int kk = 0; kk < rp2 && i0 + kk < nb; ++kk) {
                        const int ii = i0 + kk;
                        if (!(need_decision && !decided) && !P.all_mi) { stop = 1; break; }
                        const uint32_t pp = pops_sh[ii];
                        double mi = 0.0;
                        if (pp != 0 && (long long)pp != npx) {                // codec.py:520-523
                            mi = (hx_sh[ii] + Hy) - hxy_sh[kk];              // codec.py:554
                            if (!(mi > 0.0)) mi = 0.0;
                        }
                        mis_sh[ii] = mi;
                        if (need_decision && !decided) {
                            cum += mi;
                            if (cum >= target0) { s = ii + 1; decided = true; }
                        }
                    }
                    if (!(need_decision && !decided) && !P.all_mi) stop = 1;
                    ctl_sh[0] = stop;
                }
                __syncthreads();
                if (ctl_sh[0]) break;
            }
        }
        if (pair && t == 0 && P.fixed_offset < 0 && P.mode == CODEC_MODE_HYBRID) {   // wave 13's offset
            bsc = best_sc[0];   // (ordered by the rounds' barriers)
            bix = best_ix[0];
        }
        for (int i0 = 0; i0 < nb && !pair; i0 += rp) {
            const int i = i0 + wv;
            if (wv < rp && i < nb) {
                const uint32_t pp = pops_sh[i];
                double hxy = 0.0;
                if (pp != 0 && (long long)pp != npx) {
                    // joint order from the group ballots (rank group g's bit-i mask)
                    uint16_t* L = jl + (size_t)wv * m;
                    uint32_t ones = 0;
                    for (int g = lane; g < ngrp; g += 64) ones += (uint32_t)__popcll(pm[g * 16 + i]);
#pragma unroll
                    for (int o = 32; o >= 1; o >>= 1) ones += __shfl_xor(ones, o, 64);
                    uint32_t zbase = 0, obase = (uint32_t)m - ones;      // ones follow all zeros
                    // one rank group per step, the whole wave on it: lane e places rank
                    // 64 g + e at the next zero / one position (mbcnt of the group's mask), so
                    // each step is one store of two contiguous runs.  The masks of 64 groups
                    // sit one per lane and are broadcast with readlane (uniform, no LDS trip).
                    for (int blk = 0; blk < ngrp; blk += 64) {
                        const int gl = blk + lane;
                        const u64 mkl = gl < ngrp ? pm[gl * 16 + i] : 0ull;
                        const int ng = min(64, ngrp - blk);
                        if (i0 == 0 && wv == 0 && blk == 0) DTS(9);
                        for (int gg = 0; gg < ng; ++gg) {
                            const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)mkl, gg);
                            const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(mkl >> 32), gg);
                            const u64 mk = (u64)lo | ((u64)hi << 32);
                            const int g = blk + gg;
                            const int nr = min(64, (int)m - g * 64);        // ranks in group g
                            const u64 valid = nr >= 64 ? ~0ull : ((1ull << nr) - 1ull);
                            const u64 zm = ~mk & valid;
                            const bool one = (mk >> lane) & 1ull;
                            const uint32_t below = __builtin_amdgcn_mbcnt_hi((uint32_t)((one ? mk : zm) >> 32),
                                                   __builtin_amdgcn_mbcnt_lo((uint32_t)(one ? mk : zm), 0u));
                            if (lane < nr) L[(one ? obase : zbase) + below] = (uint16_t)(g * 64 + lane);
                            obase += (uint32_t)__popcll(mk);
                            zbase += (uint32_t)__popcll(zm);
                        }
                    }
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                    __builtin_amdgcn_wave_barrier();
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                    if (i0 == 0) DTS(7);
                    hxy = -np_sum_wave(ListTerm{tl, L}, (int)m);
                    if (i0 == 0) DTS(6);
                    if (i0 == 0) WVTS(wv);
                    if (lane == 0) hx_sh[wv] = -(plogp(lut, (uint32_t)(npx - pp), Nd) + plogp(lut, pp, Nd));
                }
                if (lane == 0) hxy_sh[wv] = hxy;
            }
            __syncthreads();
            if (t == 0) {
                Hy = hy_sh;
                const double target0 = P.beta * Hy;
                int stop = 0;
                for (int k = 0; k < rp && i0 + k < nb; ++k) {
                    const int ii = i0 + k;
                    if (!(need_decision && !decided) && !P.all_mi) { stop = 1; break; }
                    const uint32_t pp = pops_sh[ii];
                    double mi = 0.0;
                    if (pp != 0 && (long long)pp != npx) {                // codec.py:520-523
                        mi = (hx_sh[k] + Hy) - hxy_sh[k];                // codec.py:554
                        if (!(mi > 0.0)) mi = 0.0;
                    }
                    mis_sh[ii] = mi;
                    if (need_decision && !decided) {
                        cum += mi;
                        if (cum >= target0) { s = ii + 1; decided = true; }
                    }
                }
                if (!(need_decision && !decided) && !P.all_mi) stop = 1;
                ctl_sh[0] = stop;
            }
            __syncthreads();
            if (ctl_sh[0]) break;
        }
        Hy = hy_sh;
    }
    if (walk) {
        // joint orders walked from the group masks, two per np_sum_walk2: (H(Y), plane 0),
        // (1, 2), (3, 4), ...; the planes are then taken in order as the sequential loop does
        const JointWalk w0{nzs, list, tcs, hist, lut, Nd, -1, Rp / 64, 0, 0, 0, 0ull};
        double tg = 0.0;
        const int nb = min(P.nbits, 16);
        bool stop = false;
        for (int i0 = -1; i0 < nb && !stop; i0 += 2) {
            if (i0 >= 0 && !(need_decision && !decided) && !P.all_mi) break;
            int run[2];
#pragma unroll
            for (int q = 0; q < 2; ++q) {
                const int i = i0 + q;
                const uint32_t pp = (i >= 0 && i < nb) ? pops_sh[i] : 0u;
                run[q] = i < 0 || (!fs && i < nb && pp != 0 && (long long)pp != npx);   // codec.py:520-523
            }
#ifdef DECIDE_TS
            long long* wts = i0 < 0 ? reinterpret_cast<long long*>(gterms + (size_t)b * R) + R - 4 : nullptr;
#else
            long long* wts = nullptr;
#endif
            double hs2[2];
            np_sum_walk2(w0, i0, run[0] ? (int)m : 0, i0 + 1, run[1] ? (int)m : 0, vals, sh64, hs2, wts);
            for (int q = 0; q < 2; ++q) {
                const int i = i0 + q;
                if (i >= nb) break;
                if (i < 0) { Hy = -hs2[0]; tg = P.beta * Hy; DTS(6); continue; }
                if (!(need_decision && !decided) && !P.all_mi) { stop = true; break; }
                const uint32_t pp = pops_sh[i];
                double mi = 0.0;
                if (run[q]) {
                    const double hx = -(plogp(lut, (uint32_t)(npx - pp), Nd) + plogp(lut, pp, Nd));
                    mi = (hx + Hy) - (-hs2[q]);                  // codec.py:554
                    if (!(mi > 0.0)) mi = 0.0;
                }
                if (t == 0) mis_sh[i] = mi;
                if (need_decision && !decided) {
                    cum += mi;
                    if (cum >= tg) { s = i + 1; decided = true; }
                }
            }
            if (i0 < 0) DTS(7);
        }
    }
    // the block-sequential path: slices off the wave path, and the fused kernel's exact sums
    // (its terms stay in LDS: joint orders at jl, tree slots at vals[512..], the layouts kept)
    const bool blockp = lut_ok && !walk && (!wfast || (LEAN && !fs));
    const double* bt = wfast ? tl : terms;
    uint16_t* bl = wfast ? jl : list;
    double* bv = wfast ? vals + 512 : vals;
    if (blockp && wfast && t < 16 * kLayW) reinterpret_cast<int32_t*>(vals)[t] = lay_v;
    if (blockp) Hy = pre ? hy_sh : -np_sum_block1024(RankTerm{bt}, (int)m, bv);
    const double target = P.beta * Hy;

    // ---- the s decision (codec.py:580-593)
    for (int i = 0; i < P.nbits && i < 16 && blockp; ++i) {
        if (!(need_decision && !decided) && !P.all_mi) break;
        const uint32_t pp = pops_sh[i];
        double mi = 0.0;
        if (m > 1 && pp != 0 && (long long)pp != npx) {          // codec.py:520-523
            build_joint_order(nzmask, v0, rank0, i, bl, sh);
            if (i == 0) DTS(6);
            const double hxy = -np_sum_block1024(ListTerm{bt, bl}, (int)m, bv);
            if (i == 0) DTS(7);
            const double hx = -(plogp(lut, (uint32_t)(npx - pp), Nd) + plogp(lut, pp, Nd));
            mi = (hx + Hy) - hxy;                                // codec.py:554
            if (!(mi > 0.0)) mi = 0.0;                           // max(0.0, mi)
        }
        if (t == 0) mis_sh[i] = mi;
        if (need_decision && !decided) {
            cum += mi;
            if (cum >= target) { s = i + 1; decided = true; }
        }
    }
    if (!need_decision) s = P.fixed_s;

    // the slice's segment layout for its s (64 ints), loaded by one wave in one round trip
    // while the offset is found, instead of thread 0's dependent loads in the windows loop
    auto& lay_sh = S.lay_sh;
    // lay_sh and everything the windows read are written and read by wave 0 (thread 0's s, the
    // offset, the layouts), so no barrier follows the fill; s itself crosses waves only on the
    // exact paths (thread 0 decided there) -- the guard band's s is every thread's
    if (t == 0) ctl_sh[1] = s;
    if (!fs) lds_barrier();
    {
        const int sl = fs ? fs : min(max(ctl_sh[1], 1), 16);
        if (t < kLayW) lay_sh[t] = wfast ? reinterpret_cast<const int32_t*>(vals)[(sl - 1) * kLayW + t]
                                         : lay_all[(sl - 1) * kLayW + t];
    }

    DTS(3);
    if (!offset_done) find_offset();

    SliceWin& Wsh = S.Wsh;   // the fused embed's window cache, filled by thread 0 below
    // ... and its segments in perm order: bit j belongs to the first k with j < seg_end[k];
    // pixel = seg_q0[k] + j (mod npx), payload bit = seg_s0[k] + j
    auto& seg_end = S.seg_end;
    auto& seg_p = S.seg_p;
    auto& seg_q0 = S.seg_q0;
    auto& seg_s0 = S.seg_s0;
    if (EMBED && pay_in_lds && role == 0 && t < E.pw) pay_sh[t] = pay_v;   // read by the embed loop (after its barrier)
    DTS(4);
    if (t < 64) {   // ---- windows and the slice record (wave 0: lane j = segment j in perm order)
    const int lane = t;
    const int sdec = ctl_sh[1];                    // thread 0's s (the wave path decides there)
    const int bix0 = __shfl(bix, 0, 64);
    const double cum0 = __shfl(cum, 0, 64);
    int offset = 0;
    if (P.fixed_offset >= 0) offset = P.fixed_offset;
    else if (P.mode == CODEC_MODE_HYBRID) offset = (bix0 / nbx) * sb * P.W + (bix0 % nbx) * sb;
    if (offset < 0 || (long long)offset >= npx) offset = 0;   // no block scored (never for valid stats)

    // ---- segment windows (codec.py:455-485 / 288-316).  The layout's perm is a permutation
    // of the planes 0..s-1, so lane j < s owns plane perm[j] and lane p in [s, 16) plane p.
    const codec_layout& L = *reinterpret_cast<const codec_layout*>(lay_sh);
    const bool segl = lane < sdec;
    const int p = segl ? L.perm[lane] : (lane & 15);
    const int len = segl ? L.len[p] : 0;
    const int n = segl ? (int)min((long long)len, npx) : 0;
    const bool lossy = segl && (len != L.sizes[p] || n != len);
    int incl = n;                                    // segments are concatenated in perm order
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) {
        const int y = __shfl_up(incl, o, 64);
        if (lane >= o) incl += y;
    }
    const int catj = incl - n;                       // == the sequential loop's `cat` before j
    const int cat = __shfl(incl, 15, 64);            // total (s <= 16)
    // pos advances by n mod npx per segment (hybrid, not aligned): (offset + cat_j) mod npx
    const int off = (!segl || P.mode == CODEC_MODE_MULTI) ? 0
                  : P.align ? offset : (int)(((long long)offset + catj) % npx);
    const int sz = !segl ? 0 : P.mode == CODEC_MODE_MULTI ? n : L.sizes[p];   // codec.py:315 / 425,487
    if (lane < 16) {
        M->perm[lane] = segl ? p : -1;
        M->n[p] = n; M->src[p] = segl ? L.src[p] : 0; M->cat[p] = catj; M->off[p] = off; M->sizes[p] = sz;
        M->mi[lane] = mis_sh[lane];
    }
    if (EMBED && segl) { seg_end[lane] = catj + n; seg_p[lane] = p; seg_q0[lane] = off - catj; seg_s0[lane] = L.src[p] - catj; }
    int maxn = n;
#pragma unroll
    for (int o = 8; o >= 1; o >>= 1) maxn = max(maxn, __shfl_xor(maxn, o, 64));
    uint32_t flags = __ballot(lossy) ? CODEC_FLAG_LOSSY : 0u;
    if (lane == 0) {
    const int s = sdec;
    if ((P.mode == CODEC_MODE_MULTI && s > 1) || (P.align && s > 1) || (long long)cat > npx) flags |= CODEC_FLAG_OVERLAP;
    if (!lut_ok) flags |= CODEC_FLAG_BADLUT;
    if (fs) flags |= CODEC_FLAG_INFO_FAST;
    if (guard_fb) flags |= CODEC_FLAG_GUARD_FALLBACK;
    M->s = s;
    M->start_offset = (P.mode == CODEC_MODE_HYBRID) ? offset : 0;
    M->total_used = cat;
    M->flags = flags;
    M->npix = (int)npx;
    M->nbits = P.nbits;
    M->status = lut_ok ? 0 : 1;
    if (collected && slot_to) { M->status = 2; flags |= CODEC_FLAG_DECIDE_TIMEOUT; M->flags = flags; }
    M->nonzero_bins = (int)m;
    M->entropy = Hy;
    M->target = target;
    M->cum_info = cum0;
    {   // circular hull of the windows (lets a streaming pass skip untouched chunks cheaply)
        const bool shared_start = (P.mode == CODEC_MODE_MULTI) || P.align;
        const long long hl = shared_start ? maxn : cat;
        M->span_lo = (P.mode == CODEC_MODE_HYBRID) ? offset : 0;
        M->span_len = (int)min(hl, npx);
    }
    if constexpr (EMBED) { Wsh.s = s; Wsh.tot = cat; Wsh.npix = (int)npx; Wsh.flags = flags; }
    DTS(5);
    }
    }
    if constexpr (EMBED) {
        const SliceWin& W = Wsh;
        // Wsh, seg_* (the meta stores need not land first).  Fused: a full barrier -- the scan's
        // stego copy stores (left in flight) must land before the window pixels are rewritten
        if constexpr (FUSEDK) __syncthreads(); else lds_barrier();
        DTS(10);
        const T* cv = static_cast<const T*>(E.cover) + (size_t)b * npx;
        T* sv = static_cast<T*>(E.stego) + (size_t)b * npx;
        const u64* pay = E.payload + (size_t)b * E.pw;
        // 8 bits per thread per round: all payload-word and cover loads of the round are
        // issued before any store (the stores may alias the cover, so a per-bit loop would
        // serialise one HBM round trip per bit)
        const int lim = min(W.tot, E.mw * 64);
        // segment ends in registers (a linear search per bit instead of dependent LDS reads)
        int ends[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) ends[k] = k < W.s ? seg_end[k] : 0x7FFFFFFF;
        for (int j0 = 0; j0 < lim; j0 += 8 * 1024) {
            int pl[8];
            long long ql[8];
            uint32_t mb[8], orig[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const int j = j0 + k * 1024 + t;
                pl[k] = -1;
                if (j < lim) {
                    int sg = 0;
#pragma unroll
                    for (int kk = 0; kk < 16; ++kk) sg += j >= ends[kk] ? 1 : 0;
                    const int p = seg_p[sg];
                    long long q = (long long)seg_q0[sg] + j;
                    if (q >= npx) q -= npx;
                    const long long sbit = (long long)seg_s0[sg] + j;
                    pl[k] = p;
                    ql[k] = q;
                    mb[k] = (uint32_t)((pay_in_lds ? pay_sh[sbit >> 6] : pay[sbit >> 6]) >> (sbit & 63)) & 1u;
                    orig[k] = cv[q];
                }
            }
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                if (j0 + k * 1024 >= lim) break;                 // uniform
                const int j = j0 + k * 1024 + t;
                uint32_t mapbit = 0;
                if (pl[k] >= 0) {
                    const int p = pl[k];
                    if (!(W.flags & CODEC_FLAG_OVERLAP)) {
                        sv[ql[k]] = (T)(((orig[k] & E.keep) & ~(1u << p)) | (mb[k] << p));
                    } else {
                        const size_t byte = (size_t)ql[k] * sizeof(T);
                        uint32_t* word = reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(sv) + (byte & ~(size_t)3));
                        const uint32_t bit = 1u << ((byte & 3) * 8 + p);
                        if (mb[k]) atomicOr(word, bit); else atomicAnd(word, ~bit);
                    }
                    mapbit = ((orig[k] >> p) & 1u) ^ mb[k];
                }
                const u64 bal = __ballot(mapbit);
                if ((t & 63) == 0 && (j >> 6) < E.mw) E.maps[(size_t)b * E.mw + (j >> 6)] = bal;
            }
        }
        // map words past the last round (no window bit): 0, so the whole map is defined (the
        // rounds above wrote the words of every 1024-bit step that starts below lim)
        for (int w = ((lim + 1023) / 1024) * 16 + t; w < E.mw; w += 1024) E.maps[(size_t)b * E.mw + w] = 0ull;
        DTS(11);
    }
    if (nsplit > 0 && !collected) {   // the other decision paths: slots still to clear
        collect();
        if (t == 0 && slot_to) { M->status = 2; M->flags |= CODEC_FLAG_DECIDE_TIMEOUT; }
    }
    // leave the workspace clean for the next call (codec_plan does not memset it): every
    // histogram bin the scan can have touched lies below max(Rp, 2) (pixel values < Rp; a
    // 16-bit wrap fix-up also writes bin v + 1 <= Rp - 1, or bin 1 when Rp = 1), plus the
    // slice's block key and OR word.  All reads of them precede this barrier.
    __syncthreads();
    if (t < nsplit && !abandoned) plane_slots[16 * (size_t)b + t] = 0ull;
    if (!flds) {   // fused with the LDS histogram: the global one was never written
        const int zr = Rp < 2 ? 2 : Rp;
        uint32_t* hz = ghist_all + (size_t)b * R;
        if ((zr & 3) == 0) {
            uint4* h4 = reinterpret_cast<uint4*>(hz);
            for (int v = t; v < zr / 4; v += 1024) h4[v] = make_uint4(0u, 0u, 0u, 0u);
        } else {
            for (int v = t; v < zr; v += 1024) hz[v] = 0u;
        }
    }
    if (t == 0) { gkey[b] = 0ull; gor[b] = 0u; }
}

template <typename T, bool EMBED = false, bool LEAN = false>
__global__ __launch_bounds__(1024) void k_decide(codec_params P, uint32_t* __restrict__ ghist_all,
                                                 uint32_t* __restrict__ gor, double* __restrict__ gterms,
                                                 u64* __restrict__ gkey, const double* __restrict__ exact,
                                                 int exact_cap, int exact_edge_only, int fast_blocks,
                                                 const double* __restrict__ lut, long long lut_len,
                                                 const codec_layout* __restrict__ table,
                                                 const int32_t* __restrict__ slice_class,
                                                 codec_slice_meta* __restrict__ meta_all, EmbedArgs E,
                                                 u64* __restrict__ plane_slots, int nsplit, uint32_t spin_max,
                                                 int dbg_late) {
    __shared__ DecideSmem<T, EMBED> S;
    decide_body<T, EMBED, false, LEAN>(S, nullptr, (int)blockIdx.x, (int)blockIdx.y, P, ghist_all, gor, gterms, gkey, exact, exact_cap, exact_edge_only, fast_blocks,
                          lut, lut_len, table, slice_class, meta_all, E, plane_slots, nsplit, spin_max, dbg_late);
}

// ------------------------------------------------------------------ K1 + K3 fused: scan + decide
// For batches whose slices each fit one scan workgroup (C3's 256 x 512^2: the row sweep runs one
// workgroup per slice anyway) the workgroup that scanned slice b decides it too, with codec_encode's
// embed, in the same launch: the histogram is still in its LDS (read by pass 1 instead of a global
// flush + reload), there is no kernel boundary, and each slice's decision starts as soon as its own
// scan ends, overlapping other slices' streaming.  The two LDS layouts are overlaid (a union: the
// decision's arena over the histogram, its `vals` over the block counters; both are dead by then).
// A slice whose counts left LDS (a 16-bit field wrapped) or whose values reach 4096 and beyond
// flushes the histogram to global memory as k_scan_rows would and decides from there.
template <typename T, int SB, bool NT>
__global__ __launch_bounds__(1024) void k_scan_decide(const T* __restrict__ cover, T* __restrict__ stego,
                                                      int bands_per_wg, codec_params P, uint32_t* __restrict__ ghist_all,
                                                      uint32_t* __restrict__ gor, double* __restrict__ gterms,
                                                      u64* __restrict__ gkey, const double* __restrict__ exact,
                                                      int exact_cap, int exact_edge_only, const double* __restrict__ lut,
                                                      long long lut_len, const codec_layout* __restrict__ table,
                                                      const int32_t* __restrict__ slice_class,
                                                      codec_slice_meta* __restrict__ meta_all, EmbedArgs E) {
    union FusedSmem {
        ScanRowsSmem<T> s;
        DecideSmem<T, true> d;
    };
    __shared__ FusedSmem U;
    const int b = blockIdx.y;
#ifdef DECIDE_TS   // diagnostic build: the workgroup's start (slot 15 of the decision's stamps)
    long long ts_start = 0;
    if (threadIdx.x == 0) ts_start = wall_clock64();
#endif
    // the decision's global inputs first: their latency hides under the scan
    const int cls = slice_class[b];
    constexpr int kLayW = (int)(sizeof(codec_layout) / 4);
    const int32_t lay_v = threadIdx.x < 16 * kLayW ? reinterpret_cast<const int32_t*>(table + (size_t)cls * 16)[threadIdx.x] : 0;
    const u64 pay_v = ((int)threadIdx.x < E.pw && E.pw <= 256) ? E.payload[(size_t)b * E.pw + threadIdx.x] : 0ull;
    scan_rows_body<T, SB, NT, true, 0, true, 4, true>(U.s, cover, stego, P.H, P.W, bands_per_wg, ghist_all, gkey, gor);
#ifdef DECIDE_TS
    if (threadIdx.x == 0) reinterpret_cast<long long*>(gterms + (size_t)b * HistCfg<T>::kBins)[HistCfg<T>::kBins - 1] = ts_start;
#ifdef DECIDE_TS_SCAN_ONLY   // diagnostic: the scan alone (decisions invalid), its start spread
    if (threadIdx.x == 0) reinterpret_cast<long long*>(gterms + (size_t)b * HistCfg<T>::kBins)[HistCfg<T>::kBins - 16] = wall_clock64();
    return;
#endif
#endif
    // scan_rows_body ended with a barrier after its last LDS write (the block key)
    FusedScan fz;
    fz.lds = U.s.lds;
    fz.orv = U.s.wor;
    fz.key = U.s.wkey;
    const int Rp = fz.orv ? (1 << (32 - __clz((int)fz.orv))) : 1;
    fz.lds_ok = sizeof(T) == 2 && U.s.wrap == 0u && Rp <= 4096;
    fz.cls = cls;
    fz.lay_v = lay_v;
    fz.pay_v = pay_v;
    if (!fz.lds_ok) {   // uniform: the global histogram path (wrap fix-ups are already there)
        hist_flush<T>(U.s.lds, ghist_all + (size_t)b * HistCfg<T>::kBins);
        __threadfence();
        __syncthreads();   // the flush lands before pass 1 reads it back
    } else {
        lds_barrier();     // every read of the scan's LDS words above precedes the decision's writes
    }
    decide_body<T, true, true>(U.d, &fz, b, 0, P, ghist_all, gor, gterms, gkey, exact, exact_cap, exact_edge_only, 1, lut,
                         lut_len, table, slice_class, meta_all, E, nullptr, 0, 0u, -1);
}

// ------------------------------------------------------------------ K4: embed (window writes)
// location-map bit j of one slice: window write of payload bit src[p] + i into plane p of
// pixel off[p] + i (codec.py:455-485 / 288-316); returns cover_bit ^ message_bit
template <typename Tin, typename Tout>
__device__ __forceinline__ uint32_t embed_bit(const Tin* __restrict__ cover, Tout* __restrict__ stego, long long npx,
                                              uint32_t keep, const u64* __restrict__ payload, const SliceWin& W, int j) {
    const int p = plane_of(W, j);
    const int i = j - W.cat[p];
    long long q = (long long)W.off[p] + i;
    if (q >= npx) q -= npx;
    const long long sbit = (long long)W.src[p] + i;
    const uint32_t mb = (uint32_t)(payload[sbit >> 6] >> (sbit & 63)) & 1u;
    const uint32_t orig = cover[q];
    if (!(W.flags & CODEC_FLAG_OVERLAP)) {
        stego[q] = (Tout)(((orig & keep) & ~(1u << p)) | (mb << p));
    } else {
        const size_t byte = (size_t)q * sizeof(Tout);
        uint32_t* word = reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(stego) + (byte & ~(size_t)3));
        const uint32_t bit = 1u << ((byte & 3) * 8 + p);
        if (mb) atomicOr(word, bit); else atomicAnd(word, ~bit);
    }
    return ((orig >> p) & 1u) ^ mb;
}

template <typename Tin, typename Tout>
__global__ __launch_bounds__(256) void k_embed(const Tin* __restrict__ cover, Tout* __restrict__ stego,
                                               long long npx, uint32_t keep, const u64* __restrict__ payload,
                                               int pw, const codec_slice_meta* __restrict__ meta,
                                               u64* __restrict__ maps, int mw) {
    __shared__ SliceWin W;
    const int b = blockIdx.y;
    load_win(meta + b, &W);
    const int j = blockIdx.x * 256 + threadIdx.x;
    if ((j & ~63) >= W.tot) {   // whole wave past the end (uniform): its map word reads 0
        if ((threadIdx.x & 63) == 0 && (j >> 6) < mw) maps[(size_t)b * mw + (j >> 6)] = 0ull;
        return;
    }
    uint32_t mapbit = 0;
    if (j < W.tot)
        mapbit = embed_bit<Tin, Tout>(cover + (size_t)b * npx, stego + (size_t)b * npx, npx, keep,
                                      payload + (size_t)b * pw, W, j);
    const u64 bal = __ballot(mapbit);
    if ((threadIdx.x & 63) == 0) maps[(size_t)b * mw + (j >> 6)] = bal;
}

// ------------------------------------------------------------------ K5: extraction
struct Range { int q0, q1, p, j0; };   // pixels [q0,q1) of plane p, map bit of q0 = j0

__device__ int build_ranges(const SliceWin& W, Range* R) {
    int k = 0;
    for (int jj = 0; jj < W.s; ++jj) {
        const int p = W.perm[jj];
        const int n = W.n[p];
        if (n <= 0) continue;
        const int off = W.off[p];
        const long long end = (long long)off + n;
        if (end <= W.npix) {
            R[k++] = Range{off, (int)end, p, W.cat[p]};
        } else {
            R[k++] = Range{off, W.npix, p, W.cat[p]};
            R[k++] = Range{0, (int)(end - W.npix), p, W.cat[p] + (W.npix - off)};
        }
    }
    return k;
}

__device__ __forceinline__ uint32_t map_bit(const u64* maps, long long j) {
    return (uint32_t)(maps[j >> 6] >> (j & 63)) & 1u;
}

// cover = stego with every window bit XOR-ed with its location-map bit (stream copy)
template <typename T, bool NT>
__global__ __launch_bounds__(256) void k_restore(const T* __restrict__ stego, T* __restrict__ cover, long long npx,
                                                 const codec_slice_meta* __restrict__ meta,
                                                 const u64* __restrict__ maps_all, int mw, long long chunks_per_wg) {
    typedef typename Vec8<T>::type V;
    __shared__ Range rg[32];
    __shared__ int nrg;
    const int b = blockIdx.y;
    const long long nchunks = npx / 8;
    const long long c0 = (long long)blockIdx.x * chunks_per_wg;
    const long long c1 = min(nchunks, c0 + chunks_per_wg);
    // prologue, parallel: lane p < s contributes plane p's (<= 2) window ranges, kept only
    // if they touch this workgroup's pixels (most workgroups keep none)
    if (threadIdx.x == 0) nrg = 0;
    __syncthreads();
    if (threadIdx.x < 16) {
        const codec_slice_meta* M = meta + b;
        const int p = threadIdx.x;
        if (p < M->s) {
            const int n = M->n[p], off = M->off[p], cat = M->cat[p];
            const long long lo = c0 * 8, hi = (blockIdx.x == gridDim.x - 1) ? npx : c1 * 8;
            if (n > 0) {
                const long long end = (long long)off + n;
                Range r0{off, (int)min(end, npx), p, cat};
                if (r0.q0 < hi && r0.q1 > lo) rg[atomicAdd(&nrg, 1)] = r0;
                if (end > npx) {
                    Range r1{0, (int)(end - npx), p, cat + (int)(npx - off)};
                    if (r1.q0 < hi && r1.q1 > lo) rg[atomicAdd(&nrg, 1)] = r1;
                }
            }
        }
    }
    __syncthreads();
    const int nr = nrg;
    const u64* maps = maps_all + (size_t)b * mw;
    const V* src = reinterpret_cast<const V*>(stego + (size_t)b * npx);
    V* dst = reinterpret_cast<V*>(cover + (size_t)b * npx);
    for (long long cb = c0 + threadIdx.x; cb < c1; cb += 4 * 256) {
      V vv[4];
#pragma unroll
      for (int u = 0; u < 4; ++u)
          if (cb + u * 256 < c1) vv[u] = ldv<NT>(src + cb + u * 256);
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const long long ch = cb + u * 256;
        if (ch >= c1) break;
        V v = vv[u];
        const long long q0 = ch * 8;
        for (int k = 0; k < nr; ++k) {
            const Range r = rg[k];
            if (q0 + 8 <= r.q0 || q0 >= r.q1) continue;
            uint32_t px[8];
            if constexpr (sizeof(T) == 2) {
                px[0] = v.x & 0xFFFFu; px[1] = v.x >> 16; px[2] = v.y & 0xFFFFu; px[3] = v.y >> 16;
                px[4] = v.z & 0xFFFFu; px[5] = v.z >> 16; px[6] = v.w & 0xFFFFu; px[7] = v.w >> 16;
            } else {
                for (int e = 0; e < 4; ++e) { px[e] = (v.x >> (8 * e)) & 0xFFu; px[4 + e] = (v.y >> (8 * e)) & 0xFFu; }
            }
            for (int e = 0; e < 8; ++e) {
                const long long q = q0 + e;
                if (q >= r.q0 && q < r.q1) px[e] ^= map_bit(maps, r.j0 + (q - r.q0)) << r.p;
            }
            if constexpr (sizeof(T) == 2) {
                v.x = px[0] | (px[1] << 16); v.y = px[2] | (px[3] << 16);
                v.z = px[4] | (px[5] << 16); v.w = px[6] | (px[7] << 16);
            } else {
                v.x = px[0] | (px[1] << 8) | (px[2] << 16) | (px[3] << 24);
                v.y = px[4] | (px[5] << 8) | (px[6] << 16) | (px[7] << 24);
            }
        }
        stv<NT>(dst + ch, v);
      }
    }
    // scalar tail (npx % 8) handled by the last workgroup
    if (blockIdx.x == gridDim.x - 1) {
        for (long long q = nchunks * 8 + threadIdx.x; q < npx; q += 256) {
            uint32_t px = stego[(size_t)b * npx + q];
            for (int k = 0; k < nr; ++k) {
                const Range r = rg[k];
                if (q >= r.q0 && q < r.q1) px ^= map_bit(maps, r.j0 + (q - r.q0)) << r.p;
            }
            cover[(size_t)b * npx + q] = (T)px;
        }
    }
}

// Grid-stride variant: the whole batch is swept as one address-ordered stream (the
// fastest pattern measured, tools/ubench_stream.hip); a chunk is tested against its slice's
// window hull (span_lo/span_len, 2 loads from the L2-resident meta) and only the rare
// chunks inside it walk the per-plane windows.
template <typename T>
__device__ __forceinline__ void restore_chunk(typename Vec8<T>::type& v, long long q0, const codec_slice_meta* M,
                                              const u64* maps, long long npx) {
    uint32_t px[8];
    if constexpr (sizeof(T) == 2) {
        px[0] = v.x & 0xFFFFu; px[1] = v.x >> 16; px[2] = v.y & 0xFFFFu; px[3] = v.y >> 16;
        px[4] = v.z & 0xFFFFu; px[5] = v.z >> 16; px[6] = v.w & 0xFFFFu; px[7] = v.w >> 16;
    } else {
        for (int e = 0; e < 4; ++e) { px[e] = (v.x >> (8 * e)) & 0xFFu; px[4 + e] = (v.y >> (8 * e)) & 0xFFu; }
    }
    const int s = M->s;
    for (int p = 0; p < s; ++p) {
        const int n = M->n[p];
        if (n <= 0) continue;
        const long long off = M->off[p], cat = M->cat[p];
        for (int e = 0; e < 8; ++e) {
            long long i = q0 + e - off;
            if (i < 0) i += npx;
            if (i < n) px[e] ^= map_bit(maps, cat + i) << p;
        }
    }
    if constexpr (sizeof(T) == 2) {
        v.x = px[0] | (px[1] << 16); v.y = px[2] | (px[3] << 16);
        v.z = px[4] | (px[5] << 16); v.w = px[6] | (px[7] << 16);
    } else {
        v.x = px[0] | (px[1] << 8) | (px[2] << 16) | (px[3] << 24);
        v.y = px[4] | (px[5] << 8) | (px[6] << 16) | (px[7] << 24);
    }
}

__device__ __forceinline__ bool span_hit(long long q0, long long lo, long long len, long long npx) {
    const long long hi = lo + len;
    return (q0 + 8 > lo && q0 < hi) || (hi > npx && q0 < hi - npx);
}

// Grid-stride variant: the whole batch is swept as one address-ordered stream.  Each
// iteration of a workgroup covers 1024 consecutive chunks; their slice (and its window
// hull span_lo/span_len) is looked up once per iteration, wave-uniformly, and only chunks
// inside the hull walk the per-plane windows.
template <typename T, bool NT, int NTH = 256>
__global__ __launch_bounds__(NTH) void k_restore_gs(const T* __restrict__ stego, T* __restrict__ cover,
                                                    uint32_t npx, uint32_t nchunks, uint32_t total_chunks,
                                                    const codec_slice_meta* __restrict__ meta,
                                                    const u64* __restrict__ maps_all, int mw,
                                                    int gather_wgs, u64* __restrict__ payload_out, int pw) {
    typedef typename Vec8<T>::type V;
    // the first gather_wgs workgroups gather the payload of slice blockIdx.x (dispatched first,
    // they overlap the stream instead of a separate launch after it)
    if ((int)blockIdx.x < gather_wgs) {
        gather_body<T, NTH>(stego, (long long)npx, meta, payload_out, pw, (int)blockIdx.x);
        return;
    }
    const uint32_t wg = blockIdx.x - (uint32_t)gather_wgs;
    const V* src = reinterpret_cast<const V*>(stego);
    V* dst = reinterpret_cast<V*>(cover);
    const uint32_t stride = (gridDim.x - (uint32_t)gather_wgs) * (4u * NTH);
    for (uint32_t base = wg * (4u * NTH); base < total_chunks; base += stride) {
        const uint32_t cb = base + threadIdx.x;
        V vv[4];
#pragma unroll
        for (int u = 0; u < 4; ++u)
            if (cb + u * (uint32_t)NTH < total_chunks) vv[u] = ldv<NT>(src + cb + u * (uint32_t)NTH);
        const uint32_t last = min(base + (4u * NTH - 1u), total_chunks - 1);
        const uint32_t b0 = __builtin_amdgcn_readfirstlane(base / nchunks);
        const uint32_t b1 = __builtin_amdgcn_readfirstlane(last / nchunks);
        if (b0 == b1) {
            const codec_slice_meta* M = meta + b0;
            const long long lo = M->span_lo, len = M->span_len;
            const long long qbase = (long long)(base - b0 * nchunks) * 8;
            const u64* maps = maps_all + (size_t)b0 * mw;
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const uint32_t g = cb + u * (uint32_t)NTH;
                if (g >= total_chunks) break;
                const long long q0 = qbase + (long long)(threadIdx.x + u * (uint32_t)NTH) * 8;
                if (span_hit(q0, lo, len, npx)) restore_chunk<T>(vv[u], q0, M, maps, npx);
                stv<NT>(dst + g, vv[u]);
            }
        } else {
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const uint32_t g = cb + u * (uint32_t)NTH;
                if (g >= total_chunks) break;
                const uint32_t b = g / nchunks;
                const codec_slice_meta* M = meta + b;
                const long long q0 = (long long)(g - b * nchunks) * 8;
                if (span_hit(q0, M->span_lo, M->span_len, npx))
                    restore_chunk<T>(vv[u], q0, M, maps_all + (size_t)b * mw, npx);
                stv<NT>(dst + g, vv[u]);
            }
        }
    }
}

// Slice-serial variant (batches of at least one slice per CU, small slices: C3's 256 x 512^2):
// one 1024-thread workgroup per slice.  D vectors per thread stay in flight in a register
// ring while the workgroup copies its slice in order -- a pure straight-line copy, so hipcc
// counts vmcnt exactly and never drains the ring -- then fixes up the window hull (rewrites
// the <= a few thousand pixels of span_lo/span_len with their restored values; the copy's
// stores to them completed at the barrier before).  The slice's payload gather runs first,
// its pixel loads behind the ring's.  At C3 the grid-stride pass streams 2048 short-lived
// workgroups (0.073 ms); this keeps one contiguous region per CU, the order this chip copies
// fastest in.
template <typename T, bool NT, int D, int G>
__global__ __launch_bounds__(1024) void k_restore_ss(const T* __restrict__ stego, T* __restrict__ cover, uint32_t npx,
                                                     const codec_slice_meta* __restrict__ meta,
                                                     const u64* __restrict__ maps_all, int mw,
                                                     u64* __restrict__ payload_out, int pw, int gather_late) {
    typedef typename Vec8<T>::type V;
    const int b = blockIdx.x;
    const uint32_t t = threadIdx.x;
    const uint32_t nv = npx / 8;                  // a multiple of 1024 * D * G (host check)
    const V* src = reinterpret_cast<const V*>(stego + (size_t)b * npx);
    V* dst = reinterpret_cast<V*>(cover + (size_t)b * npx);
    V r[D][G];
#pragma unroll
    for (int d = 0; d < D; ++d)
#pragma unroll
        for (int g = 0; g < G; ++g) r[d][g] = ldv<NT>(src + (uint32_t)(d * G + g) * 1024u + t);
    if (payload_out && !gather_late) gather_body<T, 1024>(stego, (long long)npx, meta, payload_out, pw, b);
    const uint32_t step = 1024u * D * G;
    uint32_t base = 0;
    for (; base + step < nv; base += step) {
#pragma unroll
        for (int d = 0; d < D; ++d) {
#pragma unroll
            for (int g = 0; g < G; ++g) {
                const uint32_t idx = base + (uint32_t)(d * G + g) * 1024u + t;
                stv<NT>(dst + idx, r[d][g]);
                r[d][g] = ldv<NT>(src + idx + step);   // refill from the next group
            }
        }
    }
#pragma unroll
    for (int d = 0; d < D; ++d)
#pragma unroll
        for (int g = 0; g < G; ++g) stv<NT>(dst + base + (uint32_t)(d * G + g) * 1024u + t, r[d][g]);
    if (payload_out && gather_late) gather_body<T, 1024>(stego, (long long)npx, meta, payload_out, pw, b);
    __syncthreads();   // waits for every store above (vmcnt(0)) before the hull is rewritten
    const codec_slice_meta* M = meta + b;
    const long long lo = M->span_lo, len = M->span_len;
    if (len > 0) {
        const uint32_t first = (uint32_t)(lo / 8), last = (uint32_t)((lo + len + 7) / 8);
        const u64* maps = maps_all + (size_t)b * mw;
        for (uint32_t i = t; i < last - first; i += 1024u) {
            uint32_t idx = first + i;
            if (idx >= nv) idx -= nv;
            const long long q0 = (long long)idx * 8;
            if (span_hit(q0, lo, len, npx)) {
                V v = src[idx];
                restore_chunk<T>(v, q0, M, maps, npx);
                dst[idx] = v;
            }
        }
    }
}

// Inline variant of k_restore_ss (round 3): the same register-ring copy of one slice per
// 1024-thread workgroup, but the window hull is restored and the payload gathered in the
// stream, from the vectors already in registers: the slice's location map is staged in LDS
// first, a vector inside the hull XORs its map bits back (LDS reads only, so the ring's loads
// and stores stay straight-line and hipcc's vmcnt counting exact) and ORs its payload bits into
// an LDS buffer.  No gather before the copy (its loads queued behind the ring's), no hull
// pass after it (a full vmcnt(0) drain, then a dependent load + store).  Bits as gather_body:
// bit j = stego bit p of the j-th window pixel in segment order, j = cat[p] + (q - off[p]) mod npx.
#define RIL_WORDS 4096   // 32-bit LDS words each for the map and the payload (host-checked)
// LDS-only barriers in the ring loop keep the 16 waves in step: without them the oldest waves
// ran ahead and the slice's tail was streamed by the youngest alone (as in k_pee_embed_ss).
// 2 = one barrier per ring slot (G vectors): C3 restore 0.0519 -> 0.0486 ms
// (profiles/r03/c3_ril_lockstep_ab.log); 1 = per ring group, 3 = per vector, 0 = none
#ifndef RIL_LOCKSTEP
#define RIL_LOCKSTEP 2
#endif
// NTS: the stores' cache policy (default: the loads'): plain stores are ~5 % faster at C3
// (k_restore_il 0.0485 -> 0.0455 ms, profiles/r05/ab_policy_c3.txt)
template <typename T, bool NT, int D, int G, bool NTS = NT>
__global__ __launch_bounds__(1024) void k_restore_il(const T* __restrict__ stego, T* __restrict__ cover, uint32_t npx,
                                                     const codec_slice_meta* __restrict__ meta,
                                                     const u64* __restrict__ maps_all, int mw,
                                                     u64* __restrict__ payload_out, int pw) {
    typedef typename Vec8<T>::type V;
    __shared__ uint32_t s_map[RIL_WORDS], s_pay[RIL_WORDS];
    __shared__ int s_n[16], s_off[16], s_cat[16];
    const int b = blockIdx.x;
    const uint32_t t = threadIdx.x;
    const uint32_t nv = npx / 8;   // a multiple of 1024 * D * G (host check)
    const codec_slice_meta* M = meta + b;
    // the slice's windows and location map first: their loads are ahead of the ring's
    const int s = M->s;
    const uint32_t lo = (uint32_t)M->span_lo, len = (uint32_t)M->span_len;
    if (t < 16) {
        const bool on = (int)t < s;
        s_n[t] = on ? M->n[t] : 0;
        s_off[t] = on ? M->off[t] : 0;
        s_cat[t] = on ? M->cat[t] : 0;
    }
    const u64* maps = maps_all + (size_t)b * mw;
    for (uint32_t w = t; w < (uint32_t)mw; w += 1024u) {
        const u64 m = maps[w];
        s_map[2 * w] = (uint32_t)m;
        s_map[2 * w + 1] = (uint32_t)(m >> 32);
    }
    if (payload_out)
        for (uint32_t w = t; w < 2u * (uint32_t)pw; w += 1024u) s_pay[w] = 0u;
    const V* src = reinterpret_cast<const V*>(stego + (size_t)b * npx);
    V* dst = reinterpret_cast<V*>(cover + (size_t)b * npx);
    V r[D][G];
#pragma unroll
    for (int d = 0; d < D; ++d)
#pragma unroll
        for (int g = 0; g < G; ++g) r[d][g] = ldv<NT>(src + (uint32_t)(d * G + g) * 1024u + t);
    lds_barrier();
    const uint32_t hi = lo + len;   // <= 2 npx - 1 < 2^32
    const bool wrap = len > 0 && hi > npx;
    // a vector (8 pixels from q0) inside the hull: per plane, its in-window pixels form one run
    // [e0, e1) whose bits j0 .. j0 + (e1 - e0) - 1 are consecutive in the map and the payload
    auto fix = [&](V& v, uint32_t q0) {
        uint32_t px[8];
        if constexpr (sizeof(T) == 2) {
            px[0] = v.x & 0xFFFFu; px[1] = v.x >> 16; px[2] = v.y & 0xFFFFu; px[3] = v.y >> 16;
            px[4] = v.z & 0xFFFFu; px[5] = v.z >> 16; px[6] = v.w & 0xFFFFu; px[7] = v.w >> 16;
        } else {
            for (int e = 0; e < 4; ++e) { px[e] = (v.x >> (8 * e)) & 0xFFu; px[4 + e] = (v.y >> (8 * e)) & 0xFFu; }
        }
        for (int p = 0; p < s; ++p) {
            const int n = s_n[p];
            if (n <= 0) continue;
            int i0 = (int)q0 - s_off[p];   // window index of pixel e = i0 + e (mod npx)
            if (i0 < -7) i0 += (int)npx;
            int e0 = 8, e1 = 0;
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                int i = i0 + e;
                if (i < 0) i += (int)npx;
                if (i < n) { e0 = min(e0, e); e1 = e + 1; }
            }
            if (e0 >= e1) continue;
            int ia = i0 + e0;
            if (ia < 0) ia += (int)npx;
            const uint32_t j0 = (uint32_t)(s_cat[p] + ia);
            const uint32_t wd = j0 >> 5, sh = j0 & 31u;
            const uint32_t mf = __builtin_amdgcn_alignbit(s_map[min(wd + 1, (uint32_t)RIL_WORDS - 1)], s_map[wd], sh);
            uint32_t bits = 0;
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                if (e < e0 || e >= e1) continue;
                bits |= ((px[e] >> p) & 1u) << (e - e0);
                px[e] ^= ((mf >> (e - e0)) & 1u) << p;
            }
            if (payload_out && bits) {
                atomicOr(&s_pay[wd], bits << sh);
                if (sh + (uint32_t)(e1 - e0) > 32u) atomicOr(&s_pay[wd + 1], bits >> (32u - sh));
            }
        }
        if constexpr (sizeof(T) == 2) {
            v.x = px[0] | (px[1] << 16); v.y = px[2] | (px[3] << 16);
            v.z = px[4] | (px[5] << 16); v.w = px[6] | (px[7] << 16);
        } else {
            v.x = px[0] | (px[1] << 8) | (px[2] << 16) | (px[3] << 24);
            v.y = px[4] | (px[5] << 8) | (px[6] << 16) | (px[7] << 24);
        }
    };
    auto put = [&](uint32_t idx, V& v) {
        const uint32_t q0 = idx * 8u;
        if (len > 0 && ((q0 + 8u > lo && q0 < hi) || (wrap && q0 < hi - npx))) fix(v, q0);
        stv<NTS>(dst + idx, v);
    };
    const uint32_t step = 1024u * D * G;
    uint32_t base = 0;
    for (; base + step < nv; base += step) {
#pragma unroll
        for (int d = 0; d < D; ++d) {
#pragma unroll
            for (int g = 0; g < G; ++g) {
                const uint32_t idx = base + (uint32_t)(d * G + g) * 1024u + t;
                put(idx, r[d][g]);
                r[d][g] = ldv<NT>(src + idx + step);   // refill from the next group
#if RIL_LOCKSTEP == 3
                lds_barrier();
#endif
            }
#if RIL_LOCKSTEP == 1 || RIL_LOCKSTEP == 2
            if (RIL_LOCKSTEP == 2 || d == D - 1) lds_barrier();
#endif
        }
    }
#pragma unroll
    for (int d = 0; d < D; ++d)
#pragma unroll
        for (int g = 0; g < G; ++g) put(base + (uint32_t)(d * G + g) * 1024u + t, r[d][g]);
    if (payload_out) {
        lds_barrier();   // every payload OR done
        for (uint32_t w = t; w < (uint32_t)pw; w += 1024u)
            payload_out[(size_t)b * pw + w] = (u64)s_pay[2 * w] | ((u64)s_pay[2 * w + 1] << 32);
    }
}

// scalar variant for slices whose rows are not 8-pixel aligned
template <typename T>
__global__ __launch_bounds__(256) void k_restore_scalar(const T* __restrict__ stego, T* __restrict__ cover,
                                                        long long npx, const codec_slice_meta* __restrict__ meta,
                                                        const u64* __restrict__ maps_all, int mw) {
    __shared__ SliceWin W;
    __shared__ Range rg[32];
    __shared__ int nrg;
    const int b = blockIdx.y;
    load_win(meta + b, &W);
    if (threadIdx.x == 0) nrg = build_ranges(W, rg);
    __syncthreads();
    const u64* maps = maps_all + (size_t)b * mw;
    const long long stride = (long long)gridDim.x * 256;
    for (long long q = (long long)blockIdx.x * 256 + threadIdx.x; q < npx; q += stride) {
        uint32_t px = stego[(size_t)b * npx + q];
        for (int k = 0; k < nrg; ++k) {
            const Range r = rg[k];
            if (q >= r.q0 && q < r.q1) px ^= map_bit(maps, r.j0 + (q - r.q0)) << r.p;
        }
        cover[(size_t)b * npx + q] = (T)px;
    }
}

// payload bits in segment order: bit j = stego bit p at the j-th window pixel
// payload bits back out of the windows: one 1024-thread workgroup per slice, 8 bits per
// thread per round with all loads issued first; every payload word is written (zeros past
// total_used), so the caller needs no memset
// payload bits of slice b back out of its windows (ballot-packed, 8 loads in flight per
// thread per round); NTH threads.  Used by k_gather and as the leading workgroups of
// k_restore_gs (codec_extract out of place: the two read the stego independently)
template <typename T, int NTH>
__device__ __forceinline__ void gather_body(const T* __restrict__ stego, long long npx,
                                            const codec_slice_meta* __restrict__ meta,
                                            u64* __restrict__ out, int pw, int b) {
    __shared__ SliceWin W;
    __shared__ int seg_p[16], seg_q0[16];
    load_win(meta + b, &W);
    int ends[16];
    win_segments(W, seg_p, seg_q0, ends);
    const T* sv = stego + (size_t)b * npx;
    const int t = threadIdx.x;
    for (int j0 = 0; j0 < pw * 64; j0 += 8 * NTH) {
        uint32_t v[8];
        int pl[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const int j = j0 + k * NTH + t;
            pl[k] = -1;
            v[k] = 0;
            if (j < W.tot) {
                int sg = 0;
#pragma unroll
                for (int kk = 0; kk < 16; ++kk) sg += j >= ends[kk] ? 1 : 0;
                long long q = (long long)seg_q0[sg] + j;
                if (q >= npx) q -= npx;
                pl[k] = seg_p[sg];
                v[k] = sv[q];
            }
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            if (j0 + k * NTH >= pw * 64) break;                  // uniform
            const int j = j0 + k * NTH + t;
            const u64 bal = __ballot(pl[k] >= 0 ? (v[k] >> pl[k]) & 1u : 0u);
            if ((t & 63) == 0 && (j >> 6) < pw) out[(size_t)b * pw + (j >> 6)] = bal;
        }
    }
}

template <typename T>
__global__ __launch_bounds__(1024) void k_gather(const T* __restrict__ stego, long long npx,
                                                 const codec_slice_meta* __restrict__ meta,
                                                 u64* __restrict__ out, int pw) {
    gather_body<T, 1024>(stego, npx, meta, out, pw, blockIdx.x);
}

// in-place restore: XOR every window bit with its location-map bit (only the <= T window
// pixels are touched; 32-bit atomics because windows of different planes may share a pixel)
template <typename T>
__global__ __launch_bounds__(256) void k_unxor(T* img, long long npx, const codec_slice_meta* __restrict__ meta,
                                               const u64* __restrict__ maps_all, int mw) {
    __shared__ SliceWin W;
    const int b = blockIdx.y;
    load_win(meta + b, &W);
    const int j = blockIdx.x * 256 + threadIdx.x;
    if (j >= W.tot || !map_bit(maps_all + (size_t)b * mw, j)) return;
    const int p = plane_of(W, j);
    const int i = j - W.cat[p];
    long long q = (long long)W.off[p] + i;
    if (q >= npx) q -= npx;
    if (!(W.flags & CODEC_FLAG_OVERLAP)) {   // every window pixel has one owner: plain RMW
        T* px = img + (size_t)b * npx + q;
        *px = (T)(*px ^ (1u << p));
        return;
    }
    const size_t byte = ((size_t)b * npx + q) * sizeof(T);
    uint32_t* word = reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(img) + (byte & ~(size_t)3));
    atomicXor(word, 1u << ((byte & 3) * 8 + p));
}

// ------------------------------------------------------------------ K6: reference decode
// python `seq[:k]` length for a sequence of length `count`
__device__ __forceinline__ int pyslice_take(int count, int k) {
    if (k >= 0) return min(count, k);
    return max(0, count + k);
}

// decode_message (codec.py:752-787) from packed maps: one workgroup per slice
template <typename T>
__global__ __launch_bounds__(256) void k_refdecode(const T* __restrict__ stego, long long npx,
                                                   const codec_slice_meta* __restrict__ meta,
                                                   const u64* __restrict__ maps_all, int mw,
                                                   uint8_t* __restrict__ out_all, int cap,
                                                   int32_t* __restrict__ counts) {
    __shared__ SliceWin W;
    __shared__ uint32_t sh[8];
    const int b = blockIdx.x;
    load_win(meta + b, &W);
    const u64* maps = maps_all + (size_t)b * mw;
    uint8_t* out = out_all + (size_t)b * cap;
    const T* img = stego + (size_t)b * npx;
    int outpos = 0;
    for (int p = 0; p < W.s; ++p) {                        // plane-index order (codec.py:776)
        const int n = W.n[p];
        uint32_t local = 0;
        for (int i = threadIdx.x; i < n; i += 256) local += map_bit(maps, (long long)W.cat[p] + i);
        const uint32_t count = block_sum_u32<256>(local, sh);
        const int K = pyslice_take((int)count, W.sizes[p]);   // [:segments_lengths[p]]
        const int rs = ((long long)W.off[p] + n > npx) ? (int)(npx - W.off[p]) : 0;
        uint32_t running = 0;
        for (int base = 0; base < n && (int)running < K; base += 256) {
            const int r = base + threadIdx.x;
            uint32_t bit = 0;
            int i = 0;
            if (r < n) {
                i = r + rs;
                if (i >= n) i -= n;
                bit = map_bit(maps, (long long)W.cat[p] + i);
            }
            uint32_t tot;
            const uint32_t rank = running + block_excl_scan<256>(bit, sh, &tot);
            if (bit && (int)rank < K && outpos + (int)rank < cap) {
                long long q = (long long)W.off[p] + i;
                if (q >= npx) q -= npx;
                out[outpos + rank] = (uint8_t)((img[q] >> p) & 1u);
            }
            running += tot;
        }
        outpos += K;
    }
    if (threadIdx.x == 0) counts[b] = outpos;
}

// dense variant, phase A: non-zero count per (slice, plane)
__global__ __launch_bounds__(1024) void k_dense_count(const uint8_t* __restrict__ dense, int smax, long long npx,
                                                      const codec_slice_meta* __restrict__ meta,
                                                      int32_t* __restrict__ nzcount) {
    __shared__ uint32_t sh[20];
    const int p = blockIdx.x, b = blockIdx.y;
    if (p >= meta[b].s) return;
    const uint8_t* d = dense + ((size_t)b * smax + p) * npx;
    uint32_t local = 0;
    for (long long q = threadIdx.x; q < npx; q += 1024) local += d[q] != 0;
    const uint32_t tot = block_sum_u32<1024>(local, sh);
    if (threadIdx.x == 0) nzcount[b * 16 + p] = (int32_t)tot;
}

// dense variant, phase B: ordered compaction of the first K non-zero positions
template <typename T>
__global__ __launch_bounds__(1024) void k_dense_emit(const T* __restrict__ src, int src_is_planes,
                                                     const uint8_t* __restrict__ dense, int smax, long long npx,
                                                     const codec_slice_meta* __restrict__ meta,
                                                     const int32_t* __restrict__ nzcount,
                                                     uint8_t* __restrict__ out_all, int cap,
                                                     int32_t* __restrict__ counts) {
    __shared__ uint32_t sh[20];
    const int p = blockIdx.x, b = blockIdx.y;
    const codec_slice_meta* M = meta + b;
    const int s = M->s;
    if (p >= s) return;
    int outpos = 0, K = 0, total = 0;
    for (int pp = 0; pp < s; ++pp) {
        const int k = pyslice_take(nzcount[b * 16 + pp], M->sizes[pp]);
        if (pp < p) outpos += k;
        if (pp == p) K = k;
        total += k;
    }
    if (p == s - 1 && threadIdx.x == 0) counts[b] = total;
    const uint8_t* d = dense + ((size_t)b * smax + p) * npx;
    uint8_t* out = out_all + (size_t)b * cap;
    uint32_t running = 0;
    for (long long base = 0; base < npx && (int)running < K; base += 1024) {
        const long long q = base + threadIdx.x;
        const uint32_t bit = (q < npx && d[q] != 0) ? 1u : 0u;
        uint32_t tot;
        const uint32_t rank = running + block_excl_scan<1024>(bit, sh, &tot);
        if (bit && (int)rank < K && outpos + (int)rank < cap) {
            uint32_t v;
            if (src_is_planes) v = src[((size_t)b * smax + p) * npx + q] & 1u;
            else v = (src[(size_t)b * npx + q] >> p) & 1u;
            out[outpos + rank] = (uint8_t)v;
        }
        running += tot;
    }
}

// ------------------------------------------------------------------ K7: dense helpers
__global__ __launch_bounds__(256) void k_expand(const u64* __restrict__ maps_all, int mw,
                                                const codec_slice_meta* __restrict__ meta,
                                                uint8_t* __restrict__ dense, int smax, long long npx) {
    __shared__ SliceWin W;
    __shared__ Range rg[32];
    __shared__ int nrg;
    const int p = blockIdx.y, b = blockIdx.z;
    load_win(meta + b, &W);
    if (threadIdx.x == 0) {
        Range all[32];
        const int k = build_ranges(W, all);
        int c = 0;
        for (int i = 0; i < k; ++i)
            if (all[i].p == p) rg[c++] = all[i];
        nrg = c;
    }
    __syncthreads();
    const u64* maps = maps_all + (size_t)b * mw;
    uint8_t* d = dense + ((size_t)b * smax + p) * npx;
    const long long stride = (long long)gridDim.x * 256;
    for (long long q = (long long)blockIdx.x * 256 + threadIdx.x; q < npx; q += stride) {
        uint8_t v = 0;
        if (p < W.s) {
            for (int k = 0; k < nrg; ++k)
                if (q >= rg[k].q0 && q < rg[k].q1) v = (uint8_t)map_bit(maps, rg[k].j0 + (q - rg[k].q0));
        }
        d[q] = v;
    }
}

template <typename T>
__global__ __launch_bounds__(256) void k_restore_dense(const T* __restrict__ stego, const uint8_t* __restrict__ dense,
                                                       int smax, long long npx,
                                                       const codec_slice_meta* __restrict__ meta,
                                                       T* __restrict__ cover) {
    const int b = blockIdx.y;
    const int s = meta[b].s;
    const long long stride = (long long)gridDim.x * 256;
    for (long long q = (long long)blockIdx.x * 256 + threadIdx.x; q < npx; q += stride) {
        uint32_t v = stego[(size_t)b * npx + q];
        for (int p = 0; p < s; ++p) v ^= (uint32_t)(dense[((size_t)b * smax + p) * npx + q] & 1u) << p;
        cover[(size_t)b * npx + q] = (T)v;
    }
}

template <typename Tin, typename Tout>
__global__ __launch_bounds__(256) void k_unpack(const Tin* __restrict__ img, long long npx, int first, int count,
                                                Tout* __restrict__ planes) {
    const int b = blockIdx.y;
    const long long stride = (long long)gridDim.x * 256;
    for (long long q = (long long)blockIdx.x * 256 + threadIdx.x; q < npx; q += stride) {
        const uint32_t v = img[(size_t)b * npx + q];
        for (int k = 0; k < count; ++k) {
            const int sh = first + k;
            planes[((size_t)b * count + k) * npx + q] = (Tout)(sh < 32 ? (v >> sh) & 1u : 0u);
        }
    }
}

template <typename Tp, typename Tout>
__global__ __launch_bounds__(256) void k_merge(const Tp* __restrict__ planes, int nplanes, long long npx,
                                               Tout* __restrict__ out) {
    const int b = blockIdx.y;
    const long long stride = (long long)gridDim.x * 256;
    for (long long q = (long long)blockIdx.x * 256 + threadIdx.x; q < npx; q += stride) {
        uint32_t acc = 0;
        for (int k = 0; k < nplanes && k < 8 * (int)sizeof(Tout); ++k) {
            const uint32_t pv = (Tout)planes[((size_t)b * nplanes + k) * npx + q];
            acc |= (uint32_t)(Tout)(pv << k);
        }
        out[(size_t)b * npx + q] = (Tout)acc;
    }
}

// ====================================================================== host side


static int check_params(const codec_params* P) {
    if (!P) return set_err(CODEC_EINVAL, "params is NULL");
    if (P->B < 1 || P->H < 1 || P->W < 1) return set_err(CODEC_EINVAL, "bad shape B=%d H=%d W=%d", P->B, P->H, P->W);
    if ((long long)P->H * P->W > 0x7FFFFFFFLL) return set_err(CODEC_EINVAL, "H*W must fit int32");
    if (P->in_bytes != 1 && P->in_bytes != 2) return set_err(CODEC_EINVAL, "in_bytes must be 1 or 2");
    if (P->out_bytes != 1 && P->out_bytes != 2) return set_err(CODEC_EINVAL, "out_bytes must be 1 or 2");
    if (P->nbits < 1 || P->nbits > 16) return set_err(CODEC_EINVAL, "nbits must be in 1..16");
    if (P->block < 1) return set_err(CODEC_EINVAL, "block must be >= 1");
    if (P->mode != CODEC_MODE_HYBRID && P->mode != CODEC_MODE_MULTI) return set_err(CODEC_EINVAL, "bad mode");
    if (P->fixed_s > 16) return set_err(CODEC_EINVAL, "fixed_s must be <= 16");
    if (P->fixed_offset >= 0 && (long long)P->fixed_offset >= (long long)P->H * P->W)
        return set_err(CODEC_EINVAL, "fixed_offset out of range");
    return 0;
}


static bool pow2_fast_block(int b) { return b == 8 || b == 16 || b == 32 || b == 64; }

static bool use_fast_scan(const codec_params* P, const void* cover, const void* stego) {
    const size_t va = P->in_bytes == 2 ? 16 : 8;
    return (P->W % 8) == 0 && pow2_fast_block(P->block) && P->in_bytes == P->out_bytes &&
           P->nbits >= 8 * P->in_bytes && ((uintptr_t)cover % va) == 0 && ((uintptr_t)stego % va) == 0;
}

static int host_exact_count(const codec_params* P, bool edge_only) {
    const int sb = P->block;
    const int nby = (P->H + sb - 1) / sb, nbx = (P->W + sb - 1) / sb;
    if (!edge_only) return nby * nbx;
    const int ncol = (P->W % sb) ? nby : 0;
    const int nrow = (P->H % sb) ? (nbx - ((P->W % sb) ? 1 : 0)) : 0;
    return ncol + nrow;
}

struct WsLayout {
    size_t hist, keys, orv, slots, exact, terms, total;
    int exact_cap;
};

static WsLayout ws_layout(const codec_params* P) {
    WsLayout L;
    const size_t R = P->in_bytes == 2 ? 65536 : 256;
    // capacity for the worst case (generic path: every block exact)
    const int cap = host_exact_count(P, false);
    L.exact_cap = cap > 0 ? cap : 1;
    L.hist = 0;
    L.keys = align_up(L.hist + (size_t)P->B * R * 4, 256);
    L.orv = align_up(L.keys + (size_t)P->B * 8, 256);
    L.slots = align_up(L.orv + (size_t)P->B * 4, 256);      // split decision: 16 u64 per slice
    L.exact = align_up(L.slots + (size_t)P->B * 16 * 8, 256);  // [0, exact) is zeroed on errors
    L.terms = align_up(L.exact + (size_t)P->B * L.exact_cap * 8, 256);
    L.total = align_up(L.terms + (size_t)P->B * R * 8, 256);
    return L;
}

extern "C" {

int codec_abi_version(void) { return CODEC_ABI_VERSION; }
int codec_set_tuning(int32_t on) { return g_tuning.exchange(on ? 1 : 0); }

int codec_profile_begin(int32_t capacity) {
    if (g_prof.ev) return set_err(CODEC_EINVAL, "profile window already open");
    if (capacity < 1 || capacity > (1 << 20)) return set_err(CODEC_EINVAL, "capacity must be in 1..2^20");
    hipEvent_t* ev = new hipEvent_t[2 * (size_t)capacity];
    for (int i = 0; i < 2 * capacity; ++i) {
        const hipError_t e = hipEventCreate(&ev[i]);
        if (e != hipSuccess) {   // leave no half-open window behind (the next begin must work)
            for (int j = 0; j < i; ++j) (void)hipEventDestroy(ev[j]);
            delete[] ev;
            return set_err(-(int)e, "hipEventCreate: %s", hipGetErrorString(e));
        }
    }
    g_prof.ev = ev;
    g_prof.tag = new int32_t[capacity];
    g_prof.cap = capacity;
    g_prof.n = 0;
    return 0;
}

int codec_profile_end(float* ms, int32_t* tag, int32_t capacity) {
    if (!g_prof.ev) return set_err(CODEC_EINVAL, "no profile window open");
    const int n = g_prof.n < capacity ? g_prof.n : (capacity > 0 ? capacity : 0);
    int rc = 0;
    for (int i = 0; i < n; ++i) {
        float t = 0.f;
        hipError_t e = hipEventElapsedTime(&t, g_prof.ev[2 * i], g_prof.ev[2 * i + 1]);
        if (e != hipSuccess && rc == 0) rc = set_err(-(int)e, "hipEventElapsedTime: %s", hipGetErrorString(e));
        if (ms) ms[i] = t;
        if (tag) tag[i] = g_prof.tag[i];
    }
    for (int i = 0; i < 2 * g_prof.cap; ++i) (void)hipEventDestroy(g_prof.ev[i]);
    delete[] g_prof.ev;
    delete[] g_prof.tag;
    g_prof = ProfWin();
    return rc ? rc : n;
}

const char* codec_last_error(void) { return g_err; }

size_t codec_workspace_bytes(const codec_params* P) {
    if (check_params(P)) return 0;
    return ws_layout(P).total;
}

}  // extern "C"

template <typename T>
static int launch_scan_fast(const codec_params* P, const void* cover, void* stego, uint32_t* hist, u64* keys,
                            uint32_t* orv, hipStream_t st) {
    const int sb = P->block;
    const int nb = (P->H + sb - 1) / sb;
    // workgroups per slice: enough to fill the CUs for small batches, and about one per
    // 2 MiB of slice otherwise (each workgroup zeroes and flushes a 128 KiB LDS histogram,
    // so small regions cost more than they stream: measured 256 x 512^2 0.066 ms at one
    // workgroup per slice vs 0.108 at four; 256 x 2048^2 best at four)
    const long long slice_bytes = (long long)P->H * P->W * sizeof(T);
    // batches under 128 MiB (e.g. 1..8 slices of 2048^2): the band order (1 x 2048^2: 0.020 ms
    // vs 0.032 for the row sweep) with 256 workgroups since the flush reads only the counted
    // range (2 / 4 / 8 x 2048^2: 0.0193 / 0.025 / 0.036 ms vs 0.0205 / 0.029 / 0.046 at 128 and
    // 0.019 / 0.034 / 0.044 at 512, profiles/r03/scan_small_sweep.log; a lone slice has 128 bands)
    const bool small = (long long)P->B * slice_bytes < (128LL << 20);
    const int per_slice = small ? (256 + P->B - 1) / P->B
                                : (int)std::max<long long>((256 + P->B - 1) / P->B, (slice_bytes + (2 << 20) - 1) / (2 << 20));
    const int target = (int)knob("CODEC_SCAN_WGS", (long long)per_slice * P->B);   // tools/tune.py
    const bool nt = knob("CODEC_NT", 1) != 0;
    int wgps = (target + P->B - 1) / P->B;
    // column-band sweep of a batch with fewer bands than the target (a lone 2048^2 slice has
    // 128 bands for 256 CUs): each band's columns are split over csplit workgroups
    // (CODEC_SCAN_CSPLIT; whole block columns per segment)
    const int want = wgps;
    wgps = wgps < 1 ? 1 : (wgps > nb ? nb : wgps);
    const int bpw = (nb + wgps - 1) / wgps;
    wgps = (nb + bpw - 1) / bpw;
    const int gcols = (P->W / 8 + sb / 8 - 1) / (sb / 8);   // block columns (G chunks each)
    // off by default: a lone 2048^2 slice scans slower split (256 workgroups 0.0191 vs 128
    // 0.0167 ms: every workgroup's flush adds to the same slice's words, profiles/r03/c2_csplit.log)
    int csplit = (int)knob("CODEC_SCAN_CSPLIT", 1);
    (void)want;
    csplit = csplit < 1 ? 1 : (csplit > gcols ? gcols : (csplit > 8 ? 8 : csplit));
    dim3 grid(wgps * csplit, P->B);
    const T* c = static_cast<const T*>(cover);
    T* s = static_cast<T*>(stego);
    // the row sweep needs one band's full blocks to fit its LDS counters; wider images
    // (e.g. a flattened 1 x N view) take the column-band sweep
    // Measured (tools/tune.py): the row sweep wins for the copying scan (0.77 vs 0.80-0.83
    // ms at 256 x 2048^2), the column-band sweep for the read-only scan, which is bound by
    // LDS atomic throughput (0.54 vs 0.61 ms: concurrent waves of one band hit the same bins)
    const long long kind = s ? knob("CODEC_SCAN_KIND", small ? 0 : 1) : knob("CODEC_SCAN_READ_KIND", 0);
    if (kind == 1 && P->W / sb <= 2 * SCAN_ROWS_CNT_WORDS) {
        // row-major sweep: bands per workgroup from CODEC_SCAN_ROWS_WGS, capped by the LDS
        // block-counter capacity
        const int fullbx = P->W / sb;
        const int rtarget = s ? (int)knob("CODEC_SCAN_ROWS_WGS", (long long)per_slice * P->B)
                              : (int)knob("CODEC_SCAN_ROWS_READ_WGS", (long long)per_slice * P->B);
        int rw = (rtarget + P->B - 1) / P->B;
        rw = rw < 1 ? 1 : (rw > nb ? nb : rw);
        int rb = (nb + rw - 1) / rw;
        const int cap = 2 * SCAN_ROWS_CNT_WORDS;
        if (fullbx > 0 && rb * fullbx > cap) rb = cap / fullbx;
        rw = (nb + rb - 1) / rb;
        dim3 g2(rw, P->B);
#define ROWS(SBV, ST)                                                                                   \
        hipLaunchKernelGGL((k_scan_rows<T, SBV, true, ST>), g2, dim3(1024), 0, st, c, s, P->H, P->W, rb, hist, keys, orv)
        if (!s) {
            ProfScope prof(st, CODEC_K_SCAN_ROWS_READ);
            switch (sb) { case 8: ROWS(8, false); break; case 16: ROWS(16, false); break;
                          case 32: ROWS(32, false); break; default: ROWS(64, false); break; }
            LAUNCH_CHECK("k_scan_rows(read)");
        } else {
            ProfScope prof(st, CODEC_K_SCAN_ROWS);
            const int diag = (int)knob("CODEC_DIAG_ROWS", 0);   // timing diagnostics only: s is wrong
            if (sb == 16 && diag == 1) hipLaunchKernelGGL((k_scan_rows<T, 16, true, true, 1>), g2, dim3(1024), 0, st, c, s, P->H, P->W, rb, hist, keys, orv);
            else if (sb == 16 && diag == 4) hipLaunchKernelGGL((k_scan_rows<T, 16, true, true, 4>), g2, dim3(1024), 0, st, c, s, P->H, P->W, rb, hist, keys, orv);
            else if (sb == 16 && diag == 5) hipLaunchKernelGGL((k_scan_rows<T, 16, true, true, 5>), g2, dim3(1024), 0, st, c, s, P->H, P->W, rb, hist, keys, orv);
            else switch (sb) { case 8: ROWS(8, true); break; case 16: ROWS(16, true); break;
                          case 32: ROWS(32, true); break; default: ROWS(64, true); break; }
            LAUNCH_CHECK("k_scan_rows");
        }
#undef ROWS
        return 0;
    }
    if (!s) {
        ProfScope prof(st, CODEC_K_SCAN_READ);
        switch (sb) {
            case 8: hipLaunchKernelGGL((k_scan_read<T, 8>), grid, dim3(1024), 0, st, c, P->H, P->W, bpw, hist, keys, orv, csplit); break;
            case 16: hipLaunchKernelGGL((k_scan_read<T, 16>), grid, dim3(1024), 0, st, c, P->H, P->W, bpw, hist, keys, orv, csplit); break;
            case 32: hipLaunchKernelGGL((k_scan_read<T, 32>), grid, dim3(1024), 0, st, c, P->H, P->W, bpw, hist, keys, orv, csplit); break;
            default: hipLaunchKernelGGL((k_scan_read<T, 64>), grid, dim3(1024), 0, st, c, P->H, P->W, bpw, hist, keys, orv, csplit); break;
        }
        LAUNCH_CHECK("k_scan_read");
        return 0;
    }
    // workgroups counting fewer than 65 536 pixels (e.g. a lone 2048^2 slice: one 16-row band
    // each) cannot wrap a 16-bit LDS field: their histogram adds need no return
    const int CRp_ = (P->W / 8 + sb / 8 - 1) / (sb / 8) * (sb / 8);
    const long long seg_cols = (long long)((CRp_ / (sb / 8) + csplit - 1) / csplit) * (sb / 8) * 8;
    const bool noret = sizeof(T) == 2 && (long long)bpw * sb * std::min<long long>(P->W, seg_cols) < 65536 &&
                       knob("CODEC_SCAN_NORET", 1) != 0;
    ProfScope prof(st, CODEC_K_SCAN_FAST);
    switch (sb) {
        case 8: if (nt) hipLaunchKernelGGL((k_scan_fast<T, 8, true>), grid, dim3(1024), 0, st, c, s, P->H, P->W, bpw, hist, keys, orv, csplit);
                else hipLaunchKernelGGL((k_scan_fast<T, 8, false>), grid, dim3(1024), 0, st, c, s, P->H, P->W, bpw, hist, keys, orv, csplit); break;
        case 16: if (knob("CODEC_DIAG_NOHIST", 0)) hipLaunchKernelGGL((k_scan_fast<T, 16, true, false>), grid, dim3(1024), 0, st, c, s, P->H, P->W, bpw, hist, keys, orv, csplit);   // timing diagnostics only: s is wrong
                else if (nt && noret) hipLaunchKernelGGL((k_scan_fast<T, 16, true, true, true>), grid, dim3(1024), 0, st, c, s, P->H, P->W, bpw, hist, keys, orv, csplit);
                else if (nt) hipLaunchKernelGGL((k_scan_fast<T, 16, true>), grid, dim3(1024), 0, st, c, s, P->H, P->W, bpw, hist, keys, orv, csplit);
                else hipLaunchKernelGGL((k_scan_fast<T, 16, false>), grid, dim3(1024), 0, st, c, s, P->H, P->W, bpw, hist, keys, orv, csplit); break;
        case 32: if (nt) hipLaunchKernelGGL((k_scan_fast<T, 32, true>), grid, dim3(1024), 0, st, c, s, P->H, P->W, bpw, hist, keys, orv, csplit);
                else hipLaunchKernelGGL((k_scan_fast<T, 32, false>), grid, dim3(1024), 0, st, c, s, P->H, P->W, bpw, hist, keys, orv, csplit); break;
        default: if (nt) hipLaunchKernelGGL((k_scan_fast<T, 64, true>), grid, dim3(1024), 0, st, c, s, P->H, P->W, bpw, hist, keys, orv, csplit);
                 else hipLaunchKernelGGL((k_scan_fast<T, 64, false>), grid, dim3(1024), 0, st, c, s, P->H, P->W, bpw, hist, keys, orv, csplit); break;
    }
    LAUNCH_CHECK("k_scan_fast");
    return 0;
}

template <typename Tin, typename Tout>
static int launch_scan_generic(const codec_params* P, const void* cover, void* stego, uint32_t* hist, uint32_t* orv,
                               hipStream_t st) {
    const long long npx = (long long)P->H * P->W;
    const int target = sizeof(Tin) == 2 ? 256 : 1024;
    long long wgps = (target + P->B - 1) / P->B;
    long long per = (npx + wgps - 1) / wgps;
    if (per < 4096) per = 4096;
    wgps = (npx + per - 1) / per;
    const uint32_t keep = P->nbits >= 32 ? 0xFFFFFFFFu : ((1u << P->nbits) - 1u);
    ProfScope prof(st, CODEC_K_SCAN_GENERIC);
    hipLaunchKernelGGL((k_scan_generic<Tin, Tout>), dim3((unsigned)wgps, P->B), dim3(1024), 0, st,
                       static_cast<const Tin*>(cover), static_cast<Tout*>(stego), npx, per, keep, hist, orv);
    LAUNCH_CHECK("k_scan_generic");
    return 0;
}

// codec_params.reserved bits of the decision's A/B knobs: 1 block-sequential path
// (CODEC_DECIDE_WAVES=0), 2 no walk path (CODEC_DECIDE_WALK=0), 4 one wave per plane
// (CODEC_DECIDE_PAIRS=0), 8 no guard-banded decision: the numpy-order sums always decide
// (CODEC_DECIDE_EXACT=1)
static int decide_reserved() {
    return (knob("CODEC_DECIDE_WAVES", 1) ? 0 : 1) | (knob("CODEC_DECIDE_WALK", 1) ? 0 : 2) |
           (knob("CODEC_DECIDE_PAIRS", 1) ? 0 : 4) | (knob("CODEC_DECIDE_EXACT", 0) ? 8 : 0);
}

// codec_plan's body; E != nullptr: codec_encode's fused path (k_decide embeds the payload)
static int plan_impl(const codec_params* P, const void* cover, void* stego, const double* log2_lut, int64_t lut_len,
                     const codec_layout* table, const int32_t* slice_class, codec_slice_meta* meta, void* workspace,
                     size_t workspace_bytes, void* stream, const EmbedArgs* E) {
    int rc = check_params(P);
    if (rc) return rc;
    if (!cover || !log2_lut || !table || !slice_class || !meta || !workspace)
        return set_err(CODEC_EINVAL, "codec_plan: NULL pointer argument");
    const WsLayout L = ws_layout(P);
    if (workspace_bytes < L.total) return set_err(CODEC_EINVAL, "workspace too small (%zu < %zu)", workspace_bytes, L.total);
    if (lut_len < (int64_t)P->H * P->W) return set_err(CODEC_EINVAL, "log2 table shorter than H*W");
    if (P->n_classes < 1) return set_err(CODEC_EINVAL, "n_classes must be >= 1");
    hipStream_t st = as_stream(stream);
    char* ws = static_cast<char*>(workspace);
    uint32_t* hist = reinterpret_cast<uint32_t*>(ws + L.hist);
    u64* keys = reinterpret_cast<u64*>(ws + L.keys);
    uint32_t* orv = reinterpret_cast<uint32_t*>(ws + L.orv);
    double* exact = reinterpret_cast<double*>(ws + L.exact);
    double* terms = reinterpret_cast<double*>(ws + L.terms);
    // histograms, block keys, OR words: zero on entry.  The caller zero-initialises the
    // workspace once and k_decide clears what it consumed, so no per-call memset
    // (CODEC_HIST_MEMSET=1 restores it); an error after the scan re-clears it below.
    if (knob("CODEC_HIST_MEMSET", 0)) HIP_TRY(hipMemsetAsync(ws, 0, L.exact, st));
    auto reclear = [&](int err) {
        (void)hipMemsetAsync(ws, 0, L.exact, st);
        return err;
    };

    if (stego == cover && P->in_bytes != P->out_bytes)
        return set_err(CODEC_EINVAL, "codec_plan: in place (stego == cover) needs one pixel dtype");
    const bool fast = use_fast_scan(P, cover, stego ? stego : cover);
    const bool need_blocks0 = P->mode == CODEC_MODE_HYBRID && P->fixed_offset < 0;
    // fused scan + decide (k_scan_decide): codec_encode out of place, uint16, 16x16 blocks, a
    // chip-filling batch (or CODEC_FUSED_DECIDE=2) whose slices' block counters fit one scan
    // workgroup and need no exact edge blocks
    {
        const long long fk = knob("CODEC_FUSED_DECIDE", 1);
        const int nbands = (P->H + 15) / 16;
        const bool shape_ok = E && fast && stego && stego != cover && P->in_bytes == 2 && P->out_bytes == 2 &&
                              P->block == 16 && (long long)nbands * (P->W / 16) <= 2LL * SCAN_ROWS_CNT_WORDS &&
                              (!need_blocks0 || host_exact_count(P, true) == 0);
        if (fk != 0 && shape_ok && (fk == 2 || (long long)P->B >= device_cu_count())) {
            codec_params Pv = *P;
            Pv.reserved = decide_reserved();
            ProfScope prof(st, CODEC_K_SCAN_DECIDE);
            const bool nt = knob("CODEC_NT", 1) != 0;
#define SD(NTV) hipLaunchKernelGGL((k_scan_decide<uint16_t, 16, NTV>), dim3(1, P->B), dim3(1024), 0, st, \
                static_cast<const uint16_t*>(cover), static_cast<uint16_t*>(stego), nbands, Pv, hist, orv, terms, keys, \
                exact, L.exact_cap, 1, log2_lut, (long long)lut_len, table, slice_class, meta, *E)
            if (nt) SD(true); else SD(false);
#undef SD
            const hipError_t ef = hipGetLastError();
            if (ef != hipSuccess) return reclear(set_err(-(int)ef, "launch k_scan_decide: %s", hipGetErrorString(ef)));
            return 0;
        }
    }
    if (fast) {
        // in place the stego copy is the cover itself: the scan only reads
        void* sdst = stego == cover ? nullptr : stego;
        rc = P->in_bytes == 2 ? launch_scan_fast<uint16_t>(P, cover, sdst, hist, keys, orv, st)
                              : launch_scan_fast<uint8_t>(P, cover, sdst, hist, keys, orv, st);
    } else if (P->in_bytes == 2) {
        rc = P->out_bytes == 2 ? launch_scan_generic<uint16_t, uint16_t>(P, cover, stego, hist, orv, st)
                               : launch_scan_generic<uint16_t, uint8_t>(P, cover, stego, hist, orv, st);
    } else {
        rc = P->out_bytes == 2 ? launch_scan_generic<uint8_t, uint16_t>(P, cover, stego, hist, orv, st)
                               : launch_scan_generic<uint8_t, uint8_t>(P, cover, stego, hist, orv, st);
    }
    if (rc) return reclear(rc);

    const bool need_blocks = P->mode == CODEC_MODE_HYBRID && P->fixed_offset < 0;
    const int edge_only = fast ? 1 : 0;
    const int ecount = need_blocks ? host_exact_count(P, fast) : 0;
    if (ecount > 0) {
        dim3 grid((ecount + 255) / 256, P->B);
        ProfScope prof(st, CODEC_K_BLOCK_EXACT);
        if (P->in_bytes == 2)
            hipLaunchKernelGGL(k_block_exact<uint16_t>, grid, dim3(256), 0, st, static_cast<const uint16_t*>(cover),
                               P->H, P->W, P->block, edge_only, exact, L.exact_cap);
        else
            hipLaunchKernelGGL(k_block_exact<uint8_t>, grid, dim3(256), 0, st, static_cast<const uint8_t*>(cover),
                               P->H, P->W, P->block, edge_only, exact, L.exact_cap);
        const hipError_t e1 = hipGetLastError();
        if (e1 != hipSuccess) return reclear(set_err(-(int)e1, "launch k_block_exact: %s", hipGetErrorString(e1)));
    }
    codec_params Pv = *P;
    // bit 0: force the block-sequential decision; bit 1: no walk path for wide slices
    Pv.reserved = decide_reserved();
    // small batches asking for every plane's exact MI (all_mi): the per-plane joint entropies
    // go to plane workgroups on otherwise idle CUs (1 + nb workgroups per slice, all
    // co-resident: at most 240 of them, one per CU).  Without all_mi the guard-banded decision
    // settles nearly every slice without the joint sums, and the rare slice inside the guard
    // band runs them on its own workgroup's waves; CODEC_DECIDE_SPLIT=2 splits anyway (tests),
    // 0 never.
    const int nbp = P->nbits < 16 ? P->nbits : 16;
    const long long split_knob = knob("CODEC_DECIDE_SPLIT", 1);
    const bool want_split = split_knob == 2 ? (P->fixed_s <= 0 || P->all_mi) : (split_knob != 0 && P->all_mi);
    const int nsplit = (want_split && (long long)P->B * (1 + nbp) <= 240) ? nbp : 0;
    u64* slots = reinterpret_cast<u64*>(ws + L.slots);
    // bound of the main workgroup's wait for each plane slot (polls of ~0.1 us); the plane
    // workgroups are co-resident by construction, so it only trips on a broken launch --
    // CODEC_DECIDE_SPINS / CODEC_DECIDE_DEBUG_LATE=i+1 (plane i of slice 0 publishes only
    // after the main workgroup gave up) exist to test that path
    const uint32_t spin_max = (uint32_t)debug_knob("CODEC_DECIDE_SPINS", 1 << 24);
    const int dbg_late = (int)debug_knob("CODEC_DECIDE_DEBUG_LATE", 0) - 1;
    ProfScope prof(st, E ? CODEC_K_DECIDE_EMBED : CODEC_K_DECIDE);
    const EmbedArgs Ev = E ? *E : EmbedArgs{nullptr, nullptr, nullptr, nullptr, 0, 0, 0};
    // lean instantiation (no wave-parallel exact rounds, no walk path: fewer registers, no
    // spills) where the guard band decides -- every call without all_mi / fixed_s / a split
    const bool lean = nsplit == 0 && P->fixed_s <= 0 && !P->all_mi && !(Pv.reserved & 8) && knob("CODEC_DECIDE_LEAN", 1);
#define DEC(TT, EM, LN) hipLaunchKernelGGL((k_decide<TT, EM, LN>), dim3(P->B, 1 + nsplit), dim3(1024), 0, st, Pv, hist, orv, terms, keys, \
                                       exact, L.exact_cap, edge_only, fast ? 1 : 0, log2_lut, (long long)lut_len, table, slice_class, \
                                       meta, Ev, slots, nsplit, spin_max, dbg_late)
    if (P->in_bytes == 2) {
        if (lean) { if (E) DEC(uint16_t, true, true); else DEC(uint16_t, false, true); }
        else { if (E) DEC(uint16_t, true, false); else DEC(uint16_t, false, false); }
    } else {
        if (lean) { if (E) DEC(uint8_t, true, true); else DEC(uint8_t, false, true); }
        else { if (E) DEC(uint8_t, true, false); else DEC(uint8_t, false, false); }
    }
#undef DEC
    const hipError_t e2 = hipGetLastError();
    if (e2 != hipSuccess) return reclear(set_err(-(int)e2, "launch k_decide: %s", hipGetErrorString(e2)));
    return 0;
}

extern "C" {

int codec_plan(const codec_params* P, const void* cover, void* stego, const double* log2_lut, int64_t lut_len,
               const codec_layout* table, const int32_t* slice_class, codec_slice_meta* meta, void* workspace,
               size_t workspace_bytes, void* stream) {
    return plan_impl(P, cover, stego, log2_lut, lut_len, table, slice_class, meta, workspace, workspace_bytes, stream,
                     nullptr);
}

int codec_encode(const codec_params* P, const void* cover, void* stego, const double* log2_lut, int64_t lut_len,
                 const codec_layout* table, const int32_t* slice_class, codec_slice_meta* meta, void* workspace,
                 size_t workspace_bytes, const uint64_t* payload, uint64_t* maps, void* stream) {
    int rc = check_params(P);
    if (rc) return rc;
    if (!stego || !payload || !maps) return set_err(CODEC_EINVAL, "codec_encode: NULL pointer argument");
    if (P->payload_words < 1 || P->map_words < 1) return set_err(CODEC_EINVAL, "payload_words/map_words must be >= 1");
    if ((uintptr_t)stego % 4) return set_err(CODEC_EINVAL, "stego must be 4-byte aligned");
    // fused when stego and cover share a dtype (the decision kernel is typed on it)
    if (P->in_bytes == P->out_bytes && knob("CODEC_FUSED_EMBED", 1) != 0) {
        const EmbedArgs E{cover, stego, reinterpret_cast<const u64*>(payload), reinterpret_cast<u64*>(maps),
                          P->payload_words, P->map_words, (1u << P->nbits) - 1u};
        return plan_impl(P, cover, stego, log2_lut, lut_len, table, slice_class, meta, workspace, workspace_bytes,
                         stream, &E);
    }
    rc = plan_impl(P, cover, stego, log2_lut, lut_len, table, slice_class, meta, workspace, workspace_bytes, stream,
                   nullptr);
    return rc ? rc : codec_embed(P, cover, stego, payload, meta, maps, stream);
}

int codec_embed(const codec_params* P, const void* cover, void* stego, const uint64_t* payload,
                const codec_slice_meta* meta, uint64_t* maps, void* stream) {
    int rc = check_params(P);
    if (rc) return rc;
    if (!cover || !stego || !payload || !meta || !maps) return set_err(CODEC_EINVAL, "codec_embed: NULL pointer argument");
    if (P->payload_words < 1 || P->map_words < 1) return set_err(CODEC_EINVAL, "payload_words/map_words must be >= 1");
    if ((uintptr_t)stego % 4) return set_err(CODEC_EINVAL, "stego must be 4-byte aligned");
    const long long npx = (long long)P->H * P->W;
    // every embedded bit has a map bit: total_used <= map_words*64 (host-sized)
    const long long maxbits = (long long)P->map_words * 64;
    dim3 grid((unsigned)((maxbits + 255) / 256), P->B);
    const uint32_t keep = (1u << P->nbits) - 1u;
    hipStream_t st = as_stream(stream);
    ProfScope prof(st, CODEC_K_EMBED);
#define EMB(TI, TO)                                                                                       \
    hipLaunchKernelGGL((k_embed<TI, TO>), grid, dim3(256), 0, st, static_cast<const TI*>(cover),          \
                       static_cast<TO*>(stego), npx, keep, reinterpret_cast<const u64*>(payload), P->payload_words, meta, reinterpret_cast<u64*>(maps), P->map_words)
    if (P->in_bytes == 2 && P->out_bytes == 2) EMB(uint16_t, uint16_t);
    else if (P->in_bytes == 2) EMB(uint16_t, uint8_t);
    else if (P->out_bytes == 2) EMB(uint8_t, uint16_t);
    else EMB(uint8_t, uint8_t);
#undef EMB
    LAUNCH_CHECK("k_embed");
    return 0;
}

int codec_extract(const codec_params* P, const void* stego, const uint64_t* maps, const codec_slice_meta* meta,
                  void* cover_out, uint64_t* payload_out, void* stream) {
    int rc = check_params(P);
    if (rc) return rc;
    if (!stego || !maps || !meta) return set_err(CODEC_EINVAL, "codec_extract: NULL pointer argument");
    if (P->in_bytes != P->out_bytes) return set_err(CODEC_EINVAL, "codec_extract: stego and cover share a dtype");
    const long long npx = (long long)P->H * P->W;
    hipStream_t st = as_stream(stream);
    const bool inplace = cover_out == stego;   // restore only the window pixels, after the gather
    if (payload_out && P->payload_words < 1) return set_err(CODEC_EINVAL, "payload_words must be >= 1");
    bool gathered = false;                     // done by k_restore_gs's leading workgroups
    if (cover_out && !inplace) {
        const size_t va = P->in_bytes == 2 ? 16 : 8;
        if ((uintptr_t)stego % va || (uintptr_t)cover_out % va || ((npx * P->in_bytes) % va)) {
            long long gx = (npx + 255) / 256;
            if (gx > 2048) gx = 2048;
            dim3 grid((unsigned)gx, P->B);
            if (P->in_bytes == 2)
                hipLaunchKernelGGL(k_restore_scalar<uint16_t>, grid, dim3(256), 0, st, static_cast<const uint16_t*>(stego),
                                   static_cast<uint16_t*>(cover_out), npx, meta, reinterpret_cast<const u64*>(maps), P->map_words);
            else
                hipLaunchKernelGGL(k_restore_scalar<uint8_t>, grid, dim3(256), 0, st, static_cast<const uint8_t*>(stego),
                                   static_cast<uint8_t*>(cover_out), npx, meta, reinterpret_cast<const u64*>(maps), P->map_words);
            LAUNCH_CHECK("k_restore_scalar");
        } else {
        const long long nchunks = npx / 8;
        const bool gs = knob("CODEC_RESTORE_GS", 1) != 0 && (npx % 8) == 0 && nchunks * P->B < 0xFFFFFFFFLL;
        // slice-serial (k_restore_ss): CODEC_RESTORE_SS -1 = batches of >= one slice per CU
        // with slices of <= CODEC_RESTORE_SS_MAXPX pixels, 0 = never, 1 = wherever it applies
        const long long ssk = knob("CODEC_RESTORE_SS", -1);
        const int ncu = device_cu_count();
        const bool ss = ssk != 0 && (npx % 65536) == 0 && npx <= 0x7FFFFFFFLL &&
                        (ssk == 1 || (P->B >= ncu && npx <= knob("CODEC_RESTORE_SS_MAXPX", 1 << 20)));
        if (ss) {
            ProfScope prof(st, CODEC_K_RESTORE);
            const bool ntg = knob("CODEC_NT", 1) != 0;
            const u64* mp = reinterpret_cast<const u64*>(maps);
            u64* po = reinterpret_cast<u64*>(payload_out);
            // vectors in flight per thread (A/B knob CODEC_RESTORE_SS_DEPTH: 4, 8 or 16)
            const long long dep = knob("CODEC_RESTORE_SS_DEPTH", 8);
#define RSS(TT, NTV, DD) hipLaunchKernelGGL((k_restore_ss<TT, NTV, DD, 2>), dim3((unsigned)P->B), dim3(1024), 0, st, \
                static_cast<const TT*>(stego), static_cast<TT*>(cover_out), (uint32_t)npx, meta, mp, P->map_words, po, \
                P->payload_words, glate)
            const int glate = (int)knob("CODEC_RESTORE_SS_GLATE", 0);   // payload gather after the copy (A/B)
            // inline hull restore + gather (k_restore_il) where the map and payload fit its LDS
            // buffers; CODEC_RESTORE_IL=0 for the copy-then-hull kernel
            const bool il = knob("CODEC_RESTORE_IL", 1) != 0 && 2LL * P->map_words <= RIL_WORDS &&
                            (!payload_out || 2LL * P->payload_words <= RIL_WORDS) && dep == 8 && !glate;
            // store policy (CODEC_RIL_NTS, default plain: profiles/r05/ab_policy_c3.txt)
            const bool ril_nts = knob("CODEC_RIL_NTS", 0) != 0;
#define RIL(TT, NTV, DD) hipLaunchKernelGGL((k_restore_il<TT, NTV, DD, 2, false>), dim3((unsigned)P->B), dim3(1024), 0, st, \
                static_cast<const TT*>(stego), static_cast<TT*>(cover_out), (uint32_t)npx, meta, mp, P->map_words, po, \
                P->payload_words)
            // vectors in flight per thread (A/B knob CODEC_RESTORE_IL_DEPTH: 4, 8 or 16)
            const long long idep = knob("CODEC_RESTORE_IL_DEPTH", 8);
            if (il) {
                if (P->in_bytes == 2 && ntg && idep == 16 && npx % 131072 == 0) RIL(uint16_t, true, 8);
                else if (P->in_bytes == 2 && ntg && idep == 4 && npx % 32768 == 0) RIL(uint16_t, true, 2);
                else if (P->in_bytes == 2 && ntg && ril_nts)
                    hipLaunchKernelGGL((k_restore_il<uint16_t, true, 4, 2, true>), dim3((unsigned)P->B), dim3(1024), 0, st,
                                       static_cast<const uint16_t*>(stego), static_cast<uint16_t*>(cover_out), (uint32_t)npx, meta,
                                       mp, P->map_words, po, P->payload_words);
                else if (P->in_bytes == 2) { if (ntg) RIL(uint16_t, true, 4); else RIL(uint16_t, false, 4); }
                else { if (ntg) RIL(uint8_t, true, 4); else RIL(uint8_t, false, 4); }
            }
#undef RIL
            else if (P->in_bytes == 2 && ntg && dep == 16 && npx % 131072 == 0) RSS(uint16_t, true, 8);
            else if (P->in_bytes == 2 && ntg && dep == 4 && npx % 32768 == 0) RSS(uint16_t, true, 2);
            else if (P->in_bytes == 2) { if (ntg) RSS(uint16_t, true, 4); else RSS(uint16_t, false, 4); }
            else { if (ntg) RSS(uint8_t, true, 4); else RSS(uint8_t, false, 4); }
#undef RSS
            LAUNCH_CHECK("k_restore_ss");
            gathered = payload_out != nullptr;
        } else if (gs) {
            const bool ntg = knob("CODEC_NT", 1) != 0;
            const long long g = knob("CODEC_RESTORE_GS_WGS", 1 << 30);   // default: one 1024-chunk block per WG
            const uint32_t total = (uint32_t)(nchunks * P->B);
            // measured: 256-thread workgroups stream a 2 GiB batch best (0.74 vs 0.81 ms at 1024),
            // 1024-thread ones a 128 MiB batch (256 x 512^2: 0.068 vs 0.093 ms)
            const long long sweep_bytes = (long long)total * 8 * P->in_bytes;
            const int nth = (int)knob("CODEC_RESTORE_GS_THREADS", sweep_bytes <= (512LL << 20) ? 1024 : 256);
            long long grid = (total + 4LL * nth - 1) / (4LL * nth);
            if (grid > g) grid = g;
            if (grid < 1) grid = 1;
            // payload gather: B leading workgroups of the same launch (CODEC_FUSED_GATHER=0: a
            // separate k_gather launch after the restore)
            const int gw = (payload_out && knob("CODEC_FUSED_GATHER", 1) != 0) ? P->B : 0;
            grid += gw;
            gathered = gw > 0;
            ProfScope prof(st, CODEC_K_RESTORE);
            const u64* mp = reinterpret_cast<const u64*>(maps);
            u64* po = reinterpret_cast<u64*>(payload_out);
#define RGS(TT, NTV) if (nth == 1024) hipLaunchKernelGGL((k_restore_gs<TT, NTV, 1024>), dim3((unsigned)grid), dim3(1024), 0, st, \
                static_cast<const TT*>(stego), static_cast<TT*>(cover_out), (uint32_t)npx, (uint32_t)nchunks, total, meta, mp, P->map_words, \
                gw, po, P->payload_words); \
            else hipLaunchKernelGGL((k_restore_gs<TT, NTV>), dim3((unsigned)grid), dim3(256), 0, st, \
                static_cast<const TT*>(stego), static_cast<TT*>(cover_out), (uint32_t)npx, (uint32_t)nchunks, total, meta, mp, P->map_words, \
                gw, po, P->payload_words)
            if (P->in_bytes == 2) { if (ntg) RGS(uint16_t, true); else RGS(uint16_t, false); }
            else { if (ntg) RGS(uint8_t, true); else RGS(uint8_t, false); }
#undef RGS
            LAUNCH_CHECK("k_restore_gs");
        } else {
        // many small address-ordered workgroups stream best (tools/ubench_stream.hip)
        const long long target = knob("CODEC_RESTORE_WGS", 32768);   // tools/tune.py
        const bool nt = knob("CODEC_NT", 1) != 0;
        long long wgps = (target + P->B - 1) / P->B;
        long long per = (nchunks + wgps - 1) / wgps;
        if (per < 1024) per = 1024;
        wgps = (nchunks + per - 1) / per;
        if (wgps < 1) wgps = 1;
        dim3 grid((unsigned)wgps, P->B);
        ProfScope prof(st, CODEC_K_RESTORE);
        const u64* mp = reinterpret_cast<const u64*>(maps);
        if (P->in_bytes == 2) {
            const uint16_t* sp = static_cast<const uint16_t*>(stego);
            uint16_t* cp = static_cast<uint16_t*>(cover_out);
            if (nt) hipLaunchKernelGGL((k_restore<uint16_t, true>), grid, dim3(256), 0, st, sp, cp, npx, meta, mp, P->map_words, per);
            else hipLaunchKernelGGL((k_restore<uint16_t, false>), grid, dim3(256), 0, st, sp, cp, npx, meta, mp, P->map_words, per);
        } else {
            const uint8_t* sp = static_cast<const uint8_t*>(stego);
            uint8_t* cp = static_cast<uint8_t*>(cover_out);
            if (nt) hipLaunchKernelGGL((k_restore<uint8_t, true>), grid, dim3(256), 0, st, sp, cp, npx, meta, mp, P->map_words, per);
            else hipLaunchKernelGGL((k_restore<uint8_t, false>), grid, dim3(256), 0, st, sp, cp, npx, meta, mp, P->map_words, per);
        }
        }
        LAUNCH_CHECK("k_restore");
        }
    }
    if (payload_out && !gathered) {
        ProfScope prof(st, CODEC_K_GATHER);
        dim3 grid(P->B);
        if (P->in_bytes == 2)
            hipLaunchKernelGGL(k_gather<uint16_t>, grid, dim3(1024), 0, st, static_cast<const uint16_t*>(stego), npx,
                               meta, reinterpret_cast<u64*>(payload_out), P->payload_words);
        else
            hipLaunchKernelGGL(k_gather<uint8_t>, grid, dim3(1024), 0, st, static_cast<const uint8_t*>(stego), npx,
                               meta, reinterpret_cast<u64*>(payload_out), P->payload_words);
        LAUNCH_CHECK("k_gather");
    }
    if (inplace) {
        dim3 grid((unsigned)(((long long)P->map_words * 64 + 255) / 256), P->B);
        ProfScope prof(st, CODEC_K_UNXOR);
        if (P->in_bytes == 2)
            hipLaunchKernelGGL(k_unxor<uint16_t>, grid, dim3(256), 0, st, static_cast<uint16_t*>(cover_out), npx, meta,
                               reinterpret_cast<const u64*>(maps), P->map_words);
        else
            hipLaunchKernelGGL(k_unxor<uint8_t>, grid, dim3(256), 0, st, static_cast<uint8_t*>(cover_out), npx, meta,
                               reinterpret_cast<const u64*>(maps), P->map_words);
        LAUNCH_CHECK("k_unxor");
    }
    return 0;
}

int codec_refdecode(const codec_params* P, const void* stego, const uint64_t* maps, const codec_slice_meta* meta,
                    uint8_t* bits_out, int32_t bits_cap, int32_t* counts_out, void* stream) {
    int rc = check_params(P);
    if (rc) return rc;
    if (!stego || !maps || !meta || !bits_out || !counts_out || bits_cap < 1)
        return set_err(CODEC_EINVAL, "codec_refdecode: bad arguments");
    const long long npx = (long long)P->H * P->W;
    hipStream_t st = as_stream(stream);
    if (P->out_bytes == 2)
        hipLaunchKernelGGL(k_refdecode<uint16_t>, dim3(P->B), dim3(256), 0, st, static_cast<const uint16_t*>(stego), npx,
                           meta, reinterpret_cast<const u64*>(maps), P->map_words, bits_out, bits_cap, counts_out);
    else
        hipLaunchKernelGGL(k_refdecode<uint8_t>, dim3(P->B), dim3(256), 0, st, static_cast<const uint8_t*>(stego), npx,
                           meta, reinterpret_cast<const u64*>(maps), P->map_words, bits_out, bits_cap, counts_out);
    LAUNCH_CHECK("k_refdecode");
    return 0;
}

int codec_refdecode_dense(const codec_params* P, const void* src, int32_t src_is_planes, const uint8_t* dense,
                          int32_t smax, const codec_slice_meta* meta, uint8_t* bits_out, int32_t bits_cap,
                          int32_t* counts_out, void* stream) {
    int rc = check_params(P);
    if (rc) return rc;
    if (!src || !dense || !meta || !bits_out || !counts_out || bits_cap < 1 || smax < 1 || smax > 16)
        return set_err(CODEC_EINVAL, "codec_refdecode_dense: bad arguments");
    const long long npx = (long long)P->H * P->W;
    hipStream_t st = as_stream(stream);
    // counts_out holds B*17 int32: [0,B) bit counts, then B*16 per-plane non-zero counts (scratch)
    int32_t* nz = counts_out + P->B;
    hipLaunchKernelGGL(k_dense_count, dim3(smax, P->B), dim3(1024), 0, st, dense, smax, npx, meta, nz);
    LAUNCH_CHECK("k_dense_count");
    if (P->in_bytes == 2)
        hipLaunchKernelGGL(k_dense_emit<uint16_t>, dim3(smax, P->B), dim3(1024), 0, st, static_cast<const uint16_t*>(src),
                           src_is_planes, dense, smax, npx, meta, nz, bits_out, bits_cap, counts_out);
    else
        hipLaunchKernelGGL(k_dense_emit<uint8_t>, dim3(smax, P->B), dim3(1024), 0, st, static_cast<const uint8_t*>(src),
                           src_is_planes, dense, smax, npx, meta, nz, bits_out, bits_cap, counts_out);
    LAUNCH_CHECK("k_dense_emit");
    return 0;
}

int codec_expand_maps(const codec_params* P, const uint64_t* maps, const codec_slice_meta* meta, uint8_t* dense,
                      int32_t smax, void* stream) {
    int rc = check_params(P);
    if (rc) return rc;
    if (!maps || !meta || !dense || smax < 1 || smax > 16) return set_err(CODEC_EINVAL, "codec_expand_maps: bad arguments");
    const long long npx = (long long)P->H * P->W;
    long long gx = (npx + 255) / 256;
    if (gx > 1024) gx = 1024;
    hipLaunchKernelGGL(k_expand, dim3((unsigned)gx, smax, P->B), dim3(256), 0, as_stream(stream), reinterpret_cast<const u64*>(maps), P->map_words,
                       meta, dense, smax, npx);
    LAUNCH_CHECK("k_expand");
    return 0;
}

int codec_restore_dense(const codec_params* P, const void* stego, const uint8_t* dense, int32_t smax,
                        const codec_slice_meta* meta, void* cover_out, void* stream) {
    int rc = check_params(P);
    if (rc) return rc;
    if (!stego || !dense || !meta || !cover_out || smax < 1 || smax > 16)
        return set_err(CODEC_EINVAL, "codec_restore_dense: bad arguments");
    const long long npx = (long long)P->H * P->W;
    long long gx = (npx + 255) / 256;
    if (gx > 2048) gx = 2048;
    dim3 grid((unsigned)gx, P->B);
    if (P->in_bytes == 2)
        hipLaunchKernelGGL(k_restore_dense<uint16_t>, grid, dim3(256), 0, as_stream(stream),
                           static_cast<const uint16_t*>(stego), dense, smax, npx, meta, static_cast<uint16_t*>(cover_out));
    else
        hipLaunchKernelGGL(k_restore_dense<uint8_t>, grid, dim3(256), 0, as_stream(stream),
                           static_cast<const uint8_t*>(stego), dense, smax, npx, meta, static_cast<uint8_t*>(cover_out));
    LAUNCH_CHECK("k_restore_dense");
    return 0;
}

int codec_unpack_planes(const codec_params* P, const void* img, int32_t first, int32_t count, void* planes,
                        int32_t plane_bytes, void* stream) {
    if (!P || P->B < 1 || P->H < 1 || P->W < 1 || (P->in_bytes != 1 && P->in_bytes != 2))
        return set_err(CODEC_EINVAL, "codec_unpack_planes: bad params");
    if (!img || !planes || first < 0 || count < 1 || (plane_bytes != 1 && plane_bytes != 2))
        return set_err(CODEC_EINVAL, "codec_unpack_planes: bad arguments");
    const long long npx = (long long)P->H * P->W;
    long long gx = (npx + 255) / 256;
    if (gx > 2048) gx = 2048;
    dim3 grid((unsigned)gx, P->B);
    hipStream_t st = as_stream(stream);
#define UNP(TI, TO) hipLaunchKernelGGL((k_unpack<TI, TO>), grid, dim3(256), 0, st, static_cast<const TI*>(img), npx, first, count, static_cast<TO*>(planes))
    if (P->in_bytes == 2 && plane_bytes == 2) UNP(uint16_t, uint16_t);
    else if (P->in_bytes == 2) UNP(uint16_t, uint8_t);
    else if (plane_bytes == 2) UNP(uint8_t, uint16_t);
    else UNP(uint8_t, uint8_t);
#undef UNP
    LAUNCH_CHECK("k_unpack");
    return 0;
}

int codec_merge_planes(const codec_params* P, const void* planes, int32_t nplanes, int32_t plane_bytes, void* out,
                       void* stream) {
    if (!P || P->B < 1 || P->H < 1 || P->W < 1 || (P->out_bytes != 1 && P->out_bytes != 2))
        return set_err(CODEC_EINVAL, "codec_merge_planes: bad params");
    if (!planes || !out || nplanes < 1 || (plane_bytes != 1 && plane_bytes != 2))
        return set_err(CODEC_EINVAL, "codec_merge_planes: bad arguments");
    const long long npx = (long long)P->H * P->W;
    long long gx = (npx + 255) / 256;
    if (gx > 2048) gx = 2048;
    dim3 grid((unsigned)gx, P->B);
    hipStream_t st = as_stream(stream);
#define MRG(TP, TO) hipLaunchKernelGGL((k_merge<TP, TO>), grid, dim3(256), 0, st, static_cast<const TP*>(planes), nplanes, npx, static_cast<TO*>(out))
    if (plane_bytes == 2 && P->out_bytes == 2) MRG(uint16_t, uint16_t);
    else if (plane_bytes == 2) MRG(uint16_t, uint8_t);
    else if (P->out_bytes == 2) MRG(uint8_t, uint16_t);
    else MRG(uint8_t, uint8_t);
#undef MRG
    LAUNCH_CHECK("k_merge");
    return 0;
}

int codec_block_variance(int32_t B, int32_t H, int32_t W, int32_t bytes, int32_t block, const void* planes,
                         double* scores, void* stream) {
    if (B < 1 || H < 1 || W < 1 || block < 1 || (bytes != 1 && bytes != 2) || !planes || !scores)
        return set_err(CODEC_EINVAL, "codec_block_variance: bad arguments");
    if ((long long)block * block > (1LL << 30))
        return set_err(CODEC_EINVAL, "codec_block_variance: block too large");
    const long long nby = (H + (long long)block - 1) / block, nbx = (W + (long long)block - 1) / block;
    const long long cnt = nby * nbx;
    if (cnt > INT32_MAX - 255) return set_err(CODEC_EINVAL, "codec_block_variance: too many blocks");
    hipStream_t st = as_stream(stream);
    dim3 grid((unsigned)((cnt + 255) / 256), (unsigned)B);
    ProfScope prof(st, CODEC_K_BLOCK_EXACT);
    if (bytes == 2)
        hipLaunchKernelGGL(k_block_exact<uint16_t>, grid, dim3(256), 0, st, static_cast<const uint16_t*>(planes), H, W,
                           block, 0, scores, (int)cnt);
    else
        hipLaunchKernelGGL(k_block_exact<uint8_t>, grid, dim3(256), 0, st, static_cast<const uint8_t*>(planes), H, W,
                           block, 0, scores, (int)cnt);
    LAUNCH_CHECK("k_block_exact");
    return 0;
}

int codec_lsb_runs(int32_t nplanes, int64_t npx, int32_t bytes, void* planes, uint8_t* bitmaps, const uint8_t* bits,
                   int64_t bits_stride, const int64_t* runs, int32_t nruns, void* stream) {
    if (nplanes < 1 || npx < 1 || (bytes != 1 && bytes != 2) || !planes || !bitmaps || nruns < 0 || bits_stride < 0)
        return set_err(CODEC_EINVAL, "codec_lsb_runs: bad arguments");
    if (nruns == 0) return 0;
    if (!bits || !runs) return set_err(CODEC_EINVAL, "codec_lsb_runs: bad arguments");
    hipStream_t st = as_stream(stream);
    ProfScope prof(st, CODEC_K_EMBED);
    const long long* rr = reinterpret_cast<const long long*>(runs);
    if (bytes == 2)
        hipLaunchKernelGGL(k_lsb_runs<uint16_t>, dim3((unsigned)nruns), dim3(256), 0, st, static_cast<uint16_t*>(planes),
                           bitmaps, (long long)npx, bits, (long long)bits_stride, rr);
    else
        hipLaunchKernelGGL(k_lsb_runs<uint8_t>, dim3((unsigned)nruns), dim3(256), 0, st, static_cast<uint8_t*>(planes),
                           bitmaps, (long long)npx, bits, (long long)bits_stride, rr);
    LAUNCH_CHECK("k_lsb_runs");
    return 0;
}

}  // extern "C"
