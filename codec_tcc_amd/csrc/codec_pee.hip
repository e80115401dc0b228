// codec_pee.hip -- MED-predictor prediction-error expansion on gfx950.
// Specification: oracle/pee_cpu.py (the reference has no PEE code; parity unpinned).
//
// Layout: candidates = the (odd, odd) sublattice, index k = i*(W/2) + j for pixel
// (2i+1, 2j+1).  With W % 8 == 0 an aligned 8-pixel chunk of a row pair (2i, 2i+1) holds
// exactly 4 candidates and all of their W / N / NW neighbours, so the streaming pass
// needs no halo: two 16-byte loads per lane.  A tile = 1024 candidates (256 chunks).
//
//   embed  : k_pee_scan (copy cover->stego, per-tile count of expandable candidates)
//            -> k_pee_locate (per slice: scan of tile counts, end candidate, tile offsets)
//            -> k_pee_embed (tiles <= tile_end only: block-scan bit cursor, expansion /
//               shifting, location-map bits)
//   extract: k_pee_copy (stego->cover) + k_pee_dcount (prefix tiles) + k_pee_offsets
//            -> k_pee_recover (prefix tiles: bits + restored pixels)
#include "codec_common.h"

#include <map>
#include <mutex>
#include <utility>

#define PEE_TILE 1024

struct PeeCand {
    int x, p;
    bool expand, right, safe;
};

// LOCO-I MED predictor (oracle/pee_cpu.py med): min(a,b) if c >= max(a,b), max(a,b) if
// c <= min(a,b), else a+b-c -- which is exactly median(a, b, a+b-c) (each case puts a+b-c on
// the far side of the returned value), one v_med3_i32 after an add and a subtract
__device__ __forceinline__ int med3(int a, int b, int c) {
    return max(min(a, b), min(max(a, b), a + b - c));
}

// branch-free classification: -T <= e < T as one unsigned compare; the expansion target
// y = p + 2e (+ bit) must stay in [0, maxval], i.e. (unsigned)y < maxval
__device__ __forceinline__ PeeCand pee_classify(int x, int a, int b, int c, int T, int maxval) {
    PeeCand r;
    r.x = x;
    r.p = med3(a, b, c);
    const int e = x - r.p;
    r.expand = (unsigned)(e + T) < (unsigned)(2 * T);
    r.right = e >= T;
    const int y = r.p + 2 * e;
    // non-short-circuit (&, |): a ?: chain here was compiled into divergent branches
    const bool ok_e = (unsigned)y < (unsigned)maxval, ok_r = x <= maxval - T, ok_l = x >= T;
    r.safe = (r.expand & ok_e) | (!r.expand & r.right & ok_r) | (!r.expand & !r.right & ok_l);
    return r;
}

// candidate k of a slice (scalar access; used for prefix tiles and odd shapes)
template <typename T>
__device__ __forceinline__ void pee_load(const T* img, int W, int wc, int k, int* x, int* a, int* b, int* c) {
    const int i = k / wc, j = k - (k / wc) * wc;
    const size_t y = 2 * (size_t)i + 1, xx = 2 * (size_t)j + 1;
    *x = img[y * W + xx];
    *a = img[y * W + xx - 1];
    *b = img[(y - 1) * W + xx];
    *c = img[(y - 1) * W + xx - 1];
}

__device__ __forceinline__ uint32_t px16(const uint4& v, int e) {
    const uint32_t w = e < 2 ? v.x : (e < 4 ? v.y : (e < 6 ? v.z : v.w));
    return (e & 1) ? (w >> 16) : (w & 0xFFFFu);
}
__device__ __forceinline__ uint32_t px8(const uint2& v, int e) {
    return ((e < 4 ? v.x : v.y) >> (8 * (e & 3))) & 0xFFu;
}
__device__ __forceinline__ void set_px(uint4& v, int e, uint32_t val) {
    uint32_t& w = e < 2 ? v.x : (e < 4 ? v.y : (e < 6 ? v.z : v.w));
    w = (e & 1) ? ((w & 0xFFFFu) | (val << 16)) : ((w & 0xFFFF0000u) | (val & 0xFFFFu));
}
__device__ __forceinline__ void set_px(uint2& v, int e, uint32_t val) {
    uint32_t& w = e < 4 ? v.x : v.y;
    const int sh = 8 * (e & 3);
    w = (w & ~(0xFFu << sh)) | ((val & 0xFFu) << sh);
}
template <typename V> __device__ __forceinline__ uint32_t get_px(const V& v, int e);
template <> __device__ __forceinline__ uint32_t get_px<uint4>(const uint4& v, int e) { return px16(v, e); }
template <> __device__ __forceinline__ uint32_t get_px<uint2>(const uint2& v, int e) { return px8(v, e); }

// The 4 candidates of tile slot (t, tid): k = 1024 t + 4 tid + u.  VEC (W % 8 == 0): they
// are the odd pixels of one aligned 8-pixel chunk of row pair r, loaded as two vectors;
// otherwise scalar loads per candidate.
template <typename T, bool VEC>
struct Quad {
    typedef typename Vec8<T>::type V;
    V v0, v1;           // VEC: rows 2r (N/NW) and 2r+1 (candidates, W)
    size_t o1;          // VEC: element offset of v1
    int x[4], a[4], b[4], c[4];
    __device__ __forceinline__ void load(const T* img, int W, int wc, int k0, int kmax) {
        if constexpr (VEC) {
            if (k0 > kmax) return;
            const int item = k0 >> 2, CR = W / 8;
            const int r = item / CR, cc = item - r * CR;
            const size_t o0 = (size_t)(2 * r) * W + (size_t)cc * 8;
            o1 = o0 + W;
            v0 = *reinterpret_cast<const V*>(img + o0);
            v1 = *reinterpret_cast<const V*>(img + o1);
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                x[u] = (int)get_px(v1, 2 * u + 1); a[u] = (int)get_px(v1, 2 * u);
                b[u] = (int)get_px(v0, 2 * u + 1); c[u] = (int)get_px(v0, 2 * u);
            }
        } else {
#pragma unroll
            for (int u = 0; u < 4; ++u)
                if (k0 + u <= kmax) pee_load(img, W, wc, k0 + u, &x[u], &a[u], &b[u], &c[u]);
        }
    }
    // write candidate u's new value (VEC: into v1; flushed by store())
    __device__ __forceinline__ void put(T* img, int W, int wc, int k, int u, int val) {
        if constexpr (VEC) {
            set_px(v1, 2 * u + 1, (uint32_t)val);
        } else {
            const int i = k / wc, j = k - (k / wc) * wc;
            img[(size_t)(2 * i + 1) * W + 2 * j + 1] = (T)val;
        }
    }
    __device__ __forceinline__ void store(T* img) {
        if constexpr (VEC) *reinterpret_cast<V*>(img + o1) = v1;
    }
};

// ---- scan: stream copy + per-tile count of expandable non-overflow candidates (W % 8 == 0)
// One wave per tile (256 items = 1024 candidates; 4 items per lane, two 16-B rows each, all
// 8 loads issued up front), tiles swept grid-stride over the whole batch in address order
// (global tile g = slice * ntiles + t), so the resident waves read one moving window of
// HBM; the wave's shuffle reduction writes the tile count directly (no LDS, no barrier).
template <typename T, bool NT>
__global__ __launch_bounds__(256) void k_pee_scan(const T* __restrict__ cover, T* __restrict__ stego, int H, int W,
                                                  int T0, int maxval, uint32_t* __restrict__ tile_cnt_all,
                                                  int ntiles_max, int B, const int32_t* __restrict__ tps) {
    typedef typename Vec8<T>::type V;
    const size_t npx = (size_t)H * W;
    const int CR = W / 8, hc = H / 2;
    const uint32_t items = (uint32_t)hc * (uint32_t)CR;
    const uint32_t ntiles = (items + 255u) / 256u;
    const uint32_t total = ntiles * (uint32_t)B;
    const int lane = threadIdx.x & 63;
    const uint32_t wstride = gridDim.x * 4u;
    for (uint32_t g = blockIdx.x * 4u + (threadIdx.x >> 6); g < total; g += wstride) {
        const uint32_t b = g / ntiles, t = g - b * ntiles;
        const int Tthr = tps ? tps[b] : T0;   // per-slice threshold (capacity control) or one for all
        const T* src = cover + b * npx;
        T* dst = stego + b * npx;
        V v0[4], v1[4];
        size_t o0[4];
        bool ok[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const uint32_t it = t * 256u + (uint32_t)(u * 64 + lane);
            ok[u] = it < items;
            const uint32_t r = it / (uint32_t)CR, c = it - r * (uint32_t)CR;
            o0[u] = (size_t)(2 * r) * W + (size_t)c * 8;
            if (ok[u]) {
                v0[u] = ldv<NT>(reinterpret_cast<const V*>(src + o0[u]));
                v1[u] = ldv<NT>(reinterpret_cast<const V*>(src + o0[u] + W));
            }
        }
        uint32_t cnt = 0;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            if (!ok[u]) continue;
            stv<NT>(reinterpret_cast<V*>(dst + o0[u]), v0[u]);
            stv<NT>(reinterpret_cast<V*>(dst + o0[u] + W), v1[u]);
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                int x, a, bb, cc;
                if constexpr (sizeof(T) == 2) {
                    x = (int)px16(v1[u], 2 * k + 1); a = (int)px16(v1[u], 2 * k); bb = (int)px16(v0[u], 2 * k + 1); cc = (int)px16(v0[u], 2 * k);
                } else {
                    x = (int)px8(v1[u], 2 * k + 1); a = (int)px8(v1[u], 2 * k); bb = (int)px8(v0[u], 2 * k + 1); cc = (int)px8(v0[u], 2 * k);
                }
                const PeeCand pc = pee_classify(x, a, bb, cc, Tthr, maxval);
                cnt += (pc.expand && pc.safe) ? 1u : 0u;
            }
        }
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) cnt += __shfl_xor(cnt, o, 64);
        if (lane == 0) tile_cnt_all[(size_t)b * ntiles_max + t] = cnt;
    }
    // odd H: the last row of each slice belongs to no row pair; copy it
    if (H & 1) {
        for (int b = blockIdx.x; b < B; b += gridDim.x) {
            const size_t o = (size_t)b * npx + (size_t)(H - 1) * W;
            for (int q = threadIdx.x; q < W; q += 256) stego[o + q] = cover[o + q];
        }
    }
}

// ---- scan for any shape: counts only (the copy is a separate stream copy)
template <typename T>
__global__ __launch_bounds__(256) void k_pee_count(const T* __restrict__ img, int H, int W, int T0, int maxval,
                                                   int tiles_per_wg, uint32_t* __restrict__ tile_cnt_all,
                                                   int ntiles_max, const int32_t* __restrict__ tps) {
    __shared__ uint32_t sh[8];
    const int b = blockIdx.y;
    const int Tthr = tps ? tps[b] : T0;
    const T* src = img + (size_t)b * H * W;
    const int wc = W / 2, nc = (H / 2) * wc;
    const int ntiles = (nc + PEE_TILE - 1) / PEE_TILE;
    uint32_t* tile_cnt = tile_cnt_all + (size_t)b * ntiles_max;
    const int t0 = blockIdx.x * tiles_per_wg;
    const int t1 = min(ntiles, t0 + tiles_per_wg);
    for (int t = t0; t < t1; ++t) {
        uint32_t cnt = 0;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int k = t * PEE_TILE + 4 * threadIdx.x + u;
            if (k < nc) {
                int x, a, bb, cc;
                pee_load(src, W, wc, k, &x, &a, &bb, &cc);
                const PeeCand pc = pee_classify(x, a, bb, cc, Tthr, maxval);
                cnt += (pc.expand && pc.safe) ? 1u : 0u;
            }
        }
        const uint32_t tot = block_sum_u32<256>(cnt, sh);
        if (threadIdx.x == 0) tile_cnt[t] = tot;
    }
}

// ---- per slice: exclusive tile offsets, capacity, tile holding bit L-1, exact `end`
template <typename T>
__global__ __launch_bounds__(256) void k_pee_locate(const T* __restrict__ img, int H, int W, int T0, int maxval,
                                                    const int32_t* __restrict__ lengths,
                                                    const uint32_t* __restrict__ tile_cnt_all,
                                                    uint32_t* __restrict__ tile_off_all, int ntiles_max,
                                                    codec_pee_meta* __restrict__ meta_all,
                                                    const int32_t* __restrict__ tps) {
    __shared__ uint32_t sh[8];
    __shared__ int s_tile;
    __shared__ uint32_t s_base;
    __shared__ int s_end;
    const int b = blockIdx.x;
    const int Tthr = tps ? tps[b] : T0;
    const int wc = W / 2, nc = (H / 2) * wc;
    const int ntiles = (nc + PEE_TILE - 1) / PEE_TILE;
    const uint32_t* cnt = tile_cnt_all + (size_t)b * ntiles_max;
    uint32_t* off = tile_off_all + (size_t)b * ntiles_max;
    const uint32_t L = (uint32_t)max(0, lengths[b]);
    if (threadIdx.x == 0) { s_tile = -1; s_end = -1; s_base = 0; }
    __syncthreads();
    uint32_t running = 0;
    for (int base = 0; base < ntiles; base += 256) {
        const int t = base + threadIdx.x;
        const uint32_t c = t < ntiles ? cnt[t] : 0u;
        uint32_t tot;
        const uint32_t ex = running + block_excl_scan<256>(c, sh, &tot);
        if (t < ntiles) off[t] = ex;
        if (t < ntiles && L > 0 && ex < L && ex + c >= L) { s_tile = t; s_base = ex; }
        running += tot;
    }
    __syncthreads();
    const int tile = s_tile;
    if (tile >= 0) {
        // exact end: the (L - base)-th expandable candidate of `tile`
        const T* src = img + (size_t)b * H * W;
        uint32_t flags = 0, local = 0;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int k = tile * PEE_TILE + 4 * threadIdx.x + u;
            if (k < nc) {
                int x, a, bb, cc;
                pee_load(src, W, wc, k, &x, &a, &bb, &cc);
                const PeeCand pc = pee_classify(x, a, bb, cc, Tthr, maxval);
                if (pc.expand && pc.safe) { flags |= 1u << u; ++local; }
            }
        }
        uint32_t tot;
        const uint32_t pre = block_excl_scan<256>(local, sh, &tot);
        const uint32_t need = L - s_base;   // 1-based rank inside the tile
        if (need > pre && need <= pre + local) {
            uint32_t r = pre;
#pragma unroll
            for (int u = 0; u < 4; ++u)
                if ((flags >> u) & 1u) {
                    ++r;
                    if (r == need) s_end = tile * PEE_TILE + 4 * threadIdx.x + u;
                }
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        codec_pee_meta* M = meta_all + b;
        M->T = Tthr;
        M->maxval = maxval;
        M->L = (int)L;
        M->nc = nc;
        M->ntiles = ntiles;
        M->capacity = (int)running;
        M->h = H;
        M->w = W;
        if (L == 0) {
            M->end = -1; M->tile_end = -1; M->status = 0;
        } else if (running < L) {   // payload exceeds capacity: embed `running` bits, process all
            M->end = nc - 1; M->tile_end = ntiles - 1; M->status = 1;
        } else {
            M->end = s_end; M->tile_end = tile; M->status = 0;
        }
        M->lm_count = 0;
        M->flags = 0;
    }
}

// ---- embed: prefix tiles only
template <typename T, bool VEC>
__global__ __launch_bounds__(256) void k_pee_embed(const T* __restrict__ cover, T* __restrict__ stego, int H, int W,
                                                   const u64* __restrict__ payload_all, int pw,
                                                   const uint32_t* __restrict__ tile_off_all, int ntiles_max,
                                                   codec_pee_meta* __restrict__ meta_all,
                                                   u64* __restrict__ lm_all, int lmw) {
    __shared__ uint32_t sh[8];
    __shared__ uint32_t lm32[PEE_TILE / 32];
    const int b = blockIdx.y;
    codec_pee_meta* M = meta_all + b;
    const int tile_end = M->tile_end, end = M->end, Tthr = M->T, maxval = M->maxval;
    const int wc = W / 2;
    const size_t npx = (size_t)H * W;
    const T* src = cover + b * npx;
    T* dst = stego + b * npx;
    const u64* payload = payload_all + (size_t)b * pw;
    u64* lm = lm_all + (size_t)b * lmw;
    const uint32_t* off = tile_off_all + (size_t)b * ntiles_max;
    for (int t = blockIdx.x; t <= tile_end; t += gridDim.x) {
        if (threadIdx.x < PEE_TILE / 32) lm32[threadIdx.x] = 0;
        const int k0 = t * PEE_TILE + 4 * threadIdx.x;
        Quad<T, VEC> q;
        q.load(src, W, wc, k0, end);
        PeeCand pc[4];
        uint32_t local = 0;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            pc[u].expand = pc[u].safe = pc[u].right = false;
            if (k0 + u <= end) {
                pc[u] = pee_classify(q.x[u], q.a[u], q.b[u], q.c[u], Tthr, maxval);
                local += (pc[u].expand && pc[u].safe) ? 1u : 0u;
            }
        }
        uint32_t tot;
        uint32_t cur = off[t] + block_excl_scan<256>(local, sh, &tot);   // also orders lm32 zeroing
        uint32_t nib = 0, unsafe = 0;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int k = k0 + u;
            if (k > end) continue;
            if (!pc[u].safe) { nib |= 1u << u; ++unsafe; continue; }
            int nv;
            if (pc[u].expand) {
                const int bit = (int)((payload[cur >> 6] >> (cur & 63)) & 1ull);
                ++cur;
                nv = pc[u].p + 2 * (pc[u].x - pc[u].p) + bit;
            } else {
                nv = pc[u].right ? pc[u].x + Tthr : pc[u].x - Tthr;
            }
            q.put(dst, W, wc, k, u, nv);
        }
        if (k0 <= end) q.store(dst);
        if (nib) atomicOr(&lm32[(4 * threadIdx.x) >> 5], nib << ((4 * threadIdx.x) & 31));
        const uint32_t nun = block_sum_u32<256>(unsafe, sh);
        if (threadIdx.x < PEE_TILE / 64) {
            const int w = t * (PEE_TILE / 64) + threadIdx.x;
            if (w < lmw) lm[w] = (u64)lm32[2 * threadIdx.x] | ((u64)lm32[2 * threadIdx.x + 1] << 32);
        }
        if (threadIdx.x == 0 && nun) atomicAdd(&M->lm_count, (int)nun);
        __syncthreads();
    }
}

// ---- capacity control.  The expansion safety test (p + 2e >= 0, p + 2e + 1 <= maxval)
// does not depend on T, so one pass that histograms the prediction errors of the
// candidates whose expansion would be safe gives every capacity exactly: with u = e for
// e >= 0 and -e - 1 for e < 0, e lies in [-T, T) iff u < T, so capacity(T) = sum of the
// u-bins below T.  grid (regions, B), 256 threads.  The bins are lane-private LDS
// counters (bin u of thread t at u * 256 + t: a wave's 64 lanes always hit 64 banks), so
// an update is a plain read-add-write instead of an LDS atomic on a handful of hot bins
// (the errors of a smooth slice crowd around 0: 64-way same-address atomics ran at
// ~0.5 lane-ops per cycle); equal bins of a lane's 4 candidates are merged first.  The
// workgroup's bins are reduced and added to the slice's global bins; the slice's last
// workgroup (a per-slice arrival counter) turns them into the capacity curve and the
// chosen T, and clears bins and counter (the workspace is zeroed once: no memset, no
// second launch per call).
#define PEE_TMAX_MAX 64
__device__ __forceinline__ void pee_select_slice(uint32_t* h, int tmax, long long L, int32_t* caps, int32_t* t_out) {
    long long run = 0;
    int tsel = 0;
    for (int t = 1; t <= tmax; ++t) {
        run += (long long)__hip_atomic_load(h + t - 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        h[t - 1] = 0u;
        if (caps) caps[t - 1] = (int32_t)run;
        if (!tsel && run >= L) tsel = t;
    }
    if (t_out) *t_out = tsel ? tsel : tmax;
}

// Capacity histogram update for the 4 candidates of one item (or the first nq of them):
// bin u = folded error (e >= 0 ? e : -e - 1) of every candidate whose expansion p + 2e (+1)
// stays in [0, maxval]; equal bins merged, then one independent read-add-write per distinct
// bin into the lane's own counters cnt[u * NLANES + lane] (no LDS atomics, conflict-free:
// a lane always hits its own bank).  Shared by k_pee_ehist and the fused capacity phase of
// k_pee_embed_ss.
template <int NLANES>
__device__ __forceinline__ void ehist_add4(uint32_t* cnt, int lane_ix, const int (&x)[4], const int (&a)[4],
                                           const int (&bb)[4], const int (&cc)[4], int nq, int tmax, int maxval) {
    int u[4];
    uint32_t c[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int p = med3(a[q], bb[q], cc[q]), e = x[q] - p;
        const int uq = e >= 0 ? e : -e - 1;
        u[q] = uq;
        c[q] = (q < nq) & (uq < tmax) & (p + 2 * e >= 0) & (p + 2 * e + 1 <= maxval) ? 1u : 0u;
    }
#pragma unroll
    for (int q = 1; q < 4; ++q)
#pragma unroll
        for (int r = 0; r < q; ++r) {   // branch-free merge (& instead of &&)
            const bool same = (c[r] != 0u) & (c[q] != 0u) & (u[r] == u[q]);
            c[r] += same ? c[q] : 0u;
            c[q] = same ? 0u : c[q];
        }
    uint32_t old[4];
    int ad[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        ad[q] = min(u[q], tmax - 1) * NLANES + lane_ix;
        old[q] = cnt[ad[q]];
    }
#pragma unroll
    for (int q = 0; q < 4; ++q)
        if (c[q]) cnt[ad[q]] = old[q] + c[q];   // masked: a merged duplicate must not write back
}

template <typename T, bool VEC>
__global__ __launch_bounds__(256) void k_pee_ehist(const T* __restrict__ img, int H, int W, int maxval, int tmax,
                                                   int per_wg, uint32_t* __restrict__ hist_all,
                                                   uint32_t* __restrict__ arrivals, const int32_t* __restrict__ lengths,
                                                   int32_t* __restrict__ caps, int32_t* __restrict__ t_out,
                                                   int dbg_delay) {
    typedef typename Vec8<T>::type V;
    extern __shared__ uint32_t cnt[];                 // [tmax][256]
    __shared__ uint32_t bins[PEE_TMAX_MAX];
    const int b = blockIdx.y, tid = threadIdx.x;
    const T* src = img + (size_t)b * H * W;
    for (int u = 0; u < tmax; ++u) cnt[u * 256 + tid] = 0u;
    if (tid < tmax) bins[tid] = 0u;
    auto add4 = [&](const int (&x)[4], const int (&a)[4], const int (&bb)[4], const int (&cc)[4], int nq) {
        ehist_add4<256>(cnt, tid, x, a, bb, cc, nq, tmax, maxval);
    };
    __syncthreads();
    if constexpr (VEC) {
        const uint32_t CR = (uint32_t)W / 8;
        const uint32_t items = (uint32_t)(H / 2) * CR;
        const uint32_t i0 = (uint32_t)blockIdx.x * (uint32_t)per_wg;
        const uint32_t i1 = min(items, i0 + (uint32_t)per_wg);
        const uint32_t dq = 256u / CR, dr = 256u % CR;
        uint32_t it = i0 + (uint32_t)tid;
        uint32_t r = it / CR, c = it - r * CR;             // advanced without divisions below
        // 4 items per thread per step, their 8 loads issued together (one item at a time
        // left each thread waiting a full HBM round trip per item); plain loads: the embed
        // that follows reads the same cover, and at C3 size it is still in the MALL
        constexpr int U = 4;
        for (; it < i1; it += 256 * U) {
            V v0[U], v1[U];
            bool in[U];
#pragma unroll
            for (int k = 0; k < U; ++k) {
                in[k] = it + 256u * k < i1;
                const size_t o0 = in[k] ? (size_t)(2 * r) * W + (size_t)c * 8 : 0;
                v0[k] = *reinterpret_cast<const V*>(src + o0);
                v1[k] = *reinterpret_cast<const V*>(src + o0 + W);
                c += dr;
                r += dq;
                if (c >= CR) { c -= CR; ++r; }
            }
#pragma unroll
            for (int k = 0; k < U; ++k) {
                int x[4], a[4], bb[4], cc[4];
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    x[q] = (int)get_px(v1[k], 2 * q + 1); a[q] = (int)get_px(v1[k], 2 * q);
                    bb[q] = (int)get_px(v0[k], 2 * q + 1); cc[q] = (int)get_px(v0[k], 2 * q);
                }
                add4(x, a, bb, cc, in[k] ? 4 : 0);
            }
        }
    } else {
        const int wc = W / 2;
        const int nc = (H / 2) * wc;
        const int k0 = blockIdx.x * per_wg, k1 = min(nc, k0 + per_wg);
        for (int k = k0 + tid; k < k1; k += 256) {
            int x[4] = {0, 0, 0, 0}, a[4] = {0, 0, 0, 0}, bb[4] = {0, 0, 0, 0}, cc[4] = {0, 0, 0, 0};
            pee_load(src, W, wc, k, &x[0], &a[0], &bb[0], &cc[0]);
            add4(x, a, bb, cc, 1);
        }
    }
    if (dbg_delay >= 0 && b == 0 && (int)blockIdx.x == dbg_delay % (int)gridDim.x) {
        // CODEC_PEE_EHIST_DEBUG_DELAY (tests only): this workgroup flushes its bins ~1 ms after
        // every other workgroup of the slice, i.e. it arrives last and selects T over bins
        // flushed long before -- or, with the delay after its own flush (odd knob values),
        // it arrives last right behind its own returning atomics
        if (!(dbg_delay & 1))
            for (int k = 0; k < 300; ++k) __builtin_amdgcn_s_sleep(127);
    }
    __syncthreads();
    // bin u of the workgroup: thread t sums lanes t / tmax, + 256 / tmax ... of bin t % tmax
    const int g = 256 / tmax;
    if (tid < g * tmax) {
        const int u = tid % tmax;
        uint32_t sum = 0;
        for (int l = tid / tmax; l < 256; l += g) sum += cnt[u * 256 + l];
        if (sum) atomicAdd(&bins[u], sum);
    }
    __syncthreads();
    // No __threadfence: on gfx950 an agent-scope release writes back the XCD's L2 (measured:
    // 30 -> 180 us for this kernel at C3).  The bins' device-scope atomics are returning ones
    // whose results are waited for, i.e. performed at the coherence point before the
    // barrier, and so before this workgroup's arrival atomic; the last arrival then reads
    // the bins with device-scope atomic loads.
    if (tid < tmax && bins[tid]) {
        const uint32_t prev = atomicAdd(&hist_all[(size_t)b * PEE_TMAX_MAX + tid], bins[tid]);
        asm volatile("" ::"v"(prev));   // wait for the atomic's return
    }
    __shared__ uint32_t ticket;
    if (dbg_delay >= 0 && (dbg_delay & 1) && b == 0 && (int)blockIdx.x == dbg_delay % (int)gridDim.x)
        for (int k = 0; k < 300; ++k) __builtin_amdgcn_s_sleep(127);
    __syncthreads();
    if (tid == 0) ticket = atomicAdd(&arrivals[b], 1u);
    __syncthreads();
    if (ticket == gridDim.x - 1u && tid == 0) {   // the slice's last workgroup
        const long long L = lengths ? (long long)max(0, lengths[b]) : 0;
        pee_select_slice(hist_all + (size_t)b * PEE_TMAX_MAX, tmax, L, caps ? caps + (size_t)b * tmax : nullptr,
                         t_out ? t_out + b : nullptr);
        arrivals[b] = 0u;
    }
}

// ---- decode-side cursor counts, wave per tile (W % 8 == 0): a tile's 256 items are 4 per
// lane (item u*64 + lane, 8 loads in flight), inner candidates are counted in registers and
// reduced with shuffles -- no LDS, no block barrier (0.058-0.062 vs 0.072 ms for the
// workgroup-per-tile k_pee_dcount at 256 x 2048^2).  (A wave-per-tile embed measured
// slower than k_pee_embed -- 0.109 vs 0.099 ms: its cursor needs a scan per item slot
// followed by a dependent payload load -- and was dropped.)
template <typename T>
__global__ __launch_bounds__(256) void k_pee_dcount_w(const T* __restrict__ stego, int H, int W,
                                                      const codec_pee_meta* __restrict__ meta_all,
                                                      const u64* __restrict__ lm_all, int lmw,
                                                      uint32_t* __restrict__ tile_cnt_all, int ntiles_max) {
    typedef typename Vec8<T>::type V;
    const int b = blockIdx.y;
    const codec_pee_meta* M = meta_all + b;
    const int tile_end = M->tile_end, end = M->end, Tthr = M->T;
    const T* src = stego + (size_t)b * H * W;
    const u64* lm = lm_all + (size_t)b * lmw;
    const int lane = threadIdx.x & 63;
    const int CR = W / 8;
    const uint32_t items = (uint32_t)(H / 2) * (uint32_t)CR;
    for (int t = blockIdx.x * 4 + (threadIdx.x >> 6); t <= tile_end; t += gridDim.x * 4) {
        V v0[4], v1[4];
        bool ok[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const uint32_t it = (uint32_t)t * 256u + (uint32_t)(u * 64 + lane);
            ok[u] = it < items && (int)(4 * it) <= end;
            const uint32_t r = it / (uint32_t)CR, c = it - r * (uint32_t)CR;
            const size_t o0 = (size_t)(2 * r) * W + (size_t)c * 8;
            if (ok[u]) {
                v0[u] = *reinterpret_cast<const V*>(src + o0);
                v1[u] = *reinterpret_cast<const V*>(src + o0 + W);
            }
        }
        uint32_t local = 0;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            if (!ok[u]) continue;
            const int k0 = (int)(4 * ((uint32_t)t * 256u + (uint32_t)(u * 64 + lane)));
            const uint32_t nib = (uint32_t)(lm[k0 >> 6] >> (k0 & 63)) & 0xFu;   // 4 | k0: one word
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                if (k0 + e > end || ((nib >> e) & 1u)) continue;
                const int e2 = (int)get_px(v1[u], 2 * e + 1) -
                               med3((int)get_px(v1[u], 2 * e), (int)get_px(v0[u], 2 * e + 1), (int)get_px(v0[u], 2 * e));
                local += (e2 >= -2 * Tthr && e2 < 2 * Tthr) ? 1u : 0u;
            }
        }
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) local += __shfl_xor(local, o, 64);
        if (lane == 0) tile_cnt_all[(size_t)b * ntiles_max + t] = local;
    }
}

// ---- embed, prefix tiles, W % 8 == 0: same work as k_pee_embed with one barrier per tile
// instead of seven -- the bit cursor is a wave scan plus the (double-buffered) totals of
// the tile's earlier waves, location-map words are OR-reduced over 16 lanes with shuffles
// and stored directly, the unsafe count goes out with one atomic per wave at the end.
template <typename T>
__global__ __launch_bounds__(256) void k_pee_embed_v(const T* __restrict__ cover, T* __restrict__ stego, int H, int W,
                                                     const u64* __restrict__ payload_all, int pw,
                                                     const uint32_t* __restrict__ tile_off_all, int ntiles_max,
                                                     codec_pee_meta* __restrict__ meta_all,
                                                     u64* __restrict__ lm_all, int lmw) {
    typedef typename Vec8<T>::type V;
    __shared__ uint32_t wtot[2][4];
    const int b = blockIdx.y;
    codec_pee_meta* M = meta_all + b;
    const int tile_end = M->tile_end, end = M->end, Tthr = M->T, maxval = M->maxval;
    const size_t npx = (size_t)H * W;
    const T* src = cover + b * npx;
    T* dst = stego + b * npx;
    const u64* payload = payload_all + (size_t)b * pw;
    u64* lm = lm_all + (size_t)b * lmw;
    const uint32_t* off = tile_off_all + (size_t)b * ntiles_max;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int CR = W / 8;
    int nun = 0, par = 0;
    for (int t = blockIdx.x; t <= tile_end; t += gridDim.x, par ^= 1) {
        const int item = t * 256 + threadIdx.x;
        const int k0 = 4 * item;
        const bool ok = k0 <= end;
        const int r = item / CR, c = item - r * CR;
        const size_t o0 = (size_t)(2 * r) * W + (size_t)c * 8, o1 = o0 + W;
        V v0, v1;
        if (ok) {
            v0 = *reinterpret_cast<const V*>(src + o0);
            v1 = *reinterpret_cast<const V*>(src + o1);
        }
        const uint32_t tbase = off[t];
        PeeCand pc[4];
        uint32_t local = 0;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            pc[u].expand = pc[u].safe = pc[u].right = false;
            if (ok && k0 + u <= end) {
                pc[u] = pee_classify((int)get_px(v1, 2 * u + 1), (int)get_px(v1, 2 * u), (int)get_px(v0, 2 * u + 1),
                                     (int)get_px(v0, 2 * u), Tthr, maxval);
                local += (pc[u].expand && pc[u].safe) ? 1u : 0u;
            }
        }
        uint32_t inc = local;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(inc, o, 64);
            if (lane >= o) inc += y;
        }
        if (lane == 63) wtot[par][wv] = inc;
        __syncthreads();
        uint32_t cur = tbase + inc - local;
        for (int w = 0; w < wv; ++w) cur += wtot[par][w];
        const uint32_t w0 = cur >> 6;                 // this thread's <= 4 bits: words w0, w0 + 1
        const u64 p0 = local ? payload[w0] : 0ull;
        const u64 p1 = (local && (int)w0 + 1 < pw) ? payload[w0 + 1] : 0ull;
        uint32_t nib = 0;
        bool any = false;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            if (!ok || k0 + u > end) continue;
            if (!pc[u].safe) { nib |= 1u << u; ++nun; continue; }
            int nv;
            if (pc[u].expand) {
                const u64 wd = (cur >> 6) == w0 ? p0 : p1;
                const int bit = (int)((wd >> (cur & 63)) & 1ull);
                ++cur;
                nv = pc[u].p + 2 * (pc[u].x - pc[u].p) + bit;
            } else {
                nv = pc[u].right ? pc[u].x + Tthr : pc[u].x - Tthr;
            }
            set_px(v1, 2 * u + 1, (uint32_t)nv);
            any = true;
        }
        if (any) *reinterpret_cast<V*>(dst + o1) = v1;
        // location-map word (4 * item) / 64 = 16 threads x 4 candidate bits
        u64 wm = (u64)nib << (4 * (lane & 15));
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) wm |= __shfl_xor(wm, o, 64);
        const int wi = k0 >> 6;
        if ((lane & 15) == 0 && wi < lmw) lm[wi] = wm;
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) nun += __shfl_xor(nun, o, 64);
    if (lane == 0 && nun) atomicAdd(&M->lm_count, nun);
}

// ---- extract
template <typename T, bool NT>
__global__ __launch_bounds__(256) void k_pee_copy(const T* __restrict__ src, T* __restrict__ dst, long long nbytes) {
    const long long nv = nbytes / 16;
    const uint4* s = reinterpret_cast<const uint4*>(src);
    uint4* d = reinterpret_cast<uint4*>(dst);
    const long long stride = (long long)gridDim.x * 256 * 4;
    for (long long i0 = (long long)blockIdx.x * 256 * 4 + threadIdx.x; i0 < nv; i0 += stride) {
        uint4 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u)
            if (i0 + u * 256 < nv) v[u] = ldv<NT>(s + i0 + u * 256);
#pragma unroll
        for (int u = 0; u < 4; ++u)
            if (i0 + u * 256 < nv) stv<NT>(d + i0 + u * 256, v[u]);
    }
    if (blockIdx.x == 0) {
        const char* sc = reinterpret_cast<const char*>(src);
        char* dc = reinterpret_cast<char*>(dst);
        for (long long i = nv * 16 + threadIdx.x; i < nbytes; i += 256) dc[i] = sc[i];
    }
}

__device__ __forceinline__ bool lm_bit(const u64* lm, int k, int lmw) {
    return (k >> 6) < lmw && ((lm[k >> 6] >> (k & 63)) & 1ull);
}

template <typename T, bool VEC>
__global__ __launch_bounds__(256) void k_pee_dcount(const T* __restrict__ stego, int H, int W,
                                                    const codec_pee_meta* __restrict__ meta_all,
                                                    const u64* __restrict__ lm_all, int lmw,
                                                    uint32_t* __restrict__ tile_cnt_all, int ntiles_max) {
    __shared__ uint32_t sh[8];
    const int b = blockIdx.y;
    const codec_pee_meta* M = meta_all + b;
    const int tile_end = M->tile_end, end = M->end, Tthr = M->T;
    const int wc = W / 2;
    const T* src = stego + (size_t)b * H * W;
    const u64* lm = lm_all + (size_t)b * lmw;
    for (int t = blockIdx.x; t <= tile_end; t += gridDim.x) {
        const int k0 = t * PEE_TILE + 4 * threadIdx.x;
        Quad<T, VEC> q;
        q.load(src, W, wc, k0, end);
        uint32_t local = 0;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int k = k0 + u;
            if (k <= end && !lm_bit(lm, k, lmw)) {
                const int e2 = q.x[u] - med3(q.a[u], q.b[u], q.c[u]);
                local += (e2 >= -2 * Tthr && e2 < 2 * Tthr) ? 1u : 0u;
            }
        }
        const uint32_t tot = block_sum_u32<256>(local, sh);
        if (threadIdx.x == 0) tile_cnt_all[(size_t)b * ntiles_max + t] = tot;
    }
}

__global__ __launch_bounds__(256) void k_pee_offsets(const codec_pee_meta* __restrict__ meta_all,
                                                     const uint32_t* __restrict__ tile_cnt_all,
                                                     uint32_t* __restrict__ tile_off_all, int ntiles_max) {
    __shared__ uint32_t sh[8];
    const int b = blockIdx.x;
    const int n = meta_all[b].tile_end + 1;
    const uint32_t* cnt = tile_cnt_all + (size_t)b * ntiles_max;
    uint32_t* off = tile_off_all + (size_t)b * ntiles_max;
    uint32_t running = 0;
    for (int base = 0; base < n; base += 256) {
        const int t = base + threadIdx.x;
        const uint32_t c = t < n ? cnt[t] : 0u;
        uint32_t tot;
        const uint32_t ex = running + block_excl_scan<256>(c, sh, &tot);
        if (t < n) off[t] = ex;
        running += tot;
    }
}

template <typename T, bool VEC>
__global__ __launch_bounds__(256) void k_pee_recover(const T* __restrict__ stego, T* __restrict__ cover, int H, int W,
                                                     const codec_pee_meta* __restrict__ meta_all,
                                                     const u64* __restrict__ lm_all, int lmw,
                                                     const uint32_t* __restrict__ tile_off_all, int ntiles_max,
                                                     u64* __restrict__ payload_all, int pw) {
    __shared__ uint32_t sh[8];
    const int b = blockIdx.y;
    const codec_pee_meta* M = meta_all + b;
    const int tile_end = M->tile_end, end = M->end, Tthr = M->T;
    const int wc = W / 2;
    const size_t npx = (size_t)H * W;
    const T* src = stego + b * npx;
    T* dst = cover + b * npx;
    const u64* lm = lm_all + (size_t)b * lmw;
    u64* payload = payload_all + (size_t)b * pw;
    const uint32_t* off = tile_off_all + (size_t)b * ntiles_max;
    for (int t = blockIdx.x; t <= tile_end; t += gridDim.x) {
        const int k0 = t * PEE_TILE + 4 * threadIdx.x;
        Quad<T, VEC> q;
        q.load(src, W, wc, k0, end);
        int ps[4];
        bool act[4], inner[4];
        uint32_t local = 0;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int k = k0 + u;
            act[u] = k <= end && !lm_bit(lm, k, lmw);
            inner[u] = false;
            ps[u] = 0;
            if (act[u]) {
                ps[u] = med3(q.a[u], q.b[u], q.c[u]);
                const int e2 = q.x[u] - ps[u];
                inner[u] = e2 >= -2 * Tthr && e2 < 2 * Tthr;
                local += inner[u] ? 1u : 0u;
            }
        }
        uint32_t tot;
        uint32_t cur = off[t] + block_excl_scan<256>(local, sh, &tot);
        u64 word = 0;
        int wi = -1;
        bool any = false;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            if (!act[u]) continue;
            const int e2 = q.x[u] - ps[u];
            int x;
            if (inner[u]) {
                if (e2 & 1) {      // bits of one thread are consecutive: one atomic per word
                    if (wi != (int)(cur >> 6)) {
                        if (wi >= 0 && word) atomicOr(&payload[wi], word);
                        wi = (int)(cur >> 6);
                        word = 0;
                    }
                    word |= 1ull << (cur & 63);
                }
                ++cur;
                x = ps[u] + (e2 >> 1);
            } else {
                x = e2 >= 2 * Tthr ? q.x[u] - Tthr : q.x[u] + Tthr;
            }
            q.put(dst, W, wc, k0 + u, u, x);
            any = true;
        }
        if (wi >= 0 && word) atomicOr(&payload[wi], word);
        if (any) q.store(dst);
    }
}

// Fused extract sweep (W % 8 == 0 and 256 | items per slice): stego -> cover for the whole
// batch in address order; a workgroup iteration covers 4 whole tiles (u-slot u = tile
// base/256 + u), and slots whose tile lies in the slice's prefix (<= tile_end) recover
// bits and pixels in registers with a block scan for the cursor.
template <typename T, bool NT>
__global__ __launch_bounds__(256) void k_pee_restore_gs(const T* __restrict__ stego, T* __restrict__ cover, int H, int W,
                                                        uint32_t items_per_slice, uint32_t total_items,
                                                        const codec_pee_meta* __restrict__ meta_all,
                                                        const u64* __restrict__ lm_all, int lmw,
                                                        const uint32_t* __restrict__ tile_off_all, int ntiles_max,
                                                        u64* __restrict__ payload_all, int pw) {
    typedef typename Vec8<T>::type V;
    __shared__ uint32_t sh[8];
    const int CR = W / 8;
    const uint32_t tiles_per_slice = items_per_slice / 256u;
    const size_t npx = (size_t)H * W;
    const uint32_t stride = gridDim.x * 1024u;
    for (uint32_t base = blockIdx.x * 1024u; base < total_items; base += stride) {
        V a0[4], a1[4];
        size_t o0[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const uint32_t g = base + u * 256u + threadIdx.x;
            if (g < total_items) {
                const uint32_t b = g / items_per_slice, it = g - b * items_per_slice;
                const uint32_t r = it / CR, c = it - r * CR;
                o0[u] = b * npx + (size_t)(2 * r) * W + (size_t)c * 8;
                a0[u] = ldv<NT>(reinterpret_cast<const V*>(stego + o0[u]));
                a1[u] = ldv<NT>(reinterpret_cast<const V*>(stego + o0[u] + W));
            }
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const uint32_t gt = base / 256u + u;                        // global tile (uniform)
            if (gt * 256u >= total_items) break;
            const uint32_t b = gt / tiles_per_slice, t = gt - b * tiles_per_slice;
            const codec_pee_meta* M = meta_all + b;
            if ((int)t <= M->tile_end) {                                 // uniform per slot
                const int end = M->end, Tthr = M->T;
                const u64* lm = lm_all + (size_t)b * lmw;
                const int k0 = (int)t * PEE_TILE + 4 * threadIdx.x;
                int ps[4], xs[4];
                bool act[4], inner[4];
                uint32_t local = 0;
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const int k = k0 + q;
                    xs[q] = (int)get_px(a1[u], 2 * q + 1);
                    act[q] = k <= end && !lm_bit(lm, k, lmw);
                    inner[q] = false;
                    ps[q] = 0;
                    if (act[q]) {
                        ps[q] = med3((int)get_px(a1[u], 2 * q), (int)get_px(a0[u], 2 * q + 1), (int)get_px(a0[u], 2 * q));
                        const int e2 = xs[q] - ps[q];
                        inner[q] = e2 >= -2 * Tthr && e2 < 2 * Tthr;
                        local += inner[q] ? 1u : 0u;
                    }
                }
                uint32_t tot;
                uint32_t cur = tile_off_all[(size_t)b * ntiles_max + t] + block_excl_scan<256>(local, sh, &tot);
                u64* payload = payload_all + (size_t)b * pw;
                u64 word = 0;
                int wi = -1;
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    if (!act[q]) continue;
                    const int e2 = xs[q] - ps[q];
                    int x;
                    if (inner[q]) {
                        if (e2 & 1) {
                            if (wi != (int)(cur >> 6)) {
                                if (wi >= 0 && word) atomicOr(&payload[wi], word);
                                wi = (int)(cur >> 6);
                                word = 0;
                            }
                            word |= 1ull << (cur & 63);
                        }
                        ++cur;
                        x = ps[q] + (e2 >> 1);
                    } else {
                        x = e2 >= 2 * Tthr ? xs[q] - Tthr : xs[q] + Tthr;
                    }
                    set_px(a1[u], 2 * q + 1, (uint32_t)x);
                }
                if (wi >= 0 && word) atomicOr(&payload[wi], word);
            }
            const uint32_t g = base + u * 256u + threadIdx.x;
            if (g < total_items) {
                stv<NT>(reinterpret_cast<V*>(cover + o0[u]), a0[u]);
                stv<NT>(reinterpret_cast<V*>(cover + o0[u] + W), a1[u]);
            }
        }
    }
    // odd H: the unpaired last row of every slice is copied verbatim
    if ((H & 1) && blockIdx.x == 0) {
        const uint32_t B = total_items / items_per_slice;
        for (uint32_t b = 0; b < B; ++b)
            for (int q = threadIdx.x; q < W; q += 256) cover[b * npx + (size_t)(H - 1) * W + q] = stego[b * npx + (size_t)(H - 1) * W + q];
    }
}


// ====================================================================== single pass
// Decoupled look-back (W % 8 == 0): a chunk = 4 tiles = 1024 items = 4096 candidates,
// handed out by an atomic ticket so that a chunk only ever waits on chunks that were
// handed out earlier (forward progress).  Each chunk publishes its count of expandable
// candidates (aggregate), looks back over its slice's predecessors (one wave reads 64
// status words per round) for its exclusive bit cursor, publishes the inclusive prefix
// and then embeds / recovers in registers: the cover is read once and the stego written
// once, and an in-place call touches only the chunks up to `end`.
#define PEE_CHUNK 1024                     // items per chunk
#define LB_AGG (1ull << 62)
#define LB_INC (2ull << 62)

__device__ __forceinline__ void lb_store(u64* p, u64 v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ u64 lb_load(u64* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t ld_agent(uint32_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// wave 0 of the block: exclusive prefix of chunk c (>= 1) from st[0..c-1].  The spin is
// bounded (spin_max polls).  Out of place the source buffer is never written, so a
// predecessor that has not published its aggregate by then (it would take out-of-order
// workgroup dispatch, or a workgroup that is not resident) has it computed from its pixels
// by this wave (`count`, e.g. EmbedCount) and published for the other waiters: the prefix
// is exact either way and *fallback is set (a diagnostic count).  In place (NoFallback) the
// predecessor may be rewriting its pixels, so a timeout sets *timeout and the caller flags
// the slice (sticky status, the host raises) instead of hanging the GPU.
// `done` (optional): the slice's finished flag.  It can only be set once every chunk before
// the one holding `end` has published, so a waiter that sees it set lies past `end` and
// returns `sat` (>= L) instead of waiting for predecessors that may never publish.
#ifndef PEE_LB_SLEEP
#define PEE_LB_SLEEP 1
#endif
struct NoFallback {
    static constexpr bool can = false;
    __device__ u64 operator()(int) const { return 0ull; }
};

// expandable, non-overflow candidates of chunk j (the embed's aggregate), counted by the
// calling wave (16 items per lane) and returned to every lane
template <typename T>
struct EmbedCount {
    static constexpr bool can = true;
    const T* src;
    int W, CR;
    uint32_t items;
    int Tthr, maxval;
    __device__ u64 operator()(int j) const {   // expandable | unsafe << 32 (a status word's value)
        typedef typename Vec8<T>::type V;
        const int lane = threadIdx.x & 63;
        uint32_t n = 0, un = 0;
        for (int u = 0; u < PEE_CHUNK / 64; ++u) {
            const uint32_t it = (uint32_t)j * PEE_CHUNK + (uint32_t)(u * 64 + lane);
            if (it >= items) break;
            const uint32_t r = it / (uint32_t)CR, cc = it - r * (uint32_t)CR;
            const size_t o0 = (size_t)(2 * r) * W + (size_t)cc * 8;
            const V v0 = *reinterpret_cast<const V*>(src + o0);
            const V v1 = *reinterpret_cast<const V*>(src + o0 + W);
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const PeeCand pc = pee_classify((int)get_px(v1, 2 * q + 1), (int)get_px(v1, 2 * q), (int)get_px(v0, 2 * q + 1),
                                                (int)get_px(v0, 2 * q), Tthr, maxval);
                n += (pc.expand && pc.safe) ? 1u : 0u;
                un += pc.safe ? 0u : 1u;
            }
        }
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) {
            n += __shfl_xor(n, o, 64);
            un += __shfl_xor(un, o, 64);
        }
        return (u64)n | ((u64)un << 32);
    }
};

// inner candidates of chunk j (the extract's aggregate): not in the location map, k <= end,
// -2T <= e' < 2T -- counted from the stego by the calling wave
template <typename T>
struct ExtractCount {
    static constexpr bool can = true;
    const T* src;
    const u64* lm;
    int W, CR;
    uint32_t items;
    int end, Tthr;
    __device__ u64 operator()(int j) const {
        typedef typename Vec8<T>::type V;
        const int lane = threadIdx.x & 63;
        uint32_t n = 0;
        for (int u = 0; u < PEE_CHUNK / 64; ++u) {
            const uint32_t it = (uint32_t)j * PEE_CHUNK + (uint32_t)(u * 64 + lane);
            if (it >= items || (int)(4 * it) > end) break;
            const uint32_t r = it / (uint32_t)CR, cc = it - r * (uint32_t)CR;
            const size_t o0 = (size_t)(2 * r) * W + (size_t)cc * 8;
            const V v0 = *reinterpret_cast<const V*>(src + o0);
            const V v1 = *reinterpret_cast<const V*>(src + o0 + W);
            const u64 lw = lm[(4 * it) >> 6] >> ((4 * it) & 63);
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                if ((int)(4 * it) + q > end || ((lw >> q) & 1ull)) continue;
                const int e2 = (int)get_px(v1, 2 * q + 1) - med3((int)get_px(v1, 2 * q), (int)get_px(v0, 2 * q + 1), (int)get_px(v0, 2 * q));
                n += (e2 >= -2 * Tthr && e2 < 2 * Tthr) ? 1u : 0u;
            }
        }
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) n += __shfl_xor(n, o, 64);
        return n;
    }
};

// One look-back round reads LB_WIN windows of 64 predecessor words at once (one memory round
// trip instead of LB_WIN): a chunk far from the slice's first one -- e.g. the 256 chunks of a
// lone 2048^2 slice spread over all CUs, whose predecessors have all published aggregates but
// few inclusive prefixes yet -- sums them in one round instead of one round per 64 chunks.
#ifndef LB_WIN
#define LB_WIN 4
#endif
// PEE_LB_DONE_POLL: a waiting embed chunk also polls the slice's finished flag (released as
// "past `end`" when the chunk that set it lies before it).  Measured (round 5, headline): off,
// the chunks past `end` wait out their predecessors' words instead -- k_pee_embed1 0.745 ->
// 0.79-0.80 ms; it stays on
// PEE_FIN_EARLY: out of place the chunk holding `end` sets the finished flag right after its
// look-back (before its embed loop) rather than at its end
#ifndef PEE_FIN_EARLY
#define PEE_FIN_EARLY 1
#endif
#ifndef PEE_LB_DONE_POLL
#define PEE_LB_DONE_POLL 1
#endif
#ifndef PEE_LB_PARTIAL
#define PEE_LB_PARTIAL 1   // embed: a partial sum of the published words may end the wait (past `end`)
#endif
// Status words carry two counts (round 4): bits 0-31 the chunk's (or prefix's) expandable /
// inner count, bits 32-55 its unsafe-candidate count (the embed's location-map bits, so the
// chunk holding `end` learns lm_count from the look-back itself: no meta atomics, no memset).
// The two fields are summed separately (64-bit each), so a sum can never carry between them.
// Bits 56-61 (self-cleaning calls only, round 5): the call's epoch tag, the low 6 bits of the
// chunk's arrival count.  A waiter accepts a word only with its own tag, so a word left by
// another call -- a chunk whose arrival count drifted from its slice's (a desynchronised
// workspace) reads the other parity's buffer -- is "not published" and the bounded spin ends
// in the pixel-count fallback: exact, never a stale prefix.  The high field then needs
// < 2^24 candidates per slice (PEE_SC_MAX_NC; larger slices take the zeroing path).
#define LB_LO(w) ((w) & 0xFFFFFFFFull)
#define LB_HI(w) (((w) >> 32) & 0xFFFFFFull)
#define LB_TAG_SHIFT 56
#define LB_TAGW(t) ((u64)(uint32_t)(t) << LB_TAG_SHIFT)
#define PEE_SC_MAX_NC ((1LL << 24) - 2)
struct LbSum {
    u64 e, u;   // summed low / high fields of the predecessors
};
__device__ __forceinline__ u64 wave_sum_u64(u64 v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
// The finished flag of a slice: written by the chunk holding `end` as fin_val (1, or the
// self-cleaning call's tag + 1, <= 64) in its low byte and that chunk's index + 1 above it.
// It tells chunk c "`end` lies before you" only when the recorded chunk is LOWER than c: the
// chunk holding `end` can finish before an earlier chunk has -- it needs only the earlier
// chunks' aggregates, and with the pixel-count fallback not even those -- so a set flag alone
// says nothing about chunks before it (round 5: a persistent grid that triggered the fallback
// made earlier chunks skip their bits).
__device__ __forceinline__ uint32_t pee_fin_word(uint32_t fin_val, int c) { return fin_val | ((uint32_t)(c + 1) << 8); }
__device__ __forceinline__ bool pee_fin_before(uint32_t w, uint32_t fin_val, int c) {
    // (w >> 8) in [1, c]: w - 256 wraps past every bound when the index field is 0
    return ((w & 0xFFu) == fin_val) & ((w - 256u) < ((uint32_t)c << 8));
}
// untagged calls (fin_val 1, the flag zeroed before the call: it holds 0 or 1 + 256 k): one
// compare, 0 wrapping past every bound
__device__ __forceinline__ bool pee_fin_before1(uint32_t w, int c) { return w - 257u < ((uint32_t)c << 8); }
// TWO: also sum the high field (the self-cleaning embed's unsafe counts); otherwise only the
// low one, as the zeroing paths need (fewer registers in the headline kernels).
// tag >= 0 (self-cleaning calls): only words carrying this epoch tag count as published, and
// the finished flag `done` counts as set only when it holds done_val (tag + 1 there) and names
// a chunk before c (pee_fin_before).
template <bool TWO = false, typename F>
__device__ LbSum lb_exclusive(u64* st, int c, bool* timeout, bool* fallback, uint32_t spin_max, const F& count,
                              uint32_t* done = nullptr, uint32_t sat = 0, int tag = -1, uint32_t done_val = 1u) {
    const int lane = threadIdx.x & 63;
    LbSum ex{0ull, 0ull};
    int p = c - 1;            // the highest predecessor not summed yet
    uint32_t spins = 0;
    const u64 tagw = tag >= 0 ? LB_TAGW(tag) : 0ull;
    for (;;) {
        u64 wv[LB_WIN];
#pragma unroll
        for (int r = 0; r < LB_WIN; ++r) {
            const int idx = p - 64 * r - lane;
            wv[r] = idx >= 0 ? lb_load(st + idx) : (LB_INC | tagw);
        }
        bool reload = false;
#pragma unroll
        for (int r = 0; r < LB_WIN; ++r) {   // the windows in order, from the loaded words
            const int pr = p - 64 * r;       // this window's top predecessor
            const int idx = pr - lane;
            u64 w = wv[r];
            uint32_t fl = (uint32_t)(w >> 62);
            if (tag >= 0 && (uint32_t)((w >> LB_TAG_SHIFT) & 63u) != (uint32_t)tag) fl = 0u;   // another call's word
            const u64 inc = __ballot(fl == 2u);
            const u64 notready = __ballot(fl == 0u);
            const int first = inc ? (int)__builtin_ctzll(inc) : 64;        // nearest inclusive
            const u64 need = first >= 63 ? ~0ull : ((2ull << first) - 1ull);  // lanes 0..first
            if (notready & need) {
#if PEE_LB_DONE_POLL
                if (done) {
                    const uint32_t dw = ld_agent(done);
                    if (tag >= 0 ? pee_fin_before(dw, done_val, c) : pee_fin_before1(dw, c)) return LbSum{(u64)sat, 0ull};
                }
#endif
                if (done && (PEE_LB_PARTIAL)) {
                    // the published words already bound the prefix from below (aggregates of
                    // disjoint chunks, or an inclusive prefix): reaching `sat` (= L) places this
                    // chunk past `end` without waiting for the missing ones
                    const u64 lo = wave_sum_u64((lane <= first && fl != 0u) ? LB_LO(w) : 0ull);
                    if (ex.e + lo >= sat) return LbSum{ex.e + lo, 0ull};
                }
                if (++spins <= spin_max) {
                    __builtin_amdgcn_s_sleep(PEE_LB_SLEEP);
                    p = pr;                  // reload from this window
                    reload = true;
                    break;
                }
                if constexpr (!F::can) {
                    *timeout = true;
                    return ex;
                } else {
                    // the missing aggregates from the pixels, one chunk per round of the wave; a
                    // chunk that published meanwhile keeps its own word (CAS from what was read)
                    u64 m = notready & need;
                    while (m) {
                        const int l = (int)__builtin_ctzll(m);
                        m &= m - 1ull;
                        const u64 a = count(pr - l);   // packed like a status word's value
                        if (lane == l) {
                            const u64 mine = LB_AGG | a | tagw;
                            atomicCAS(reinterpret_cast<unsigned long long*>(st + idx), (unsigned long long)w,
                                      (unsigned long long)mine);
                            w = mine;
                            fl = 1u;
                        }
                    }
                    *fallback = true;
                    spins = 0;
                }
            }
            if constexpr (TWO) {
                ex.e += wave_sum_u64(lane <= first ? LB_LO(w) : 0ull);
                ex.u += wave_sum_u64(lane <= first ? LB_HI(w) : 0ull);
            } else {   // 32-bit sums, as before the second field existed
                uint32_t v = lane <= first ? (uint32_t)w : 0u;
#pragma unroll
                for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
                ex.e += v;
            }
            if (first < 64) return ex;
            // embed (done != nullptr): a partial sum that already reaches `sat` (= L) places the
            // chunk past `end`; the caller only compares the prefix with L, and publishes it as a
            // saturated inclusive value, as the done-flag path does
            if (done && ex.e >= sat) return ex;
        }
        if (!reload) p -= 64 * LB_WIN;
    }
}

template <typename T, bool NT>
__device__ __forceinline__ void pee_load_chunk(const T* src, int W, int CR, uint32_t items, int c,
                                               typename Vec8<T>::type* a0, typename Vec8<T>::type* a1, size_t* o0) {
    typedef typename Vec8<T>::type V;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const uint32_t it = (uint32_t)c * PEE_CHUNK + u * 256u + threadIdx.x;
        if (it < items) {
            const uint32_t r = it / CR, cc = it - r * CR;
            o0[u] = (size_t)(2 * r) * W + (size_t)cc * 8;
            a0[u] = ldv<NT>(reinterpret_cast<const V*>(src + o0[u]));
            a1[u] = ldv<NT>(reinterpret_cast<const V*>(src + o0[u] + W));
        }
    }
}

// Slot v -> (slice b, chunk j).  Workgroups are observed to be dealt round-robin over the
// 8 XCDs (MI355X_MICROARCH.md: blocks b and b+8 share one), so slot lane x = v % 8 owns
// slices x, x+8, ...: a slice's chunks then start in order on one XCD and their per-slice
// tickets come back in slot order, which is what lets the speculative load of chunk j be
// the ticketed chunk (correctness never depends on it: the ticket decides the chunk).
// Out of place the lane walks its slices slice-major, in place chunk-major.
__device__ __forceinline__ bool pee_slot(uint32_t v, int B, int nchunks, int g8, int* b, int* j) {
    // g8 slice lanes per group: the groups follow one another, chunk-major inside a group
    // (g8 = B8: chunk-major over the batch; g8 = 1: slice-major).  g8 = 0 (PEE_MODE_FLAT,
    // small batches): slot v = slice-major over every XCD, the chunk then comes from the
    // per-slice ticket (a lone slice's chunks would otherwise all sit on one XCD)
    if (g8 == 0) {
        *b = (int)(v / (uint32_t)nchunks);
        *j = (int)(v - (uint32_t)*b * (uint32_t)nchunks);
        return *b < B;
    }
    const int x = (int)(v & 7u);
    const uint32_t k = v >> 3;
    const uint32_t per = (uint32_t)g8 * (uint32_t)nchunks;
    const uint32_t grp = k / per, r = k - grp * per;
    *j = (int)(r / (uint32_t)g8);
    const int bi = (int)(grp * (uint32_t)g8 + (r - (uint32_t)*j * g8));
    *b = x + 8 * bi;
    return *b < B;
}
#define PEE_MODE_FLAT 4
__host__ __device__ __forceinline__ int pee_group8(int B, int mode, bool inplace) {
    const int B8 = (B + 7) / 8;
    if (inplace) return B8;
    if (mode & PEE_MODE_FLAT) return 0;
    const int g = mode >> 8;
    if (g > 0) return g < B8 ? g : B8;
    return (mode & 1) ? B8 : 1;   // PEE_MODE_CMAJOR
}
__host__ __device__ __forceinline__ uint32_t pee_total_slots(int B, int nchunks, int g8) {
    if (g8 == 0) return (uint32_t)B * (uint32_t)nchunks;
    const int B8 = (B + 7) / 8;
    return 8u * (uint32_t)((B8 + g8 - 1) / g8 * g8) * (uint32_t)nchunks;
}

// ctl[0] = slices finished (in place); slice b: chunk ticket ctl[32 + 32 b], finished flag
// ctl[33 + 32 b] (one 128-byte line per slice: tickets of different slices never contend).
// Out of place: one workgroup per (slice, chunk) slot, slice-major.  In place: persistent
// workgroups walk the slots chunk-major, so a slice's later chunks are only reached after
// its earlier ones, and skip (without a ticket) once the slice is finished.
// launch mode of the out-of-place single pass: chunk-major slot order, and chunk = slot
// (no ticket).  Without the ticket the look-back's forward progress rests on in-order
// workgroup dispatch within an XCD (a slice's chunks all sit on one XCD, pee_slot): every
// predecessor of a resident workgroup has then been dispatched.  Should that ever fail,
// lb_exclusive's bounded spin falls back to counting the missing predecessors from their
// pixels (the cover is read-only out of place), so the result stays exact and nothing hangs.
// In place (ticketed: a predecessor always holds an earlier ticket and is resident) a
// timeout flags the slice with the sticky status CODEC_PEE_ELOOKBACK.
// dbg_skip >= 0 (CODEC_PEE_DEBUG_SKIP = chunk + 1, tests only): that chunk of slice 0 never
// publishes its aggregate/prefix, so its successors time out and take the fallback (out of
// place) or flag the slice (in place).
// diag[0] / diag[2]: chunks whose look-back used the pixel fallback / timed out unrecovered
// (cumulative since the workspace was zeroed; codec_pee_diag_offset).
// diagnostic build only (tools/lb_trace.py, -DPEE_LB_TRACE): thread 0 of every embed1
// workgroup stamps its slot's phases into LDS; threads 0..7 write them out per slot
#ifdef PEE_LB_TRACE
#define LB_TRACE_SLOTS 4096
__device__ unsigned long long g_lb_trace[LB_TRACE_SLOTS * 12];
#define LB_STAMP(k)                                                                     \
    do {                                                                                \
        unsigned long long t_;                                                          \
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");      \
        if (tid == 0) lbt[k] = t_;                                                      \
    } while (0)
#else
#define LB_STAMP(k) do { } while (0)
#endif
#define PEE_MODE_CMAJOR 1
#define PEE_MODE_NOTICKET 2
// self-cleaning out-of-place look-back (round 4): no zeroing launch before the pass.  The
// workspace holds TWO status-word buffers; a call uses buffer `par` and clears its own words
// of the other one for the next call.  The finished flag is doubled the same way; meta is
// written without atomics (status by the chunk holding `end`, lm_count from the look-back's
// second field).
// Round 5: the call's epoch comes from the host (the library counts self-cleaning calls per
// workspace, pee_ws_epoch) as a kernel argument, so every chunk of a call agrees on it by
// construction -- round 4 derived it from a per-chunk arrival counter, which a call abandoned
// mid-kernel could leave out of step with the slice's other chunks.  par = epoch & 1; every
// status word and finished flag also carries the epoch tag epoch % 63 + 1 (1..63), and a
// waiter accepts only its own tag: a word or flag left by any other call -- an abandoned one,
// a zeroing call (tag 0), a call whose clear never ran -- reads as "not published", so the
// worst a stale state can cost is the bounded wait and the pixel-count fallback, never a
// wrong prefix.  Calls that still zero (in place, ticket modes) use buffer 1 and flag 1 with
// tag 0.  A call captured into a graph would replay one epoch forever, so capture takes the
// zeroing path (codec_pee_embed_ts / codec_pee_extract).
#define PEE_MODE_SC 8
// ctl: 32 words, then 32 per slice (ticket, finished flags)
#define PEE_CTL_WORDS(B, NCH) (32 + 32 * (size_t)(B))
#define PEE_LINE_TICKET 0
#define PEE_LINE_FIN0 1
#define PEE_LINE_FIN1 4
__device__ __forceinline__ int pee_sc_tag(int epoch) { return epoch % 63 + 1; }
#define PEE_SKIP 0xFFFFFFFFu
#define PEE_STOP 0xFFFFFFFEu
// occupancy A/B (build-time, tools/r05/ab_occupancy.sh): minimum waves per SIMD for the
// look-back passes.  Measured: more waves per CU are slower (embed1 at 4: 0.738 -> 0.741 ms,
// extract1 at 5: 0.712 -> 0.733), and fewer (a dynamic-LDS pad) slower or equal
// (profiles/r05/ab_occupancy.txt, ab_ldspad.txt): the defaults stay.
#ifdef PEE_E1_WAVES
#define PEE_E1_LB __launch_bounds__(256, PEE_E1_WAVES)
#else
#define PEE_E1_LB __launch_bounds__(256)
#endif
#ifdef PEE_X1_WAVES
#define PEE_X1_LB __launch_bounds__(256, PEE_X1_WAVES)
#else
#define PEE_X1_LB __launch_bounds__(256)
#endif
template <typename T, bool NT, bool INPLACE, bool SC = false>
__global__ PEE_E1_LB void k_pee_embed1(const T* __restrict__ cover, T* stego, int H, int W, int T0,
                                                    int maxval, const int32_t* __restrict__ lengths,
                                                    const u64* __restrict__ payload_all, int pw, int nchunks, int B,
                                                    u64* status_all, uint32_t* ctl, codec_pee_meta* meta_all,
                                                    u64* __restrict__ lm_all, int lmw, int mode, uint32_t spin_max,
                                                    int dbg_skip, uint32_t* diag, const int32_t* __restrict__ tps,
                                                    int sc_epoch, int dbg_stale) {
    typedef typename Vec8<T>::type V;
    __shared__ u64 sh64[8];
    __shared__ uint32_t sh[8];
    __shared__ uint32_t s_v, s_excl, s_uexcl, s_uns[4];
    constexpr bool sc = !INPLACE && SC;   // self-cleaning: a separate instantiation (PEE_MODE_SC)
    __shared__ uint32_t lm32[4 * PEE_TILE / 32];
    __shared__ u64 s_pay[192];   // the slice's payload words when pw <= 192 (see below)
    const bool pay_st = pw <= 192;
#ifdef PEE_LB_TRACE
    __shared__ unsigned long long lbt[12];
#endif
    const int CR = W / 8;
    const uint32_t items = (uint32_t)(H / 2) * (uint32_t)CR;
    const int nc = (H / 2) * (W / 2);
    const int ntiles = (nc + PEE_TILE - 1) / PEE_TILE;
    const int g8 = pee_group8(B, mode, INPLACE);
    const uint32_t total = pee_total_slots(B, nchunks, g8);
    const size_t npx = (size_t)H * W;
    const int tid = threadIdx.x;
    for (uint32_t v = blockIdx.x; v < total; v += gridDim.x) {
        int b, j;
        if (!pee_slot(v, B, nchunks, g8, &b, &j)) continue;   // uniform; no barrier passed
        LB_STAMP(0);
        uint32_t* line = ctl + 32 + 32 * (size_t)b;
        uint32_t* tick = line + PEE_LINE_TICKET;
        const size_t stride = (size_t)B * nchunks;   // one status-word buffer
        const uint32_t L = (uint32_t)max(0, lengths[b]);
        const int Tthr = tps ? tps[b] : T0;   // per-slice threshold (capacity control) or one for all
        codec_pee_meta* M = meta_all + b;
        const T* src = cover + b * npx;
        T* dst = stego + b * npx;
        V a0[4], a1[4];
        size_t o0[4];
        // this call's status-word buffer, epoch tag and finished-flag value (self-cleaning:
        // from the host's epoch; zeroing calls: buffer 1, untagged, flag value 1)
        const int par = sc ? (sc_epoch & 1) : 1;
        const int tag = sc ? pee_sc_tag(sc_epoch) : -1;
        const u64 tagw = sc ? LB_TAGW(tag) : 0ull;
        const uint32_t fin_val = sc ? (uint32_t)tag + 1u : 1u;
        uint32_t* fin_flag = line + (par ? PEE_LINE_FIN1 : PEE_LINE_FIN0);
        // out of place the finished flag is read BEFORE the chunk's pixels are requested, so
        // waiting for it does not wait for the pixels too (vmcnt counts in issue order)
        const uint32_t dnA = !INPLACE ? ld_agent(fin_flag) : 0u;   // every lane
        // out of place: the slot's own chunk j is loaded while the ticket is in flight (the
        // ticket equals j unless workgroups were dispatched out of order)
        if (!INPLACE) pee_load_chunk<T, NT>(src, W, CR, items, j, a0, a1, o0);
        if (tid == 0) {
            uint32_t cc = PEE_SKIP;
            if (!INPLACE) {
                // a flag seen set was set before this chunk started, so `end` lies in an
                // earlier chunk; a flag set meanwhile but not seen only costs this chunk the
                // full path.  It counts only when it holds this call's value (tag + 1).
                cc = (mode & PEE_MODE_NOTICKET) ? (uint32_t)j : atomicAdd(tick, 1u);
                const bool dn = sc ? pee_fin_before(dnA, fin_val, (int)cc) : pee_fin_before1(dnA, (int)cc);
                if (dn) {   // `end` already placed: this chunk is a plain copy
                    lb_store(status_all + par * stride + (size_t)b * nchunks + cc, LB_INC | (u64)L | tagw);
                    cc |= 0x80000000u;
                }
            } else {
                // the two flag loads and the ticket go out together (one round trip); a ticket
                // taken for a finished slice is published as "prefix >= L" and skipped
                const uint32_t nd = ld_agent(ctl);
                const uint32_t dnw = ld_agent(line + PEE_LINE_FIN1);
                cc = atomicAdd(tick, 1u);
                const bool dn = pee_fin_before1(dnw, (int)cc);
                if (nd >= (uint32_t)B || dn) {
                    if (cc < (uint32_t)nchunks) lb_store(status_all + stride + (size_t)b * nchunks + cc, LB_INC | (u64)L);
                    cc = nd >= (uint32_t)B ? PEE_STOP : PEE_SKIP;
                }
            }
            s_v = cc;
        }
        if (tid < 4 * PEE_TILE / 32) lm32[tid] = 0;
        lds_barrier();
        LB_STAMP(1);
        const uint32_t cv = s_v;
        u64* st = status_all + par * stride + (size_t)b * nchunks;
        if (INPLACE) {
            if (cv == PEE_STOP) return;
            if (cv >= (uint32_t)nchunks) { lds_barrier(); continue; }
        }
        const bool copy_only = !INPLACE && (cv & 0x80000000u);
        const int c = (int)(cv & 0x7FFFFFFFu);
        if (sc && tid == 0) {   // clear this chunk's word (and chunk 0: the flag) of the next call's buffer
            // dbg_stale (tests): plant a stale but valid-looking state there instead -- an
            // inclusive prefix 0 and a set finished flag, both with this call's tag
            const bool stale = b == 0 && c == dbg_stale;
            lb_store(status_all + (1 - par) * stride + (size_t)b * nchunks + c, stale ? (LB_INC | tagw) : 0ull);
            if (c == 0 || stale)
                __hip_atomic_store(line + (par ? PEE_LINE_FIN0 : PEE_LINE_FIN1), stale ? pee_fin_word(fin_val, 0) : 0u,
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        if (INPLACE || c != j) pee_load_chunk<T, NT>(src, W, CR, items, c, a0, a1, o0);
        if (copy_only) {
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const uint32_t it = (uint32_t)c * PEE_CHUNK + u * 256u + tid;
                if (it < items) {
                    stv<NT>(reinterpret_cast<V*>(dst + o0[u]), a0[u]);
                    stv<NT>(reinterpret_cast<V*>(dst + o0[u] + W), a1[u]);
                }
            }
            if (tid < 64) {
                const int w = c * (4 * PEE_TILE / 64) + tid;
                if (w < lmw) lm_all[(size_t)b * lmw + w] = 0;
            }
            LB_STAMP(5);
            lds_barrier();
#ifdef PEE_LB_TRACE
            if (tid < 12 && v < LB_TRACE_SLOTS) g_lb_trace[v * 12 + tid] = (tid == 0 || tid == 1 || tid == 5) ? lbt[tid] : (tid == 10 ? 1ull : (unsigned long long)c);
            lds_barrier();
#endif
            continue;
        }
        uint32_t esm = 0, safem = 0, rightm = 0;   // bit 4u+q
        u64 packed = 0;
        uint32_t uns = 0;   // unsafe candidates (location-map bits when the chunk lies before `end`)
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const uint32_t it = (uint32_t)c * PEE_CHUNK + u * 256u + tid;
            if (it < items) {
                uint32_t n = 0;
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const PeeCand pc = pee_classify((int)get_px(a1[u], 2 * q + 1), (int)get_px(a1[u], 2 * q),
                                                    (int)get_px(a0[u], 2 * q + 1), (int)get_px(a0[u], 2 * q), Tthr, maxval);
                    const uint32_t bit = 1u << (4 * u + q);
                    if (pc.safe) safem |= bit;
                    if (pc.right) rightm |= bit;
                    if (pc.expand && pc.safe) { esm |= bit; ++n; }
                    if constexpr (sc) uns += pc.safe ? 0u : 1u;
                }
                packed |= (u64)n << (16 * u);
            }
        }
        if constexpr (sc) {   // the chunk's unsafe total: wave sums into LDS, read after the scan's barriers
            uint32_t ws = uns;
#pragma unroll
            for (int o = 32; o >= 1; o >>= 1) ws += __shfl_xor(ws, o, 64);
            if ((tid & 63) == 0) s_uns[tid >> 6] = ws;
        }
        u64 ptot;
        const u64 pex = block_excl_scan64_lds<256>(packed, sh64, &ptot);
        const uint32_t agg = (uint32_t)((ptot & 0xFFFFu) + ((ptot >> 16) & 0xFFFFu) + ((ptot >> 32) & 0xFFFFu) + (ptot >> 48));
        const uint32_t agg_u = sc ? s_uns[0] + s_uns[1] + s_uns[2] + s_uns[3] : 0u;
        const u64 aggw = (u64)agg | ((u64)agg_u << 32);   // the chunk's status-word value
        const bool publish = !(b == 0 && c == dbg_skip);
        LB_STAMP(2);
        // waves 1-3 (idle during wave 0's look-back) fetch the payload words into LDS meanwhile:
        // a dependent global round trip after the look-back is then an LDS read, and wave 0's
        // look-back loads -- the chain every later chunk waits on -- never wait behind them
        // (vmcnt is per wave).  Loading them in wave 0 too, before the look-back, slowed it.
        u64 pwv = 0;
        if (pay_st && tid >= 64) pwv = payload_all[(size_t)b * pw + min(tid - 64, pw - 1)];
        if (c == 0) {
            if (tid == 0) { if (publish) lb_store(st, LB_INC | aggw | tagw); s_excl = 0; s_uexcl = 0; }
        } else {
            if (tid == 0 && publish) lb_store(st + c, LB_AGG | aggw | tagw);
            if (tid < 64) {
                bool to = false, fb = false;
                LbSum ex;
                if (INPLACE) ex = lb_exclusive(st, c, &to, &fb, spin_max, NoFallback(), fin_flag, L);
                else ex = lb_exclusive<sc>(st, c, &to, &fb, spin_max, EmbedCount<T>{src, W, CR, items, Tthr, maxval}, fin_flag, L,
                                           tag, fin_val);
                if (tid == 0) {
                    if constexpr (sc) {
                        // inclusive prefix; past `end` saturated to L (successors only compare it with L)
                        const u64 ie = ex.e + agg;
                        const u64 iu = (ex.u + agg_u) & 0xFFFFFFull;
                        if (publish) lb_store(st + c, LB_INC | (ie >= L ? (u64)L : ie) | (iu << 32) | tagw);
                        s_excl = (uint32_t)min(ex.e, (u64)0xFFFFFFFFull);
                        s_uexcl = (uint32_t)ex.u;
                    } else {
                        if (publish) lb_store(st + c, LB_INC | (u64)(uint32_t)(ex.e + agg));
                        s_excl = (uint32_t)ex.e;
                    }
                    // sticky: the status words are only ever raised (atomicMax) after this
                    if (to) { atomicMax(&M->status, CODEC_PEE_ELOOKBACK); atomicAdd(diag + 2, 1u); }
                    if (fb) atomicAdd(diag, 1u);
                }
            }
        }
        if (pay_st && tid >= 64 && tid - 64 < pw) s_pay[tid - 64] = pwv;
        lds_barrier();
        LB_STAMP(3);
        const uint32_t excl = s_excl;
        const uint32_t uexcl = s_uexcl;
        const bool last = c == nchunks - 1;
        if (tid == 0) {
            if (c == 0) {
                M->T = Tthr; M->maxval = maxval; M->L = (int)L; M->nc = nc; M->ntiles = ntiles; M->h = H; M->w = W;
                if (L == 0) { M->end = -1; M->tile_end = -1; }   // status: below (out of place) / memset (in place)
                if (sc) M->reserved[0] = M->reserved[1] = M->reserved[2] = 0;
            }
            // the chunk holding `end` (or the last one on overflow) reports the capacity seen so
            // far: exact when it is the last chunk, else a lower bound (later chunks are not counted)
            const bool fin = (excl < L && excl + agg >= L) || (L == 0 && c == 0) || (last && excl + agg < L);
            if (fin) {
                M->capacity = (int)(excl + agg);
                M->flags = last ? 0 : CODEC_PEE_PARTIAL;
                // out of place the flag goes up as soon as this chunk knows it holds `end`: the
                // chunks past it only read the flag (nothing of this chunk's data), so they are
                // released before this chunk's embed loop instead of after it
                if (!INPLACE && PEE_FIN_EARLY)
                    __hip_atomic_store(fin_flag, pee_fin_word(fin_val, c), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            if (last && excl + agg < L) {
                M->end = nc - 1;
                M->tile_end = ntiles - 1;
                if (!sc) atomicMax(&M->status, 1);
            }
        }
        lds_barrier();   // lm32 zeroing vs the ORs below
        LB_STAMP(6);
        uint32_t nun = 0;
        if (excl < L) {   // some candidate of this chunk is active
            uint32_t base = excl;
            uint32_t unsafe_n = 0;
            const u64* payload = payload_all + (size_t)b * pw;
            // an item's expandable candidates take consecutive ranks [rs, rs + n): the payload
            // words holding them (one, or two across a word boundary) are loaded for all four
            // items up front instead of one dependent load per embedded bit
            uint32_t rs[4];
            u64 plo[4], phi[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                rs[u] = base + (uint32_t)((pex >> (16 * u)) & 0xFFFFu);
                base += (uint32_t)((ptot >> (16 * u)) & 0xFFFFu);
                const uint32_t n = (uint32_t)((packed >> (16 * u)) & 0xFFFFu);
                const uint32_t w = rs[u] >> 6;
                const bool any = n && rs[u] < L;
                const bool two = any && (rs[u] & 63u) + n > 64u && (int)w + 1 < pw;
                plo[u] = any ? (pay_st ? s_pay[w] : payload[w]) : 0ull;
                phi[u] = two ? (pay_st ? s_pay[w + 1] : payload[w + 1]) : 0ull;
            }
            // the payload words are waited for here, once: their uses sit in the divergent
            // candidate branches below, where hipcc otherwise waited vmcnt(0) lgkmcnt(0) --
            // i.e. for every store this chunk had issued -- at each use (~4 us per chunk)
#pragma unroll
            for (int u = 0; u < 4; ++u)
                asm volatile("" ::"v"((uint32_t)plo[u]), "v"((uint32_t)(plo[u] >> 32)), "v"((uint32_t)phi[u]),
                             "v"((uint32_t)(phi[u] >> 32)));
            // branch-free per item (a divergent candidate loop with a global store inside cost
            // ~4 us per chunk): this item's expandable candidates take ranks [rs, rs + n), the
            // first m = min(L - rs, 4) of them carry bits, and candidate q is processed iff
            // fewer than m expandable candidates precede it in the item
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const uint32_t it = (uint32_t)c * PEE_CHUNK + u * 256u + tid;
                const bool ok = it < items;
                const uint32_t eb = (esm >> (4 * u)) & 15u, sb = (safem >> (4 * u)) & 15u, rb = (rightm >> (4 * u)) & 15u;
                const uint32_t rsu = rs[u];
                const uint32_t mcnt = (ok & (rsu < L)) ? min(L - rsu, 4u) : 0u;
                const uint32_t o = rsu & 63u;
                const u64 field = o ? ((plo[u] >> o) | (phi[u] << (64u - o))) : plo[u];
                uint32_t procm = 0, nib = 0;
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const uint32_t bit = 1u << q;
                    const uint32_t pre = (uint32_t)__popc(eb & (bit - 1u));
                    const bool proc = pre < mcnt;
                    procm |= proc ? bit : 0u;
                    nib |= (proc & !(sb & bit)) ? bit : 0u;
                    const int x = (int)get_px(a1[u], 2 * q + 1);
                    const int pr = med3((int)get_px(a1[u], 2 * q), (int)get_px(a0[u], 2 * q + 1), (int)get_px(a0[u], 2 * q));
                    const int nv_e = 2 * x - pr + (int)((field >> pre) & 1ull);   // p + 2e + bit
                    const int nv_s = (rb & bit) ? x + Tthr : x - Tthr;
                    const int nv = (proc & ((sb & bit) != 0u)) ? ((eb & bit) ? nv_e : nv_s) : x;
                    set_px(a1[u], 2 * q + 1, (uint32_t)nv);
                }
                unsafe_n += (uint32_t)__popc(nib);
                // the item holding rank L - 1 (1 <= L - rs <= n): `end` is its last processed
                // expandable candidate (status stays 0: zeroed before the pass)
                if (mcnt != 0u && L - rsu <= (uint32_t)__popc(eb)) {
                    const int k = (int)(4 * it) + 31 - __clz(procm & eb);
                    M->end = k;
                    M->tile_end = k / PEE_TILE;
                }
                if (nib) __hip_atomic_fetch_or(&lm32[u * 32 + (tid >> 3)], nib << (4 * (tid & 7)), __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_WORKGROUP);
                if (INPLACE && procm) stv<NT>(reinterpret_cast<V*>(dst + o0[u] + W), a1[u]);
            }
            LB_STAMP(7);
            nun = block_sum_u32_lds<256>(unsafe_n, sh);   // also orders the lm32 ORs
            LB_STAMP(8);
            if (!sc && tid == 0 && nun) atomicAdd(&M->lm_count, (int)nun);
        }
        LB_STAMP(4);
        if (tid == 0) {   // `end` is in this chunk (or there is none): later chunks need no cursor
            const bool fin = (excl < L && excl + agg >= L) || (L == 0 && c == 0) || (last && excl + agg < L);
            if (fin) {
                if (INPLACE || !PEE_FIN_EARLY)
                    __hip_atomic_store(fin_flag, pee_fin_word(fin_val, c), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (INPLACE) atomicAdd(ctl, 1u);
                if (sc) {   // no meta atomics (nothing zeroed it): the chunk holding `end` writes them
                    M->status = (last && excl + agg < L) ? 1 : 0;
                    M->lm_count = (int)(uexcl + nun);
                }
            }
        }
        if (!INPLACE) {
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const uint32_t it = (uint32_t)c * PEE_CHUNK + u * 256u + tid;
                if (it < items) {
                    stv<NT>(reinterpret_cast<V*>(dst + o0[u]), a0[u]);
                    stv<NT>(reinterpret_cast<V*>(dst + o0[u] + W), a1[u]);
                }
            }
        }
        // location-map words of this chunk (zeros past `end`); in place only where active
        if (!INPLACE || excl < L) {
            if (tid < 64) {
                const int w = c * (4 * PEE_TILE / 64) + tid;
                if (w < lmw) lm_all[(size_t)b * lmw + w] = (u64)lm32[2 * tid] | ((u64)lm32[2 * tid + 1] << 32);
            }
        }
        LB_STAMP(5);
        lds_barrier();
#ifdef PEE_LB_TRACE
        if (tid < 12 && v < LB_TRACE_SLOTS) g_lb_trace[v * 12 + tid] = tid < 10 ? lbt[tid] : (tid == 10 ? 0ull : (unsigned long long)c);
        lds_barrier();
#endif
    }
}

// The extract's read-ahead (self-cleaning payload writes): the bits of the first `need` (1..63)
// inner candidates at or after item it0, in rank order, as the low bits of a u64 -- what
// the following chunks will recover, computed from their (read-only) stego pixels and map
// words.  One wave, 4 items per lane per round.  The first round's loads are issued early
// (load(), at the chunk's start, so they land during the look-back); bits() consumes them
// and runs further rounds only if those 256 items held fewer than `need` inner candidates.
template <typename T>
struct PeeReadAhead {
    typedef typename Vec8<T>::type V;
    V v0[4], v1[4];
    u64 lw[4];
    __device__ __forceinline__ void load(const T* src, const u64* lm, int W, int CR, uint32_t items, uint32_t itb) {
        const int lane = threadIdx.x & 63;
#pragma unroll
        for (int u = 0; u < 4; ++u) {   // clamped addresses: every load is valid
            const uint32_t it = min(itb + (uint32_t)(u * 64 + lane), items - 1u);
            const uint32_t r = it / (uint32_t)CR, cc = it - r * (uint32_t)CR;
            const size_t o = (size_t)(2 * r) * W + (size_t)cc * 8;
            v0[u] = *reinterpret_cast<const V*>(src + o);
            v1[u] = *reinterpret_cast<const V*>(src + o + W);
            lw[u] = lm[(4 * it) >> 6];
        }
    }
    __device__ u64 bits(const T* src, const u64* lm, int W, int CR, uint32_t items, int end, int Tthr, uint32_t it0,
                        uint32_t need) {
        const int lane = threadIdx.x & 63;
        u64 ra = 0ull;
        uint32_t got = 0;
        for (uint32_t itb = it0; got < need && itb < items && (int)(4 * itb) <= end; itb += 256u) {   // uniform
            if (itb != it0) load(src, lm, W, CR, items, itb);
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const uint32_t it = itb + (uint32_t)(u * 64 + lane);
                const u64 mw = lw[u] >> ((4 * it) & 63);
                uint32_t pk = 0, n = 0;
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const int k = (int)(4 * it) + q;
                    const int x = (int)get_px(v1[u], 2 * q + 1);
                    const int e2 = x - med3((int)get_px(v1[u], 2 * q), (int)get_px(v0[u], 2 * q + 1), (int)get_px(v0[u], 2 * q));
                    const bool inner = it < items && k <= end && !((mw >> q) & 1ull) && e2 >= -2 * Tthr && e2 < 2 * Tthr;
                    pk |= (inner ? (uint32_t)(e2 & 1) : 0u) << n;
                    n += inner ? 1u : 0u;
                }
                const uint32_t incl = wave_incl_scan(n);
                const uint32_t pos = got + incl - n;
                u64 contrib = pos < 64u ? (u64)pk << pos : 0ull;
#pragma unroll
                for (int o = 32; o >= 1; o >>= 1) contrib |= __shfl_xor(contrib, o, 64);
                ra |= contrib;
                got += (uint32_t)__shfl(incl, 63, 64);
            }
        }
        return need >= 64u ? ra : (ra & ((1ull << need) - 1ull));
    }
};

// extract: chunks up to the one holding `end` recover bits + pixels (look-back over the
// inner-candidate counts); later chunks are a plain copy (out of place) or skipped.
template <typename T, bool NT, bool INPLACE, bool SC = false>
__global__ PEE_X1_LB void k_pee_extract1(const T* stego, T* cover, int H, int W,
                                                      const codec_pee_meta* __restrict__ meta_all,
                                                      const u64* __restrict__ lm_all, int lmw, int nchunks, int B,
                                                      u64* status_all, uint32_t* ctl, u64* __restrict__ payload_all,
                                                      int pw, int mode, uint32_t spin_max, int dbg_skip, uint32_t* diag,
                                                      int sc_epoch, int dbg_stale) {
    typedef typename Vec8<T>::type V;
    __shared__ u64 sh64[8];
    __shared__ uint32_t s_v, s_excl;
    __shared__ int s_cmax;
    __shared__ u64 s_ra;
    // self-cleaning (PEE_MODE_SC, small out-of-place batches): status words by call parity, and
    // the payload written without atomics or a zeroed buffer -- every word by the chunk holding
    // its first bit, which reads the word's later bits ahead from the following chunks' pixels
    constexpr bool sc = !INPLACE && SC;   // a separate instantiation: the read-ahead's registers
    const size_t stride = (size_t)B * nchunks;
    // the chunk's recovered bits: ranks [excl, excl + agg), agg <= 4096, from word excl / 64
    __shared__ u64 pbuf[PEE_CHUNK * 4 / 64 + 2];
    const int CR = W / 8;
    const uint32_t items = (uint32_t)(H / 2) * (uint32_t)CR;
    const size_t npx = (size_t)H * W;
    const int tid = threadIdx.x;
    const int g8 = pee_group8(B, mode, INPLACE);
    const uint32_t total = pee_total_slots(B, nchunks, g8);
    int cmax = nchunks - 1;
    if (INPLACE) {   // chunk-major slots: nothing past the last chunk any slice needs
        if (tid == 0) s_cmax = -1;
        lds_barrier();
        int cm = -1;
        for (int b = tid; b < B; b += 256) {
            const int e = meta_all[b].end;
            cm = max(cm, e >= 0 ? (e >> 2) / PEE_CHUNK : -1);
        }
        if (cm >= 0) atomicMax(&s_cmax, cm);
        lds_barrier();
        cmax = s_cmax;
    }
    for (uint32_t v = blockIdx.x; v < total; v += gridDim.x) {
        int b, j;
        const bool valid = pee_slot(v, B, nchunks, g8, &b, &j);
        if (j > cmax) return;                           // in place: a lane's chunks only grow
        if (!valid) continue;
        const codec_pee_meta* M = meta_all + b;
        const int end = M->end, Tthr = M->T;
#ifdef PEE_X_COPYONLY   // diagnostic build (tools): every chunk a plain copy
        const int cend = -1;
        (void)end;
#else
        const int cend = end >= 0 ? (end >> 2) / PEE_CHUNK : -1;
#endif
        if (INPLACE && j > cend) continue;              // uniform: no barrier passed yet
        const T* src = stego + b * npx;
        T* dst = cover + b * npx;
        V a0[4], a1[4];
        size_t o0[4];
        // out of place chunk j is loaded while the ticket is in flight (a plain copy when past
        // `end`); in place only the ticketed chunk is read
        if (!INPLACE) pee_load_chunk<T, NT>(src, W, CR, items, j, a0, a1, o0);
        const u64* lm = lm_all + (size_t)b * lmw;
        const bool noticket = !INPLACE && (mode & PEE_MODE_NOTICKET);
        u64 lwv[4] = {0, 0, 0, 0};   // location-map word of each item (4 bits of it used)
        if (noticket && j <= cend) {   // the chunk is known: its map words go out with its pixels
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const uint32_t it = (uint32_t)j * PEE_CHUNK + u * 256u + tid;
                if (it < items) lwv[u] = lm[(4 * it) >> 6];
            }
        }
        // the read-ahead's first round (wave 1): the first 256 items after this chunk, issued
        // behind the chunk's own loads so that they land while wave 0 looks back (used only if
        // this chunk's last payload word is incomplete; c == j without tickets)
        PeeReadAhead<T> rah;
        if (sc && j < cend && tid >= 64 && tid < 128) rah.load(src, lm, W, CR, items, (uint32_t)(j + 1) * PEE_CHUNK);
        int c = j;
        if (j <= cend && !noticket) {   // exactly cend+1 slots take tickets 0..cend
            if (tid == 0) s_v = atomicAdd(ctl + 32 + 32 * (size_t)b, 1u);
            lds_barrier();
            c = (int)s_v;
            if (INPLACE || c != j) pee_load_chunk<T, NT>(src, W, CR, items, c, a0, a1, o0);
        }
        // status-word buffer and epoch tag (calls that zero first use buffer 1, untagged)
        const int par = sc ? (sc_epoch & 1) : 1;
        const int tag = sc ? pee_sc_tag(sc_epoch) : -1;
        const u64 tagw = sc ? LB_TAGW(tag) : 0ull;
        if (sc) {
            if (tid == 0) {
                // the next call's word (dbg_stale, tests: a stale inclusive prefix 0 instead)
                lb_store(status_all + (1 - par) * stride + (size_t)b * nchunks + j,
                         (b == 0 && j == dbg_stale) ? (LB_INC | tagw) : 0ull);
                // the in-place look-back flag (codec_pee_extract_flag_offset) reads clear after
                // this call: an earlier in-place call may have set it, out of place nothing does
                if (b == 0 && j == 0) __hip_atomic_store(ctl + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                // the next call's finished flag (an embed's) starts clear: every self-cleaning
                // call clears the other parity's flag, whichever kernel it is
                if (j == 0)
                    __hip_atomic_store(ctl + 32 + 32 * (size_t)b + (par ? PEE_LINE_FIN0 : PEE_LINE_FIN1), 0u,
                                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
        if (c <= cend) {
            uint32_t actm = 0, innm = 0;
            u64 packed = 0;
            if (!noticket) {   // the map words of the ticketed chunk, all four in flight at once
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const uint32_t it = min((uint32_t)c * PEE_CHUNK + u * 256u + tid, items - 1u);
                    lwv[u] = lm[(4 * it) >> 6];
                }
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const uint32_t it = (uint32_t)c * PEE_CHUNK + u * 256u + tid;
                if (it >= items) continue;
                const u64 lw = lwv[u] >> ((4 * it) & 63);   // 4 bits, same word
                uint32_t n = 0;
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const int k = (int)(4 * it) + q;
                    if (k > end || ((lw >> q) & 1ull)) continue;
                    actm |= 1u << (4 * u + q);
                    const int p = med3((int)get_px(a1[u], 2 * q), (int)get_px(a0[u], 2 * q + 1), (int)get_px(a0[u], 2 * q));
                    const int e2 = (int)get_px(a1[u], 2 * q + 1) - p;
                    if (e2 >= -2 * Tthr && e2 < 2 * Tthr) { innm |= 1u << (4 * u + q); ++n; }
                }
                packed |= (u64)n << (16 * u);
            }
            if (tid < PEE_CHUNK * 4 / 64 + 2) pbuf[tid] = 0;   // ordered by the scan's barriers
            u64 ptot;
            const u64 pex = block_excl_scan64_lds<256>(packed, sh64, &ptot);
            const uint32_t agg = (uint32_t)((ptot & 0xFFFFu) + ((ptot >> 16) & 0xFFFFu) + ((ptot >> 32) & 0xFFFFu) + (ptot >> 48));
            u64* st = status_all + par * stride + (size_t)b * nchunks;
            const bool publish = c < cend && !(b == 0 && c == dbg_skip);
            if (c == 0) {
                if (tid == 0) { if (publish) lb_store(st, LB_INC | (u64)agg | tagw); s_excl = 0; }
            } else {
                if (tid == 0 && publish) lb_store(st + c, LB_AGG | (u64)agg | tagw);
                if (tid < 64) {
                    bool to = false, fb = false;
                    LbSum ex;
                    if (INPLACE) ex = lb_exclusive(st, c, &to, &fb, spin_max, NoFallback());
                    else ex = lb_exclusive(st, c, &to, &fb, spin_max, ExtractCount<T>{src, lm, W, CR, items, end, Tthr},
                                           nullptr, 0u, sc ? tag : -1);
                    if (tid == 0) {
                        if (publish) lb_store(st + c, LB_INC | ((ex.e + agg) & 0xFFFFFFFFull) | tagw);
                        s_excl = (uint32_t)ex.e;
                        if (to) { atomicOr(ctl + 1, 1u); atomicAdd(diag + 3, 1u); }   // codec_pee_extract_flag_offset
                        if (fb) atomicAdd(diag + 1, 1u);
                    }
                }
            }
            lds_barrier();
            const uint32_t excl = s_excl;
            const int w0 = (int)(excl >> 6);
            uint32_t base = excl;
            u64* payload = payload_all + (size_t)b * pw;
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                uint32_t r = base + (uint32_t)((pex >> (16 * u)) & 0xFFFFu);
                base += (uint32_t)((ptot >> (16 * u)) & 0xFFFFu);
                // branch-free per item: the item's inner candidates take ranks [r, r + n), n <= 4;
                // their bits are gathered into one nibble and OR-ed into at most two words
                const uint32_t am = (actm >> (4 * u)) & 0xFu, im = (innm >> (4 * u)) & 0xFu;
                uint32_t bits = 0;
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const uint32_t bit = 1u << q;
                    const int x = (int)get_px(a1[u], 2 * q + 1);
                    const int p = med3((int)get_px(a1[u], 2 * q), (int)get_px(a0[u], 2 * q + 1), (int)get_px(a0[u], 2 * q));
                    const int e2 = x - p;
                    const bool inner = (im & bit) != 0u;
                    bits |= (inner ? (uint32_t)(e2 & 1) : 0u) << __popc(im & (bit - 1u));
                    const int nx = inner ? p + (e2 >> 1) : (e2 >= 2 * Tthr ? x - Tthr : x + Tthr);
                    set_px(a1[u], 2 * q + 1, (uint32_t)((am & bit) ? nx : x));
                }
                if (bits) {
                    const uint32_t o = r & 63u;
                    const int wl = (int)(r >> 6) - w0;
                    __hip_atomic_fetch_or(&pbuf[wl], (u64)bits << o, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    if (o > 60u && (bits >> (64u - o)))
                        __hip_atomic_fetch_or(&pbuf[wl + 1], (u64)(bits >> (64u - o)), __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_WORKGROUP);
                }
                if (INPLACE && am) stv<NT>(reinterpret_cast<V*>(dst + o0[u] + W), a1[u]);
            }
            // one store per payload word instead of a global atomic per item: words wholly
            // inside [excl, excl + agg) belong to this chunk alone; the first and last may be
            // shared with the neighbouring chunks (OR-ed in); the host zeroed the payload
            lds_barrier();
            const int nw = (int)(((excl & 63u) + agg + 63u) >> 6);
            const uint32_t f = excl + agg;
            if (!sc) {
                if (tid < nw) {
                    const u64 wv = pbuf[tid];
                    if (wv) {
                        const bool shared = (tid == 0 && (excl & 63u)) || (tid == nw - 1 && (f & 63u));
                        if (shared) atomicOr(&payload[w0 + tid], wv);
                        else payload[w0 + tid] = wv;
                    }
                }
            } else {
                // self-cleaning: this chunk writes the words that START in [excl, f) whole; the
                // last one's bits past f come from the following chunks (read ahead from their
                // pixels by wave 1, ranks f .. next word boundary); the word holding excl, when
                // excl is not word-aligned, is the previous owner's.  The chunk holding `end`
                // zeroes the words after its last one.
                const bool ahead = c < cend && (f & 63u) != 0u;   // uniform
                if (ahead) {
                    if (tid >= 64 && tid < 128) {
                        const u64 ra = rah.bits(src, lm, W, CR, items, end, Tthr, (uint32_t)(c + 1) * PEE_CHUNK,
                                                64u - (f & 63u));
                        if (tid == 64) s_ra = ra;
                    }
                    lds_barrier();
                }
                if (tid < nw) {
                    const int w = w0 + tid;
                    const bool owned = tid > 0 || (excl & 63u) == 0u;
                    if (owned && w < pw) {
                        u64 wv = pbuf[tid];
                        if (ahead && tid == nw - 1) wv |= s_ra << (f & 63u);
                        payload[w] = wv;
                    }
                }
                if (c == cend)
                    for (int w = (int)((f + 63u) >> 6) + tid; w < pw; w += 256) payload[w] = 0ull;
            }
        } else if (sc && c == 0 && cend < 0) {   // no embedded bit at all: the payload is zero
            u64* payload = payload_all + (size_t)b * pw;
            for (int w = tid; w < pw; w += 256) payload[w] = 0ull;
        }
        if (!INPLACE) {
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const uint32_t it = (uint32_t)c * PEE_CHUNK + u * 256u + tid;
                if (it < items) {
                    stv<NT>(reinterpret_cast<V*>(dst + o0[u]), a0[u]);
                    stv<NT>(reinterpret_cast<V*>(dst + o0[u] + W), a1[u]);
                }
            }
        }
        lds_barrier();
    }
}

// ====================================================================== slice-serial single pass
// For batches that fill the chip (B >= the CU count and a near multiple of it): one
// 1024-thread workgroup per slice streams that slice's chunks (1024 items = 4096
// candidates = 32 KB of uint16) in order.  The running count of expandable candidates is
// a register of the workgroup -- no look-back, no status words, no ticket, nothing to
// memset -- and D chunks of pixels are in flight per workgroup (a register ring refilled
// right after each chunk).  The payload words of a wave's rank range are wave-uniform
// loads (scalar cache, lgkmcnt), so waiting for them never drains the vector-load ring.
// A static LDS pad keeps exactly one workgroup per CU: one contiguous region streamed per
// CU is the fastest order this chip copies in (DESIGN §3, 6.2 TB/s).  In place a slice
// stops after the chunk holding `end`; out of place the chunks past `end` are copied and
// only counted (exact capacity).
//
// Why the code is shaped the way it is: hipcc counts vmcnt precisely only through
// straight-line vector memory code.  Every vector load and store of a chunk is therefore
// unconditional -- loads of lanes/chunks past the end read a clamped valid address,
// stores that must not land are redirected to a per-lane sink in the workspace -- and the
// only branches left in the ring loop contain no vector memory instruction.  Barriers are
// LDS-only (raw s_barrier): __syncthreads()'s fence waits vmcnt(0).
#define SS_THREADS 1024
#ifndef SS_LOCKSTEP
#define SS_LOCKSTEP 1   // copy chunks: a barrier every SS_LOCKSTEP chunks keeps the waves in step
#endif
// diagnostic build only (tools/ss_trace.py, -DPEE_SS_TRACE): workgroup 0, wave 0 stamps the
// chunk phases into LDS (no vector memory in the loop) and writes them out at the end
#ifdef PEE_SS_TRACE
#define SS_TRACE_N 2048
__device__ unsigned long long g_ss_trace[SS_TRACE_N];
// slot i of wave w: ss_trace[w * 128 + i - 4 * K0] (chunks K0 .. K0+31 traced)
#ifndef PEE_SS_TRACE_K0
#define PEE_SS_TRACE_K0 0
#endif
#define SS_STAMP(i)                                                                           \
    do {                                                                                      \
        unsigned long long t_;                                                                \
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");          \
        const int j_ = (i) - 4 * PEE_SS_TRACE_K0;                                             \
        if ((threadIdx.x & 63) == 0 && j_ >= 0 && j_ < 128) ss_trace[(threadIdx.x >> 6) * 128 + j_] = t_; \
    } while (0)
#else
#define SS_STAMP(i) do { } while (0)
#endif
#define SS_PAD_WORDS (21 * 1024)     // 84 KB of the CU's 160 KB: a second workgroup does not fit
#define SS_PAY_WORDS (SS_PAD_WORDS / 2 - 1)   // the embed keeps payloads of up to 10 751 words in that pad
// sink for stores that must not land: one 64-B slot per wave (two 16-B pixel vectors and one
// 8-B word), shared by the wave's lanes -- a store instruction whose lanes all go to the sink
// touches one line instead of 64 (per-lane slots made the extract's mostly-sunk payload-word
// stores scatter over 64 lines per wave and chunk)
#define SS_SINK_SLOT(b, tid) ((size_t)((b) * (SS_THREADS / 64) + ((tid) >> 6)) * 64)
#define SS_SINK_BYTES(B) ((size_t)(B) * (SS_THREADS / 64) * 64)


// wave-level primitives without LDS round trips (each __shfl is a ds_bpermute, ~100 cycles):
// OR over the 16 lanes of a DPP row, and an exclusive scan of 0..7 per lane from three ballots
__device__ __forceinline__ uint32_t row_or16(uint32_t v) {
    v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false);    // quad_perm [1,0,3,2]
    v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xF, 0xF, false);    // quad_perm [2,3,0,1]
    v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x141, 0xF, 0xF, false);   // row_half_mirror
    v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x140, 0xF, 0xF, false);   // row_mirror
    return v;
}
__device__ __forceinline__ u64 row_or16_64(u64 v) {
    return (u64)row_or16((uint32_t)v) | ((u64)row_or16((uint32_t)(v >> 32)) << 32);
}
__device__ __forceinline__ uint32_t mbcnt64(u64 m) {   // set bits of m below this lane
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}
// n in 0..7 per lane -> exclusive prefix within the wave, and the wave's total
__device__ __forceinline__ uint32_t wave_excl_small(uint32_t n, uint32_t* total) {
    const u64 b0 = __ballot(n & 1u), b1 = __ballot(n & 2u), b2 = __ballot(n & 4u);
    *total = (uint32_t)(__popcll(b0) + 2 * __popcll(b1) + 4 * __popcll(b2));
    return mbcnt64(b0) + 2u * mbcnt64(b1) + 4u * mbcnt64(b2);
}

// exclusive scan of n (0..7) over the 1024 threads with ONE barrier and no shuffles: ballot
// scans inside the waves, wave totals through LDS (double-buffered by parity: a wave cannot
// rewrite wtot[par] before every wave has passed the next barrier).  The 16 wave totals are
// scanned across the 16 lanes of each DPP row (4 row_shr adds) and the wave's base and the
// block total read back with readlane into scalars: 8 VALU instead of 16 per-lane sums.
__device__ __forceinline__ void ss_scan_small(uint32_t n, uint32_t (*wtot)[16], int par, uint32_t* excl, uint32_t* tot,
                                              uint32_t* wbase) {
    const int lane = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    uint32_t wt;
    const uint32_t ex = wave_excl_small(n, &wt);
    if (lane == 0) wtot[par][wv] = wt;
    lds_barrier();
    int x = (int)wtot[par][lane & 15];
    x += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xF, 0xF, true);   // row_shr:1 (lane 0 of a row reads 0)
    x += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xF, 0xF, true);   // row_shr:2
    x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xF, 0xF, true);   // row_shr:4
    x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xF, 0xF, true);   // row_shr:8
    const uint32_t t = (uint32_t)__builtin_amdgcn_readlane(x, 15);
    const uint32_t wb = wv ? (uint32_t)__builtin_amdgcn_readlane(x, wv - 1) : 0u;
    *excl = wb + ex;
    *tot = t;
    *wbase = wb;
}

// item -> element offset of its 8-pixel column chunk in the top row of its row pair, advanced
// chunk by chunk without divisions or multiplies: item + 1024 moves (row pair, column chunk)
// by (1024 / CR, 1024 % CR) with at most one carry, i.e. the offset by a fixed step plus a
// fixed wrap correction.  Lanes/chunks past the end load a clamped valid address (data
// unused): straight-line loads let hipcc count vmcnt exactly.
struct SsCursor {
    uint32_t cc, o;
    __device__ __forceinline__ void init(uint32_t it, uint32_t CR, uint32_t W) {
        const uint32_t rr = it / CR;
        cc = it - rr * CR;
        o = 2u * rr * W + 8u * cc;
    }
    // ostep = 2 W (1024 / CR) + 8 (1024 % CR), owrap = 2 W - 8 CR (uniform)
    __device__ __forceinline__ void step(uint32_t dr, uint32_t CR, uint32_t ostep, uint32_t owrap) {
        cc += dr;
        o += ostep;
        const bool wrap = cc >= CR;
        cc = wrap ? cc - CR : cc;
        o = wrap ? o + owrap : o;
    }
};

template <typename T, bool NT>
__device__ __forceinline__ void ss_load_at(const T* src, uint32_t W, uint32_t o0, typename Vec8<T>::type& x0,
                                           typename Vec8<T>::type& x1) {
    typedef typename Vec8<T>::type V;
    x0 = ldv<NT>(reinterpret_cast<const V*>(src + o0));
    x1 = ldv<NT>(reinterpret_cast<const V*>(src + o0 + W));
}

// exclusive scan of n over the 1024 threads with ONE barrier (wave totals double-buffered
// by parity: a wave cannot rewrite wtot[par] before every wave has passed the next barrier)
__device__ __forceinline__ void ss_scan(uint32_t n, uint32_t (*wtot)[16], int par, uint32_t* excl, uint32_t* tot,
                                        uint32_t* wbase) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint32_t inc = wave_incl_scan(n);
    if (lane == 63) wtot[par][wv] = inc;
    lds_barrier();
    uint32_t wb = 0, t = 0;
#pragma unroll
    for (int w = 0; w < 16; ++w) {
        const uint32_t v = wtot[par][w];
        t += v;
        wb += w < wv ? v : 0u;
    }
    *excl = wb + inc - n;
    *tot = t;
    *wbase = wb;
}

// counters of the fused capacity phase (AUTO): the top tmax * 1024 words of the pad, below
// its last word; the payload (PAY_LDS) sits at the bottom
#define SS_AUTO_CNT_BASE(tmax) (SS_PAD_WORDS - 1 - (tmax) * SS_THREADS)
#define SS_AUTO_TMAX 16

// AUTO (capacity control fused in, codec_pee_embed_auto): before embedding, the workgroup
// streams its whole slice once and builds the capacity histogram of k_pee_ehist in
// lane-private LDS counters, then takes the smallest T <= tmax whose capacity holds the
// slice's payload (pee_select_slice's rule).  The embed that follows re-reads the slice from
// the MALL (C3: 134 MB batch); no second launch, no global histogram, no arrival counter.
// NTS: the stores' cache policy (default: the loads'); in place plain stores -- the candidate
// rows go back into lines the chunk has just read -- beat non-temporal ones by 11 % (embed) and
// 15 % (extract) at 256 x 2048^2 (profiles/r05/ab_policy.txt), out of place they lose
template <typename T, bool NT, bool INPLACE, int D, bool PAY_LDS, bool AUTO = false, bool NTS = NT>
__global__ __launch_bounds__(SS_THREADS) void k_pee_embed_ss(const T* __restrict__ cover, T* stego, int H, int W, int T0,
                                                             int maxval, const int32_t* __restrict__ lengths,
                                                             const int32_t* __restrict__ tps,
                                                             const u64* __restrict__ payload_all, int pw,
                                                             codec_pee_meta* __restrict__ meta_all,
                                                             u64* __restrict__ lm_all, int lmw, char* __restrict__ sink,
                                                             int tmax, int32_t* __restrict__ t_out) {
    typedef typename Vec8<T>::type V;
    __shared__ uint32_t ss_pad[SS_PAD_WORDS];
    __shared__ uint32_t wtot[2][16];
    __shared__ uint32_t red[2][16];
    __shared__ int s_end;
    __shared__ uint32_t s_bins[AUTO ? PEE_TMAX_MAX : 1];
    __shared__ int s_T;
#ifdef PEE_SS_TRACE
    __shared__ unsigned long long ss_trace[SS_TRACE_N];
#endif
    const int b = blockIdx.x;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int CR = W / 8;
    const uint32_t items = (uint32_t)(H / 2) * (uint32_t)CR;
    const int nchunks = (int)((items + SS_THREADS - 1) / SS_THREADS);
    const int nc = (H / 2) * (W / 2);
    const int ntiles = (nc + PEE_TILE - 1) / PEE_TILE;
    const uint32_t L = (uint32_t)max(0, lengths[b]);
    int Tthr = tps ? tps[b] : T0;
    const size_t npx = (size_t)H * W;
    const T* src = cover + b * npx;
    T* dst = stego + b * npx;
    const u64* payload = payload_all + (size_t)b * pw;
    u64* lm = lm_all + (size_t)b * lmw;
    V* sink_v = reinterpret_cast<V*>(sink + SS_SINK_SLOT(b, tid));
    u64* sink_w = reinterpret_cast<u64*>(sink + SS_SINK_SLOT(b, tid) + 32);
    u64* pay = reinterpret_cast<u64*>(ss_pad);   // PAY_LDS: the slice's payload words
    if (tid == 0) {
        s_end = -1;
        ss_pad[SS_PAD_WORDS - 1] = 0u;   // the occupancy pad stays allocated
    }
    V r0[D], r1[D];
    // cursors of this lane's item in the current chunk and in the chunk D ahead (the refill)
    const uint32_t dq = SS_THREADS / (uint32_t)CR, dr = SS_THREADS % (uint32_t)CR;
    const uint32_t ostep = 2u * (uint32_t)W * dq + 8u * dr, owrap = 2u * (uint32_t)W - 8u * (uint32_t)CR;
    uint32_t off_last;
    {
        SsCursor l;
        l.init(items - 1u, (uint32_t)CR, (uint32_t)W);
        off_last = l.o;
    }
    if constexpr (AUTO) {
        // capacity phase: 4 items per thread per step, their 8 loads issued together; plain
        // loads (the embed below re-reads the slice), lane-private counters (no barrier)
        uint32_t* cnt = ss_pad + SS_AUTO_CNT_BASE(tmax);
        for (int u = 0; u < tmax; ++u) cnt[u * SS_THREADS + tid] = 0u;
        constexpr int U = 4;
        SsCursor cur;
        cur.init((uint32_t)tid, (uint32_t)CR, (uint32_t)W);
        for (uint32_t it = (uint32_t)tid; it < items; it += SS_THREADS * U) {
            V a0[U], a1[U];
            bool in[U];
#pragma unroll
            for (int k = 0; k < U; ++k) {
                in[k] = it + (uint32_t)(SS_THREADS * k) < items;
                ss_load_at<T, false>(src, (uint32_t)W, in[k] ? cur.o : 0u, a0[k], a1[k]);
                cur.step(dr, (uint32_t)CR, ostep, owrap);
            }
#pragma unroll
            for (int k = 0; k < U; ++k) {
                int x[4], a[4], bb[4], cc[4];
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    x[q] = (int)get_px(a1[k], 2 * q + 1); a[q] = (int)get_px(a1[k], 2 * q);
                    bb[q] = (int)get_px(a0[k], 2 * q + 1); cc[q] = (int)get_px(a0[k], 2 * q);
                }
                ehist_add4<SS_THREADS>(cnt, tid, x, a, bb, cc, in[k] ? 4 : 0, tmax, maxval);
            }
        }
    }
    // ro[d]: the offset ring slot d was loaded from (= the item's store offset)
    uint32_t ro[D];
    SsCursor ahead;
    ahead.init((uint32_t)tid, (uint32_t)CR, (uint32_t)W);
    uint32_t it_a = (uint32_t)tid;
#pragma unroll
    for (int d = 0; d < D; ++d) {
        ro[d] = it_a < items ? ahead.o : off_last;
        ss_load_at<T, NT>(src, (uint32_t)W, ro[d], r0[d], r1[d]);
        ahead.step(dr, (uint32_t)CR, ostep, owrap);
        it_a += SS_THREADS;
    }
    if constexpr (AUTO) {
        // the ring's first loads are in flight (they do not depend on T): reduce the counters
        uint32_t* cnt = ss_pad + SS_AUTO_CNT_BASE(tmax);
        lds_barrier();
        // bin u: wave u % 16 sums the 1024 lane counters (16 per lane, then the wave)
        for (int u = wv; u < tmax; u += SS_THREADS / 64) {
            uint32_t s = 0;
#pragma unroll
            for (int j = 0; j < SS_THREADS / 64; ++j) s += cnt[u * SS_THREADS + j * 64 + lane];
#pragma unroll
            for (int o = 32; o >= 1; o >>= 1) s += __shfl_xor(s, o, 64);
            if (lane == 0) s_bins[u] = s;
        }
        lds_barrier();
        if (tid == 0) {   // pee_select_slice's rule: the smallest T whose capacity >= L, else tmax
            long long run = 0;
            int tsel = 0;
            for (int t = 1; t <= tmax; ++t) {
                run += (long long)s_bins[t - 1];
                if (!tsel && run >= (long long)L) tsel = t;
            }
            s_T = tsel ? tsel : tmax;
            if (t_out) t_out[b] = s_T;
        }
        lds_barrier();
        Tthr = s_T;
    }
    if (PAY_LDS) {   // the payload in LDS once: no dependent global round trip per chunk
        const int nw = min(pw, (int)((L + 63u) >> 6));
        for (int w = tid; w < nw; w += SS_THREADS) pay[w] = payload[w];
        lds_barrier();
    }
    uint32_t running = 0, rest = 0, unsafe_n = 0;
    int par = 0, last = -1;
    bool live = L > 0;   // uniform: the chunk holding bit L-1 is still to come

    // one chunk, processed in the ring registers, then the ring slot is refilled.  D == 1
    // (EARLY): the chunk's data is taken into working registers and the slot refilled at
    // once, so the next chunk's loads are in flight through this chunk's scan barrier and
    // compute (tools/ubench_inplace.hip: "early ring 1" streams the in-place pattern ~3 %
    // faster than a ring of 2 refilled after the stores, with the same one chunk of reads
    // wasted past `end`)
    constexpr bool EARLY = D == 1;
    auto refill = [&](int d) {
        // in place, once `end` is reached the rest of the group refills from one clamped
        // address (L2 hits): the group still runs to its end, see the loop below
        ro[d] = it_a < items && (!INPLACE || live) ? ahead.o : off_last;
        ss_load_at<T, NT>(src, (uint32_t)W, ro[d], r0[d], r1[d]);
        ahead.step(dr, (uint32_t)CR, ostep, owrap);
        it_a += SS_THREADS;
    };
    auto chunk = [&](int d, int k) {
        V w0, w1;
        if constexpr (EARLY) { w0 = r0[d]; w1 = r1[d]; }
        V& v0 = EARLY ? w0 : r0[d];
        V& v1 = EARLY ? w1 : r1[d];
        const uint32_t it = (uint32_t)k * SS_THREADS + tid;
        const bool ok = it < items;
        const uint32_t o0 = ro[d];
        SS_STAMP(4 * k);
        // the chunk's registers are waited for here, once, outside any branch (an empty asm
        // reading them): the compiler then counts vmcnt exactly around the branches below
        asm volatile("" ::"v"(v0.x), "v"(v1.x));
        if constexpr (EARLY) refill(d);
        SS_STAMP(4 * k + 1);
        uint32_t wm = 0;
        bool touched = false;
        const bool was_live = live;
        if (live) {   // uniform; no vector memory instruction inside
            uint32_t esm = 0, safem = 0;
            int pq[4];
            bool eb[4], sb[4], rb[4];   // per-candidate lane masks (SGPR pairs) for the selects below
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const PeeCand pc = pee_classify((int)get_px(v1, 2 * q + 1), (int)get_px(v1, 2 * q), (int)get_px(v0, 2 * q + 1),
                                                (int)get_px(v0, 2 * q), Tthr, maxval);
                pq[q] = pc.p;
                eb[q] = pc.expand;
                sb[q] = pc.safe;
                rb[q] = pc.right;
                safem |= pc.safe ? 1u << q : 0u;
                esm |= (pc.expand & pc.safe) ? 1u << q : 0u;
            }
            if (!ok) esm = 0u;
            const uint32_t n = (uint32_t)__popc(esm);
            last = k;
            uint32_t ex, tot, wb;
            ss_scan_small(n, wtot, par, &ex, &tot, &wb);
            SS_STAMP(4 * k + 2);
            par ^= 1;
            // this lane's expandable candidates take ranks [rs, rs + n): their payload bits
            // are one <= 4-bit field of at most two consecutive 32-bit payload words; the
            // first m of them carry bits, and candidate q is processed iff fewer than m
            // expandable candidates precede it in the lane
            const uint32_t rs = running + ex;
            const uint32_t m = (ok & (L > rs)) ? min(L - rs, 4u) : 0u;
            uint32_t field;
            if (PAY_LDS) {
                const uint32_t* pay32 = reinterpret_cast<const uint32_t*>(pay);
                const uint32_t w = min(rs >> 5, 2u * (uint32_t)SS_PAY_WORDS - 2u);
                field = __builtin_amdgcn_alignbit(pay32[w + 1], pay32[w], rs & 31u);
            } else {
                // wave-uniform scalar loads: the wave's ranks lie in [running + wb, +256)
                const uint32_t w0 = __builtin_amdgcn_readfirstlane((running + wb) >> 6);
                u64 pwd[6];
#pragma unroll
                for (int i = 0; i < 6; ++i) pwd[i] = (w0 + (uint32_t)i < (uint32_t)pw) ? payload[w0 + i] : 0ull;
                const uint32_t wi = (rs >> 6) - w0, sh = rs & 63u;       // 0..4
                const u64 lo = wi == 0 ? pwd[0] : wi == 1 ? pwd[1] : wi == 2 ? pwd[2] : wi == 3 ? pwd[3] : pwd[4];
                const u64 hi = wi == 0 ? pwd[1] : wi == 1 ? pwd[2] : wi == 2 ? pwd[3] : wi == 3 ? pwd[4] : pwd[5];
                field = (uint32_t)(sh ? (lo >> sh) | (hi << (64u - sh)) : lo);
            }
            uint32_t procm = 0;
#pragma unroll
            for (int q = 0; q < 4; ++q) {   // branch-free
                const uint32_t bit = 1u << q;
                const uint32_t pre = (uint32_t)__popc(esm & (bit - 1u));
                const bool proc = pre < m;
                procm |= proc ? bit : 0u;
                const int x = (int)get_px(v1, 2 * q + 1);
                const int nv_e = 2 * x - pq[q] + (int)((field >> pre) & 1u);   // p + 2e + bit
                const int nv_s = rb[q] ? x + Tthr : x - Tthr;
                const int nv = (proc & sb[q]) ? (eb[q] ? nv_e : nv_s) : x;
                set_px(v1, 2 * q + 1, (uint32_t)nv);
            }
            touched = procm != 0;
            // the lane holding rank L-1 (1 <= L - rs <= n): `end` is its last processed
            // expandable candidate; one lane of the slice, once
            if (m != 0 && L - rs <= n) s_end = (int)(4 * it) + 31 - __clz(procm & esm);
            const uint32_t nib = procm & ~safem;
            unsafe_n += (uint32_t)__popc(nib);
            // location-map word (4 it) / 64 = 16 lanes x 4 candidate bits: each half is the
            // OR over 8 lanes (two quad permutes + a half-row mirror), stored as a 32-bit word
            // by lanes 0 and 8 of the DPP row
            wm = nib << (4 * (lane & 7));
            wm |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)wm, 0xB1, 0xF, 0xF, false);    // quad_perm [1,0,3,2]
            wm |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)wm, 0x4E, 0xF, 0xF, false);    // quad_perm [2,3,0,1]
            wm |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)wm, 0x141, 0xF, 0xF, false);   // row_half_mirror
            running += tot;
            if (running >= L) live = false;
        } else if (SS_LOCKSTEP && (k % SS_LOCKSTEP) == SS_LOCKSTEP - 1) {
            // past `end` (out of place) the chunk is a plain copy: not classified (capacity
            // stays a lower bound, CODEC_PEE_PARTIAL, as on the look-back path).  Without a
            // barrier the oldest waves (scheduled first) run ahead and finish, and the youngest
            // stream the slice's tail alone with a quarter of the loads in flight
            // (tools/ss_trace.py: 0.37 ms of drift by chunk 100; 0.80 -> 0.74 ms with it)
            lds_barrier();
        }
        // stores, unconditional (lanes 0 / 8 of a DPP row store the map word's low / high half)
        const uint32_t wix = (4 * it) >> 6;
        *(ok && (!INPLACE || was_live) && (lane & 7) == 0 && (int)wix < lmw
              ? reinterpret_cast<uint32_t*>(lm + wix) + ((lane >> 3) & 1)
              : reinterpret_cast<uint32_t*>(sink_w)) = wm;
        if (INPLACE) {
            stv<NTS>(ok && touched ? reinterpret_cast<V*>(dst + o0 + W) : sink_v, v1);
        } else {
            stv<NTS>(ok ? reinterpret_cast<V*>(dst + o0) : sink_v, v0);
            stv<NTS>(ok ? reinterpret_cast<V*>(dst + o0 + W) : sink_v + 1, v1);
        }
        if constexpr (!EARLY) refill(d);
        SS_STAMP(4 * k + 3);
    };

    // Full groups of D chunks, no guard around any chunk.  In place the loop is left only
    // at the end of a group (a chunk past `end` is a no-op): an exit after any chunk is
    // folded by the CFG structurizer into the loop latch, and hipcc's vmcnt bookkeeping then
    // merges the exit paths into the loop header's state (vmcnt(2) instead of (14): every
    // D-th chunk waited for the loads issued one chunk earlier).
    const int nfull = nchunks / D * D;
    for (int k0 = 0; k0 < nfull; k0 += D) {
#pragma unroll
        for (int d = 0; d < D; ++d) chunk(d, k0 + d);
        if (INPLACE && !live) break;
    }
    if (!INPLACE || live) {
#pragma unroll
        for (int d = 0; d < D; ++d)
            if (nfull + d < nchunks && (!INPLACE || live)) chunk(d, nfull + d);
    }
    // lm_count and the capacity past `end`: one block reduction
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
        unsafe_n += __shfl_xor(unsafe_n, o, 64);
        rest += __shfl_xor(rest, o, 64);
    }
    if (lane == 0) { red[0][wv] = unsafe_n; red[1][wv] = rest; }
    lds_barrier();
#ifdef PEE_SS_TRACE
    if (b == 0)
        for (int i = tid; i < SS_TRACE_N; i += SS_THREADS) g_ss_trace[i] = ss_trace[i];
#endif
    if (tid == 0) {
        uint32_t un = 0, re = 0;
        for (int w = 0; w < 16; ++w) { un += red[0][w]; re += red[1][w]; }
        codec_pee_meta* M = meta_all + b;
        const uint32_t cap = running + re;   // re = 0: chunks past `end` are not counted
        M->T = Tthr; M->maxval = maxval; M->L = (int)L; M->nc = nc; M->ntiles = ntiles; M->h = H; M->w = W;
        M->lm_count = (int)un;
        M->capacity = (int)cap;
        // the count stops with the chunk holding `end`: a lower bound unless it was the last
        M->flags = last < nchunks - 1 ? CODEC_PEE_PARTIAL : 0;
        M->reserved[0] = M->reserved[1] = M->reserved[2] = 0;
        if (L == 0) { M->end = -1; M->tile_end = -1; M->status = 0; }
        else if (running < L) { M->end = nc - 1; M->tile_end = ntiles - 1; M->status = 1; }   // truncated
        else { M->end = s_end; M->tile_end = s_end / PEE_TILE; M->status = 0; }
    }
}

// ---- resident fused auto embed (out of place, uint16, small slices: C3 / C4 at 512^2) ----
// k_pee_embed_ss<..., AUTO> streams a slice twice: a capacity pass (histogram of folded
// errors -> T), then the embed at T re-reads it (PMC: 1.43x the algorithmic bytes at C3).
// Here the slice is read ONCE and kept on the CU in between: a 512-thread workgroup (two
// waves per SIMD, up to 256 VGPRs per lane) keeps, per item, the odd row's 16-B vector (the
// candidates x and their W neighbours a) and the 4 prediction errors clamped to 8 bits
// (exact wherever they are used: expansion needs |e| < T <= 16, shifting only the sign) in
// registers -- 20 B per item, 5 VGPRs, NI items per lane.  The even rows hold no candidate,
// so the read phase writes them to the stego at once (their writes overlap the reads);
// after T is chosen, the embed phase rewrites only the odd rows, from registers: no load.
// HBM traffic = read cover + write stego, the algorithmic bytes.
#define RES_THREADS 512
#define RES_WAVES (RES_THREADS / 64)
#define RES_PAD_WORDS (24 * 1024)   // 96 KB static pad: one workgroup per CU
// LIN (1024 threads): the kept error words live in LDS ([NI][1024] below the counters, which
// are 16-bit pairs [8][1024]): 16 VGPRs fewer per lane -- at 128 VGPRs the register-kept
// words spilled, and each scratch reload made the embed phase wait for every store in flight
#define RES_PAD_WORDS_LIN (28 * 1024)
#define RES_CNT_BASE(tmax) (RES_PAD_WORDS - (tmax) * RES_THREADS)

// read phase: an LDS-only barrier every RES_LOCKSTEP items keeps the waves in step (without
// it the oldest ran ahead and the slice's last items were streamed by a few waves): C3 embed
// 0.0540 -> 0.0494 ms at 1 or 2 (profiles/r03/lockstep_ab.log); 0 = none
#ifndef RES_LOCKSTEP
#define RES_LOCKSTEP 1
#endif
#ifndef RES_ELOCK
#define RES_ELOCK 0   // embed phase: the same every RES_ELOCK items (build-time A/B)
#endif
#ifndef RES_G1024
#define RES_G1024 2   // the same at 1024 threads (build-time A/B: 1 ties, 3 and 4 are slower once the
                      // read phase runs in lockstep, profiles/r03/c3_res_depth_ab.log)
#endif
#ifndef RES_G
#define RES_G 4   // items per thread in flight ahead of the one processed (read phase)
#endif
// inclusive scan over the wave: 16-lane rows by row_shr, then rows by row_bcast:15 / :31
__device__ __forceinline__ uint32_t wave_incl_dpp(uint32_t x) {
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xF, 0xF, true);   // row_shr:1
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xF, 0xF, true);   // row_shr:2
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xF, 0xF, true);   // row_shr:4
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xF, 0xF, true);   // row_shr:8
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xA, 0xF, false);  // row_bcast:15 -> rows 1, 3
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xC, 0xF, false);  // row_bcast:31 -> rows 2, 3
    return x;
}
// The resident embed's kept error byte per candidate: bits 0-5 the error clamped to
// [-32, 30] (6-bit two's complement; exact wherever used: expansion needs |e| < T <= 16 and a
// shift only the side of +-T, with room for the payload bit: e + 1 stays in 6 bits), bit 6
// "near" (a shift of up to tmax towards e's side could leave [0, maxval]), bit 7 = the
// expansion stays in [0, maxval - 1] (both independent of T).  The embed phase works on the
// four bytes of an item at once (SWAR) with masks in the bytes' bit 7.
__device__ __forceinline__ uint32_t res_opaque(uint32_t x) {   // keeps shift/add forms: left
    asm("" : "+v"(x));                                         // free, hipcc folded them into
    return x;                                                  // quarter-rate multiplies
}
// expandable: folded error u = e >= 0 ? e : -e - 1 (XOR of the low 5 bits with the sign) < T
// (bit 7 of (u | 0x80) - T: no borrow between bytes, u <= 31, T <= 16)
__device__ __forceinline__ uint32_t res_ex_bytes(uint32_t ep, int T) {
    const uint32_t s5 = ep & 0x20202020u;
    const uint32_t m = res_opaque(s5) - (s5 >> 5);                  // sign ? 0x1F : 0 per byte
    const uint32_t u = ((ep ^ m) & 0x1F1F1F1Fu) | 0x80808080u;
    return ~(u - (uint32_t)T * 0x01010101u) & 0x80808080u;
}
// bytes' bit 7 -> byte q = number of set bits in bytes below q (0..3)
__device__ __forceinline__ uint32_t res_prefix(uint32_t b7) {
    const uint32_t e1 = b7 >> 7;
    const uint32_t i1 = res_opaque(e1 << 8) + e1;
    const uint32_t incl = res_opaque(i1 << 16) + i1;
    return incl << 8;
}
__device__ __forceinline__ uint32_t res_nibble(uint32_t b7) {           // bytes' bit 7 -> 4 bits
    return ((b7 >> 7) & 1u) | ((b7 >> 14) & 2u) | ((b7 >> 21) & 4u) | ((b7 >> 28) & 8u);
}
__device__ __forceinline__ int res_med3(int x, int lo, int hi) {
    int r;
    asm("v_med3_i32 %0, %1, %2, %3" : "=v"(r) : "v"(x), "v"(lo), "v"(hi));
    return r;
}
// the capacity histogram from an item's kept bytes: lane-private counters [tmax][NTH] (no
// bank conflicts), bin min(u, tmax - 1) += (u < tmax) & expansion safe, one LDS add per
// candidate (no return; candidates of one item sharing a bin need no merge)
template <int NTH, bool PACK = false>
__device__ __forceinline__ void res_hist4(uint32_t* cnt, int tid, uint32_t ep, bool in, int tmax) {
    const uint32_t s5 = ep & 0x20202020u;
    const uint32_t u_b = (ep ^ (res_opaque(s5) - (s5 >> 5))) & 0x1F1F1F1Fu;
    const uint32_t c_b = ~((u_b | 0x80808080u) - (uint32_t)tmax * 0x01010101u) & ep & (in ? 0x80808080u : 0u);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const uint32_t u = min(__builtin_amdgcn_ubfe(u_b, 8 * q, 5), (uint32_t)tmax - 1u);
        if constexpr (PACK)   // bins 2i and 2i + 1 as the halves of word i (a lane counts <= 64 per bin)
            __hip_atomic_fetch_add(cnt + (u >> 1) * NTH + tid, __builtin_amdgcn_ubfe(c_b, 8 * q + 7, 1) << (16 * (u & 1)),
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        else
            __hip_atomic_fetch_add(cnt + u * NTH + tid, __builtin_amdgcn_ubfe(c_b, 8 * q + 7, 1), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_WORKGROUP);
    }
}

// phase stamps (CODEC_PEE_RES_TRACE=1, diagnostics only): per workgroup wall_clock64() at
// entry, end of the read phase, T chosen, end of the embed phase (codec_debug_res_trace)
#define RES_TRACE_WG 1024
__device__ unsigned long long g_res_trace[RES_TRACE_WG * 5];
#define RES_STAMP(i)                                                                          \
    do {                                                                                      \
        if (trace && tid == 0 && b < RES_TRACE_WG) g_res_trace[b * 5 + (i)] = wall_clock64(); \
    } while (0)

// LIN: every lane's items are in range and item k + 1 lies a fixed offset KS after item k
// (NTH a multiple of the items per row pair, items a multiple of NTH: e.g. 512^2 at 1024
// threads): no cursor, no lane masks, no sink; the location-map halves are zeroed in the read
// phase by the lanes that may later write them (same lane, same address: ordered), so the
// embed phase stores a map word only where a wave has an unsafe candidate (rare), and the
// lane-exclusive ranks stay in registers
template <int NI, bool NT, bool NTS, int NTH, bool LIN = false>
__global__ __launch_bounds__(NTH) void k_pee_embed_res(const uint16_t* __restrict__ cover,
                                                               uint16_t* __restrict__ stego, int H, int W, int maxval,
                                                               const int32_t* __restrict__ lengths,
                                                               const u64* __restrict__ payload_all, int pw,
                                                               codec_pee_meta* __restrict__ meta_all,
                                                               u64* __restrict__ lm_all, int lmw, char* __restrict__ sink,
                                                               int tmax, int32_t* __restrict__ t_out, int trace) {
    typedef uint4 V;
    constexpr int NWV = NTH / 64;
    static_assert(NWV <= 16, "wave totals are scanned along one DPP row");
    static_assert(NI % 8 == 0, "pass A packs four items per word, the wave bases four word pairs per scan");
    constexpr int PADW = LIN ? RES_PAD_WORDS_LIN : RES_PAD_WORDS;
    __shared__ uint32_t pad[PADW];
    __shared__ uint32_t s_wt[NI / 2][NWV];   // embed phase: wave totals of the packed counters
    __shared__ uint32_t s_wb[NI / 2][NWV];    // embed phase: wave bases of the packed counters
    __shared__ uint32_t s_cb[NI];                   // embed phase: rank of each chunk's first candidate
    __shared__ uint32_t s_tot[NI / 2];              // embed phase: chunk totals (16-bit pairs)
    __shared__ uint32_t red[NWV];
    __shared__ uint32_t s_bins[SS_AUTO_TMAX];
    __shared__ int s_end, s_T;
    __shared__ uint32_t s_cap;
    const int b = blockIdx.x;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int CR = W / 8;
    const uint32_t items = (uint32_t)(H / 2) * (uint32_t)CR;
    const int nc = (H / 2) * (W / 2);
    const int ntiles = (nc + PEE_TILE - 1) / PEE_TILE;
    const size_t npx = (size_t)H * W;
    const uint16_t* src = cover + b * npx;
    uint16_t* dst = stego + b * npx;
    u64* lm = lm_all + (size_t)b * lmw;
    V* sink_v = reinterpret_cast<V*>(sink + SS_SINK_SLOT(b, tid));
    uint32_t* sink_w = reinterpret_cast<uint32_t*>(sink + SS_SINK_SLOT(b, tid) + 32);
    RES_STAMP(0);
    const int crow = LIN ? (tmax + 1) / 2 : tmax;   // counter rows (LIN: 16-bit pairs)
    uint32_t* cnt = pad + (PADW - crow * NTH);      // lane-private capacity counters [crow][NTH]
    uint32_t* s_re = pad + (PADW - (8 + NI) * NTH);   // LIN: kept error words [NI][NTH]
    const u64* payload = payload_all + (size_t)b * pw;
    u64* pay = reinterpret_cast<u64*>(pad);       // the slice's payload words
    const uint32_t dq = NTH / (uint32_t)CR, dr = NTH % (uint32_t)CR;
    const uint32_t ostep = 2u * (uint32_t)W * dq + 8u * dr, owrap = 2u * (uint32_t)W - 8u * (uint32_t)CR;
    // LIN: item k of this lane at o_lin + k KS (the host checked dr == 0, items % NTH == 0)
    const uint32_t KS = ostep;
    const uint32_t o_lin = 2u * ((uint32_t)tid / (uint32_t)CR) * (uint32_t)W + 8u * ((uint32_t)tid % (uint32_t)CR);
    // LIN: this lane's location-map half for item k (lanes 8j own one 32-bit half; others: sink)
    uint32_t* const lm_half = (lane & 7) == 0 ? reinterpret_cast<uint32_t*>(lm + (tid >> 4)) + ((lane >> 3) & 1) : sink_w;
    const uint32_t lm_step = (lane & 7) == 0 ? (NTH / 16) * 2 : 0u;   // 32-bit words per k

    // ---- read phase: every item once; even row -> stego now, odd row + errors kept
    uint32_t L;   // the slice's payload bits: read once the first loads are out
    V r1[NI];
    uint32_t re[LIN ? 1 : NI];
    {
        // G items per thread in flight ahead of the one processed: item k + G is issued just
        // before item k is processed (a ring of G + 1 even-row vectors)
        constexpr int G = NTH == 1024 ? RES_G1024 : RES_G;   // 4 waves per SIMD: half the registers, as many loads in flight per CU
        V v0[G + 1];
        uint32_t oo[G + 1];
        SsCursor cur;
        cur.init((uint32_t)tid, (uint32_t)CR, (uint32_t)W);
        auto issue = [&](int k) {
            if constexpr (LIN) {
                const uint32_t o = o_lin + (uint32_t)k * KS;
                oo[k % (G + 1)] = o;
                v0[k % (G + 1)] = ldv<NT>(reinterpret_cast<const V*>(src + o));
                r1[k] = ldv<NT>(reinterpret_cast<const V*>(src + o + W));
                return;
            }
            uint32_t itv = (uint32_t)(k * NTH + tid);
            asm volatile("" : "+v"(itv));   // no lane mask computed ahead (see the embed phase)
            const bool in = itv < items;
            const uint32_t o = in ? cur.o : 0u;
            oo[k % (G + 1)] = in ? cur.o : 0xFFFFFFFFu;
            v0[k % (G + 1)] = ldv<NT>(reinterpret_cast<const V*>(src + o));
            r1[k] = ldv<NT>(reinterpret_cast<const V*>(src + o + W));
            cur.step(dr, (uint32_t)CR, ostep, owrap);
        };
#pragma unroll
        for (int k = 0; k < G && k < NI; ++k) issue(k);
        // the slice's first loads go out before the setup below: the payload's copy into LDS
        // is a dependent round trip (load -> LDS write -> barrier), and in front of them it
        // held them back by one memory latency (C3 embed 0.0553 -> 0.0538 ms)
        asm volatile("" ::: "memory");
        L = (uint32_t)max(0, lengths[b]);
        for (int u = 0; u < crow; ++u) cnt[u * NTH + tid] = 0u;
        if (tid == 0) s_end = -1;
        {   // the payload into LDS (read by the embed phase, after the barriers below)
            const int nw = min(pw, (int)((L + 63u) >> 6));
            for (int w = tid; w < nw; w += NTH) pay[w] = payload[w];
        }
        lds_barrier();   // counters zeroed before any lane adds
#pragma unroll
        for (int k = 0; k < NI; ++k) {
            // the next load goes out here and no earlier: left free, hipcc hoisted every load of
            // the slice to the top (2 x NI vectors live at once: spills at NI = 16)
            asm volatile("" ::: "memory");
            if (k + G < NI) issue(k + G);
            asm volatile("" ::: "memory");
            V& a0 = v0[k % (G + 1)];
            V& a1 = r1[k];
            // one item at a time: left free, hipcc interleaved several items' unpacked pixels
            // and masks (~25 VGPRs each) for ILP and spilled the kept rows at NI = 16
            asm volatile("" : "+v"(a0.x), "+v"(a0.y), "+v"(a0.z), "+v"(a0.w), "+v"(a1.x), "+v"(a1.y), "+v"(a1.z),
                         "+v"(a1.w));
            const bool in = oo[k % (G + 1)] != 0xFFFFFFFFu;
            int x[4], a[4], bb[4], cc[4];
            uint32_t ep = 0;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                x[q] = (int)get_px(a1, 2 * q + 1); a[q] = (int)get_px(a1, 2 * q);
                bb[q] = (int)get_px(a0, 2 * q + 1); cc[q] = (int)get_px(a0, 2 * q);
                const int e = x[q] - med3(a[q], bb[q], cc[q]);
                // byte q (res_ex_bytes): the clamped error, near, expansion safe (p + 2e = x + e)
                const uint32_t sfe = (unsigned)(x[q] + e) < (unsigned)maxval ? 0x80u : 0u;
                const uint32_t nr = (unsigned)(x[q] + (e >= 0 ? tmax : -tmax)) > (unsigned)maxval ? 0x40u : 0u;
                ep |= (((uint32_t)res_med3(e, -32, 30) & 0x3Fu) | nr | sfe) << (8 * q);
            }
            // computed here, in the read phase: left free, hipcc sank it into the embed phase
            // and kept the even row's pixels alive for it (spills at NI = 16)
            asm volatile("" : "+v"(ep));
            if constexpr (LIN) s_re[k * NTH + tid] = ep;
            else re[k] = ep;
            res_hist4<NTH, LIN>(cnt, tid, ep, LIN || in, tmax);
            if constexpr (LIN) {
                stv<NTS>(reinterpret_cast<V*>(dst + oo[k % (G + 1)]), a0);
                lm_half[(uint32_t)k * lm_step] = 0u;   // cleared now; the embed phase ORs nothing in
            } else {
                stv<NTS>(in ? reinterpret_cast<V*>(dst + oo[k % (G + 1)]) : sink_v, a0);
            }
#if RES_LOCKSTEP
            if ((k % RES_LOCKSTEP) == RES_LOCKSTEP - 1) lds_barrier();
#endif
        }
    }
    lds_barrier();
    RES_STAMP(1);
    // ---- T: the smallest T <= tmax whose capacity holds L (pee_select_slice's rule)
    for (int u = wv; u < tmax; u += NWV) {
        uint32_t s = 0;
#pragma unroll
        for (int j = 0; j < NTH / 64; ++j)
            s += LIN ? (cnt[(u >> 1) * NTH + j * 64 + lane] >> (16 * (u & 1))) & 0xFFFFu : cnt[u * NTH + j * 64 + lane];
        s = wave_incl_dpp(s);   // DPP, not shuffles: lane 63 holds the bin's total
        if (lane == 63) s_bins[u] = s;
    }
    lds_barrier();
    if (wv == 0) {   // lane t - 1: capacity(t) = bins 0..t-1; T = the first t with capacity >= L
        const uint32_t run = wave_incl_dpp(lane < tmax ? s_bins[lane] : 0u);   // <= 4 x items: no overflow
        const u64 hit = __ballot(lane < tmax && run >= L);
        const int tsel = hit ? (int)__builtin_ctzll(hit) + 1 : 0;
        const uint32_t cap = (uint32_t)__builtin_amdgcn_readlane((int)run, (tsel ? tsel : tmax) - 1);
        if (lane == 0) {
            s_T = tsel ? tsel : tmax;
            s_cap = cap;   // the exact capacity at T over the whole slice
            if (t_out) t_out[b] = s_T;
        }
    }
    lds_barrier();
    const int Tthr = s_T;
    RES_STAMP(2);

    // ---- embed phase: the odd rows from registers, in item order (no loads).  Every rank is
    // known before any candidate moves: pass A counts each item's expandable candidates, ONE
    // block scan (the NI chunks' counters packed two per word, 16-bit fields) gives every
    // item its exclusive rank, pass B embeds every item with no further barrier.  A block
    // scan per chunk (or per 2-4 chunks) left this phase latency-bound: a barrier and its LDS
    // round trips per chunk with two waves per SIMD, 20 of 60 us at C3 (tools/res_trace.py)
    const uint32_t* pay32 = reinterpret_cast<const uint32_t*>(pay);
    // the field's two words: ranks < L lie in the staged words; larger ranks (unused bits)
    // only need an address inside the pad
    const uint32_t pmax = PADW - 2;
    const bool embed = trace != 2;   // trace 2: timing diagnostics only (no embedding: wrong stego)
    // pass A: each item's expandable+safe candidates counted from its kept bytes (SWAR,
    // res_ex_bytes), items 4j .. 4j + 3 in the bytes of one word, one wave scan per word: the
    // lane-exclusive prefixes (<= 63 x 4) never overflow a byte, only lane 63's inclusive sum
    // (never read by another lane); they go to LDS (the counters' words, free once T is
    // chosen; the registers are full of kept rows), the wave totals (<= 256) as 16-bit pairs
    uint32_t* s_ex = pad + PADW - (NI / 4) * NTH;
#ifndef RES_EXR
#define RES_EXR 0
#endif
    constexpr bool EXR = LIN && RES_EXR;   // the lane-exclusive prefixes in registers (spills at 1024)
    uint32_t exr[EXR ? NI / 4 : 1];
#pragma unroll
    for (int j = 0; j < NI / 4; ++j) {
        uint32_t itv[4], ep[4];
#pragma unroll
        for (int h = 0; h < 4; ++h) {
            itv[h] = (uint32_t)(4 * j + h) * NTH + (uint32_t)tid;
            ep[h] = LIN ? s_re[(4 * j + h) * NTH + tid] : re[4 * j + h];
        }
        asm volatile("" : "+v"(itv[0]), "+v"(itv[1]), "+v"(itv[2]), "+v"(itv[3]), "+v"(ep[0]), "+v"(ep[1]),
                     "+v"(ep[2]), "+v"(ep[3]));   // nothing of pass B ahead
        uint32_t c = 0;
#pragma unroll
        for (int h = 0; h < 4; ++h)
            c |= (uint32_t)__popc(res_ex_bytes(ep[h], Tthr) & ep[h] & (itv[h] < items ? ~0u : 0u)) << (8 * h);
        const uint32_t ex = wave_incl_dpp(c) - c;
        if constexpr (EXR) exr[j] = ex;
        else s_ex[j * NTH + tid] = ex;
        if (lane == 63) {   // chunk totals: fields 0 and 2 / 1 and 3 as 16-bit halves
            const uint32_t lo = (ex & 0x00FF00FFu) + (c & 0x00FF00FFu);
            const uint32_t hi = ((ex >> 8) & 0x00FF00FFu) + ((c >> 8) & 0x00FF00FFu);
            s_wt[2 * j][wv] = (lo & 0xFFFFu) | (hi << 16);
            s_wt[2 * j + 1][wv] = (lo >> 16) | (hi & 0xFFFF0000u);
        }
    }
    lds_barrier();
    if (wv == 0) {   // wave bases per pair of chunks (four pairs at once, one per DPP row), then
                     // the chunks' bases over the whole slice
        const int r = lane >> 4, j = lane & 15;
#pragma unroll
        for (int it = 0; it < NI / 8; ++it) {
            const int i = 4 * it + r;
            const int x = j < NWV ? (int)s_wt[i][j] : 0;
            int y = x;
            y += __builtin_amdgcn_update_dpp(0, y, 0x111, 0xF, 0xF, true);   // row_shr:1
            y += __builtin_amdgcn_update_dpp(0, y, 0x112, 0xF, 0xF, true);   // row_shr:2
            y += __builtin_amdgcn_update_dpp(0, y, 0x114, 0xF, 0xF, true);   // row_shr:4
            if constexpr (NWV > 8) y += __builtin_amdgcn_update_dpp(0, y, 0x118, 0xF, 0xF, true);   // row_shr:8
            if (j < NWV) s_wb[i][j] = (uint32_t)(y - x);   // per-field: a chunk's total < 2^16
            if (j == NWV - 1) s_tot[i] = (uint32_t)y;
        }
        const uint32_t t = lane < NI ? (s_tot[lane >> 1] >> (16 * (lane & 1))) & 0xFFFFu : 0u;
        const uint32_t cb = wave_incl_dpp(t) - t;
        if (lane < NI) s_cb[lane] = cb;
    }
    lds_barrier();   // wave and chunk bases
    RES_STAMP(3);
    uint32_t unsafe_n = 0;
    SsCursor cur;
    cur.init((uint32_t)tid, (uint32_t)CR, (uint32_t)W);
    // LIN: lane k of every wave holds the wave's base rank for item k (read back by readlane)
    uint32_t vb = 0;
    if constexpr (LIN) {
        const int kk = lane < NI ? lane : 0;
        vb = s_cb[kk] + ((s_wb[kk / 2][wv] >> (16 * (kk & 1))) & 0xFFFFu);
    }
    // item k's rank and payload field are read from LDS one item ahead (during item k - 1), so
    // their two LDS round trips are off the item's own dependency chain
    auto rank_of = [&](int k) {
        if constexpr (EXR)
            return (uint32_t)__builtin_amdgcn_readlane((int)vb, k) + ((exr[k / 4] >> (8 * (k & 3))) & 0xFFu);
        if constexpr (LIN)
            return (uint32_t)__builtin_amdgcn_readlane((int)vb, k) + ((s_ex[(k / 4) * NTH + tid] >> (8 * (k & 3))) & 0xFFu);
        const uint32_t ex = s_ex[(k / 4) * NTH + tid], wb = s_wb[k / 2][wv];
        return s_cb[k] + ((wb >> (16 * (k & 1))) & 0xFFFFu) + ((ex >> (8 * (k & 3))) & 0xFFu);
    };
    auto field_at = [&](uint32_t rs) {
        const uint32_t w = min(rs >> 5, pmax);
        return __builtin_amdgcn_alignbit(pay32[w + 1], pay32[w], rs & 31u);
    };
    uint32_t rs_n = rank_of(0);
    uint32_t field_n = field_at(rs_n);
#pragma unroll
    for (int k = 0; k < NI; ++k) {
        uint32_t itv = (uint32_t)k * NTH + (uint32_t)tid;
        uint32_t ep = LIN ? s_re[k * NTH + tid] : re[k];
        V& v1 = r1[k];
        const uint32_t rs = rs_n, field = field_n;
        if (k + 1 < NI) {
            rs_n = rank_of(k + 1);
            field_n = field_at(rs_n);
        }
        // this item's values enter here: nothing derived from them is computed ahead for all
        // items at once (registers), no lane mask is kept across items (SGPRs)
        asm volatile("" : "+v"(v1.x), "+v"(v1.y), "+v"(v1.z), "+v"(v1.w), "+v"(ep), "+v"(itv), "+v"(cur.o),
                     "+v"(cur.cc));
        uint32_t ob = o_lin;
        asm volatile("" : "+v"(ob));   // LIN: the address is formed here (hoisted: 16 spilled pointers)
        const uint32_t o1 = LIN ? ob + (uint32_t)k * KS + (uint32_t)W : cur.o + (uint32_t)W;
        if constexpr (!LIN) cur.step(dr, (uint32_t)CR, ostep, owrap);
        const bool ok = LIN || itv < items;
        uint32_t ns_b = 0;   // processed candidates left unchanged as unsafe (the location map)
        if (embed && rs < L) {   // divergent only at the lane holding `end`; no memory op inside
            const uint32_t ex_b = res_ex_bytes(ep, Tthr);
            const uint32_t esm_b = ex_b & ep;   // expandable + safe: carry payload bits
            const uint32_t m = ok ? min(L - rs, 4u) : 0u;
            const uint32_t pre_b = res_prefix(esm_b);
            // processed: fewer than m payload carriers before the candidate in the item
            const uint32_t proc_b = ~((pre_b | 0x80808080u) - __builtin_amdgcn_perm(m, m, 0u)) & 0x80808080u;
            // safe: expandable -> the kept bit; shifted -> not near (else checked exactly below)
            uint32_t safe_b = ((ex_b & ep) | (~ex_b & ~(ep << 1))) & 0x80808080u;
            const uint32_t nr_b = ~ex_b & (ep << 1) & proc_b;
            if (__builtin_amdgcn_ballot_w64(nr_b != 0u)) {   // wave-uniform; rare on smooth data
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const uint32_t w = q == 0 ? v1.x : q == 1 ? v1.y : q == 2 ? v1.z : v1.w;
                    const int y = (int)(w >> 16) + res_med3(__builtin_amdgcn_sbfe((int)ep, 8 * q, 6), -Tthr, Tthr);
                    if (((nr_b >> (8 * q + 7)) & 1u) && (unsigned)y <= (unsigned)maxval) safe_b |= 0x80u << (8 * q);
                }
            }
            const uint32_t sel_b = proc_b & safe_b;
            // a moved candidate: y = x + clamp(e + bit, -T, T); the bit (field bit pre_q) is
            // absorbed by the clamp for a shifted one (e >= T or e < -T)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                uint32_t& w = q == 0 ? v1.x : q == 1 ? v1.y : q == 2 ? v1.z : v1.w;
                const int bit = q == 0 ? (int)(field & 1u) : (int)__builtin_amdgcn_ubfe(field, pre_b >> (8 * q), 1);
                int d = res_med3(__builtin_amdgcn_sbfe((int)ep, 8 * q, 6) + bit, -Tthr, Tthr);
                d &= __builtin_amdgcn_sbfe((int)sel_b, 8 * q + 7, 1);
                w += (uint32_t)d << 16;
            }
            if (m != 0 && L - rs <= (uint32_t)__popc(esm_b))
                s_end = (int)(4 * itv) + ((31 - __clz(proc_b & esm_b)) >> 3);
            ns_b = proc_b & ~safe_b;
        }
        uint32_t wm = 0;
        if (__builtin_amdgcn_ballot_w64(ns_b != 0u)) {   // wave-uniform; rare
            const uint32_t nib = res_nibble(ns_b);
            unsafe_n += (uint32_t)__popc(nib);
            wm = nib << (4 * (lane & 7));
            wm |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)wm, 0xB1, 0xF, 0xF, false);    // quad_perm [1,0,3,2]
            wm |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)wm, 0x4E, 0xF, 0xF, false);    // quad_perm [2,3,0,1]
            wm |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)wm, 0x141, 0xF, 0xF, false);   // row_half_mirror
            if constexpr (LIN) {   // over the read phase's zero (address formed here, not CSE'd with it)
                uint32_t ls = lm_step;
                asm volatile("" : "+v"(ls));
                lm_half[(uint32_t)k * ls] = wm;
            }
        }
        if constexpr (LIN) {
            stv<NTS>(reinterpret_cast<V*>(dst + o1), v1);
#if RES_ELOCK
            if ((k % RES_ELOCK) == RES_ELOCK - 1) lds_barrier();
#endif
            continue;
        }
        // stores, unconditional: the map word halves (zeros past `end`), the odd row
        const uint32_t wix = (4 * itv) >> 6;
        *(ok && (lane & 7) == 0 && (int)wix < lmw ? reinterpret_cast<uint32_t*>(lm + wix) + ((lane >> 3) & 1) : sink_w) =
            wm;
        stv<NTS>(ok ? reinterpret_cast<V*>(dst + o1) : sink_v + 1, v1);
#if RES_ELOCK
        if ((k % RES_ELOCK) == RES_ELOCK - 1) lds_barrier();
#endif
    }
    const uint32_t running = s_cap;   // expandable candidates of the slice at T
    // lm_count: one block reduction
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) unsafe_n += __shfl_xor(unsafe_n, o, 64);
    if (lane == 0) red[wv] = unsafe_n;
    lds_barrier();
    RES_STAMP(4);
    if (tid == 0) {
        uint32_t un = 0;
        for (int w = 0; w < NWV; ++w) un += red[w];
        codec_pee_meta* M = meta_all + b;
        M->T = Tthr; M->maxval = maxval; M->L = (int)L; M->nc = nc; M->ntiles = ntiles; M->h = H; M->w = W;
        M->lm_count = (int)un;
        M->capacity = (int)s_cap;   // exact: the read phase counted the whole slice
        M->flags = 0;
        M->reserved[0] = M->reserved[1] = M->reserved[2] = 0;
        if (L == 0) { M->end = -1; M->tile_end = -1; M->status = 0; }
        else if (running < L) { M->end = nc - 1; M->tile_end = ntiles - 1; M->status = 1; }   // truncated
        else { M->end = s_end; M->tile_end = s_end / PEE_TILE; M->status = 0; }
    }
}

// EARLY: the ring slot is refilled as soon as its data is taken (before the chunk's barrier
// and compute), as the in-place embed does with D = 1 (k_pee_embed_ss)
template <typename T, bool NT, bool INPLACE, int D, bool EARLY = false, bool NTS = NT>   // NTS: k_pee_embed_ss
__global__ __launch_bounds__(SS_THREADS) void k_pee_extract_ss(const T* __restrict__ stego, T* cover, int H, int W,
                                                               const codec_pee_meta* __restrict__ meta_all,
                                                               const u64* __restrict__ lm_all, int lmw,
                                                               u64* __restrict__ payload_all, int pw,
                                                               uint32_t* __restrict__ lb_flag, char* __restrict__ sink) {
    typedef typename Vec8<T>::type V;
    __shared__ uint32_t ss_pad[SS_PAD_WORDS];
    __shared__ uint32_t wtot[2][16];
    __shared__ u64 pbuf[2][SS_THREADS * 4 / 64 + 2];
    __shared__ u64 s_carry[2];
    const int b = blockIdx.x;
    const int tid = threadIdx.x;
    const int CR = W / 8;
    const uint32_t items = (uint32_t)(H / 2) * (uint32_t)CR;
    const int nchunks = (int)((items + SS_THREADS - 1) / SS_THREADS);
    const codec_pee_meta* M = meta_all + b;
    const int end = M->end, Tthr = M->T;
    const int cend = end >= 0 ? (end >> 2) / SS_THREADS : -1;
    const int nproc = INPLACE ? cend + 1 : nchunks;
    const int klast = max(nproc, 1) - 1;
    const size_t npx = (size_t)H * W;
    const T* src = stego + b * npx;
    T* dst = cover + b * npx;
    const u64* lm = lm_all + (size_t)b * lmw;
    u64* payload = payload_all + (size_t)b * pw;
    V* sink_v = reinterpret_cast<V*>(sink + SS_SINK_SLOT(b, tid));
    u64* sink_w = reinterpret_cast<u64*>(sink + SS_SINK_SLOT(b, tid) + 32);
    if (tid == 0) {
        s_carry[0] = s_carry[1] = 0ull;
        ss_pad[SS_PAD_WORDS - 1] = 0u;
        if (b == 0) *lb_flag = 0u;   // codec_pee_extract_flag_offset: no look-back here, never set
    }
    if (tid < SS_THREADS * 4 / 64 + 2) pbuf[0][tid] = pbuf[1][tid] = 0ull;
    V r0[D], r1[D];
    u64 rl[D];
    const uint32_t dq = SS_THREADS / (uint32_t)CR, dr = SS_THREADS % (uint32_t)CR;
    const uint32_t ostep = 2u * (uint32_t)W * dq + 8u * dr, owrap = 2u * (uint32_t)W - 8u * (uint32_t)CR;
    // the ring never loads past chunk klast (in place: the chunk holding `end`)
    const uint32_t items_l = min(items, (uint32_t)(klast + 1) * SS_THREADS);
    uint32_t off_last;
    {
        SsCursor l;
        l.init(items_l - 1u, (uint32_t)CR, (uint32_t)W);
        off_last = l.o;
    }
    uint32_t ro[D];
    SsCursor ahead;
    ahead.init((uint32_t)tid, (uint32_t)CR, (uint32_t)W);
    uint32_t it_a = (uint32_t)tid;
#pragma unroll
    for (int d = 0; d < D; ++d) {
        const bool in = it_a < items_l;
        ro[d] = in ? ahead.o : off_last;
        ss_load_at<T, NT>(src, (uint32_t)W, ro[d], r0[d], r1[d]);
        rl[d] = lm[(4 * (in ? it_a : items_l - 1u)) >> 6];
        ahead.step(dr, (uint32_t)CR, ostep, owrap);
        it_a += SS_THREADS;
    }
    uint32_t running = 0;
    int par = 0;
    // The payload words of chunk j are written during chunk j+1, after its scan barrier (one
    // barrier per chunk): pending = chunk j's word range.  Chunk j's first word continues the
    // previous partial word (s_carry[(j-1)&1]); a partial last word goes to s_carry[j&1].
    bool pend = false;
    uint32_t p_lo = 0, p_hi = 0;
    int p_par = 0;

    // words of the pending chunk for thread tid: (value, absolute index, store it?)
    auto emit = [&](u64* wout, uint32_t* wabs, bool* wstore) {
        const int nw = (int)(((p_lo & 63u) + (p_hi - p_lo) + 63u) >> 6);
        if (tid < nw) {
            const uint32_t a = (p_lo >> 6) + (uint32_t)tid;
            const u64 wv = pbuf[p_par][tid] | (tid == 0 ? s_carry[p_par ^ 1] : 0ull);
            if ((a + 1u) * 64u <= p_hi) { *wout = wv; *wabs = a; *wstore = (int)a < pw; }
            else s_carry[p_par] = wv;
        }
        if (tid == 0 && (p_hi & 63u) == 0u) s_carry[p_par] = 0ull;
    };

    auto refill = [&](int d) {   // branch-free; past chunk klast the last item's address, data unused
        const bool in = it_a < items_l;
        ro[d] = in ? ahead.o : off_last;
        ss_load_at<T, NT>(src, (uint32_t)W, ro[d], r0[d], r1[d]);
        rl[d] = lm[(4 * (in ? it_a : items_l - 1u)) >> 6];
        ahead.step(dr, (uint32_t)CR, ostep, owrap);
        it_a += SS_THREADS;
    };
    auto chunk = [&](int d, int k) {
        V w0, w1;
        if constexpr (EARLY) { w0 = r0[d]; w1 = r1[d]; }
        V& v0 = EARLY ? w0 : r0[d];
        V& v1 = EARLY ? w1 : r1[d];
        const u64 lw = rl[d];
        const uint32_t it = (uint32_t)k * SS_THREADS + tid;
        const bool ok = it < items;
        const uint32_t o0 = ro[d];
        // the chunk's registers are waited for here, once, outside any branch (see k_pee_embed_ss)
        asm volatile("" ::"v"(v0.x), "v"(v1.x), "v"((uint32_t)lw));
        if constexpr (EARLY) refill(d);
        uint32_t actm = 0;
        u64 wout = 0;
        bool wstore = false;
        uint32_t wabs = 0;
        if (k <= cend) {   // uniform; no vector memory instruction inside
            uint32_t innm = 0;
            int pq[4];
            const uint32_t l4 = (uint32_t)(lw >> ((4 * it) & 63u));
            const int rem = end - (int)(4 * it);   // candidate q of this item is at or before `end` iff q <= rem
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const bool act = ok & (q <= rem) & !((l4 >> q) & 1u);   // & : no branches
                const int p = med3((int)get_px(v1, 2 * q), (int)get_px(v0, 2 * q + 1), (int)get_px(v0, 2 * q));
                const int e2 = (int)get_px(v1, 2 * q + 1) - p;
                pq[q] = p;
                actm |= act ? 1u << q : 0u;
                innm |= (act & ((unsigned)(e2 + 2 * Tthr) < (unsigned)(4 * Tthr))) ? 1u << q : 0u;
            }
            const uint32_t n = (uint32_t)__popc(innm);
            // pbuf[par] was last read (and re-zeroed below) by these same threads two chunks ago
            uint32_t ex, tot, wb;
            ss_scan_small(n, wtot, par, &ex, &tot, &wb);
            if (pend) emit(&wout, &wabs, &wstore);          // the previous chunk's words
            if (tid < SS_THREADS * 4 / 64 + 2 && pend) pbuf[p_par][tid] = 0ull;
            // this lane's inner candidates take ranks [rs, rs + n): their bits form one <= 4-bit
            // field, OR-ed into at most two words of the chunk's LDS buffer
            const uint32_t rs = running + ex;
            uint32_t field = 0;
#pragma unroll
            for (int q = 0; q < 4; ++q) {   // branch-free
                const uint32_t bit = 1u << q;
                const int x = (int)get_px(v1, 2 * q + 1);
                const int p = pq[q];
                const int e2 = x - p;
                const bool act = (actm & bit) != 0, inner = (innm & bit) != 0;
                field |= ((uint32_t)inner & (uint32_t)e2 & 1u) << __popc(innm & (bit - 1u));
                const int v_in = p + (e2 >> 1), v_sh = x + ((e2 >= 2 * Tthr) ? -Tthr : Tthr);
                const int nx = act ? (inner ? v_in : v_sh) : x;
                set_px(v1, 2 * q + 1, (uint32_t)nx);
            }
            if (field) {   // <= 4 bits at chunk bit o: one or two 32-bit words of the LDS buffer
                uint32_t* pb32 = reinterpret_cast<uint32_t*>(pbuf[par]);
                const uint32_t o = rs - (running & ~63u), wi = o >> 5, sh = o & 31u;
                atomicOr(&pb32[wi], field << sh);
                if (sh > 28u && (field >> (32u - sh))) atomicOr(&pb32[wi + 1], field >> (32u - sh));
            }
            pend = true;
            p_lo = running;
            p_hi = running + tot;
            p_par = par;
            par ^= 1;
            running += tot;
        } else if (SS_LOCKSTEP && (k % SS_LOCKSTEP) == SS_LOCKSTEP - 1) {
            lds_barrier();   // copy chunks: keep the waves in step (see k_pee_embed_ss; 0.91 -> 0.78 ms)
        }
        // stores, unconditional (redirected to the sink when they must not land)
        *(wstore ? payload + wabs : sink_w) = wout;
        if (INPLACE) {
            stv<NTS>(ok && actm ? reinterpret_cast<V*>(dst + o0 + W) : sink_v, v1);
        } else {
            stv<NTS>(ok ? reinterpret_cast<V*>(dst + o0) : sink_v, v0);
            stv<NTS>(ok ? reinterpret_cast<V*>(dst + o0 + W) : sink_v + 1, v1);
        }
        if constexpr (!EARLY) refill(d);
    };

    const int nfull = nproc / D * D;
    for (int k0 = 0; k0 < nfull; k0 += D) {
#pragma unroll
        for (int d = 0; d < D; ++d) chunk(d, k0 + d);
    }
#pragma unroll
    for (int d = 0; d < D; ++d)
        if (nfull + d < nproc) chunk(d, nfull + d);
    // the last chunk's words, its partial last word, then zeros to the end of the payload row
    lds_barrier();
    if (pend) {
        u64 wout = 0;
        bool wstore = false;
        uint32_t wabs = 0;
        emit(&wout, &wabs, &wstore);
        if (wstore) payload[wabs] = wout;
        lds_barrier();
        if (tid == 0 && (running & 63u) && (int)(running >> 6) < pw) payload[running >> 6] = s_carry[p_par];
    }
    const uint32_t full = (running + 63u) >> 6;
    for (uint32_t w = full + tid; w < (uint32_t)pw; w += SS_THREADS) payload[w] = 0ull;
}

// ====================================================================== host side
struct PeeWs {
    size_t cnt, off, st, ctl, diag, hist, sink, total;
    int ntiles_max, nchunks;
};

static PeeWs pee_ws(const codec_pee_params* P) {
    PeeWs L;
    const long long nc = (long long)(P->H / 2) * (P->W / 2);
    L.ntiles_max = (int)((nc + PEE_TILE - 1) / PEE_TILE);
    if (L.ntiles_max < 1) L.ntiles_max = 1;
    const long long items = (long long)(P->H / 2) * (P->W / 8);
    L.nchunks = (int)((items + PEE_CHUNK - 1) / PEE_CHUNK);
    if (L.nchunks < 1) L.nchunks = 1;
    L.cnt = 0;
    L.off = align_up((size_t)P->B * L.ntiles_max * 4, 256);
    L.st = align_up(L.off + (size_t)P->B * L.ntiles_max * 4, 256);
    // two status-word buffers (PEE_MODE_SC), then ctl; zeroing calls clear them all together
    L.ctl = L.st + 2 * (size_t)P->B * L.nchunks * 8;
    // diag: 4 cumulative uint32 counters (codec_pee_diag_offset), outside the per-call memset
    L.diag = align_up(L.ctl + PEE_CTL_WORDS(P->B, L.nchunks) * 4, 16);
    // capacity-control error histogram (codec_pee_capacity; cleared by that call)
    L.hist = align_up(L.diag + 16, 256);
    // slice-serial kernels: per-lane sink for stores that must not land (contents unused)
    L.sink = align_up(L.hist + (size_t)P->B * (PEE_TMAX_MAX + 1) * 4, 256);   // + per-slice arrival counters
    L.total = align_up(L.sink + SS_SINK_BYTES(P->B), 256);
    return L;
}


// Measured at B = 256 (profiles/r02/ss_vs_lookback.json): in place the slice-serial pass
// wins at every size (2048^2 embed 0.145 -> 0.111 ms, extract 0.115 -> 0.109); out of place
// it streams at ~4.9 TB/s per chip, which beats the look-back pass on small slices
// (512^2: embed 0.066 -> 0.059, extract 0.077 -> 0.069) but not on 2048^2 ones (look-back
// 0.71-0.73 ms vs 0.88), so out of place it is used up to CODEC_PEE_SS_OOP_MAXCH chunks.
static bool pee_use_slice_serial(const codec_pee_params* P, bool inplace) {
    const long long k = knob("CODEC_PEE_SS", -1);
    if (k == 0) return false;
    if (k == 1) return true;
    const long long ncu = device_cu_count();
    if (P->B < ncu) return false;
    const long long rounds = (P->B + ncu - 1) / ncu;
    if ((double)P->B / (double)(rounds * ncu) < 0.85) return false;   // the last round nearly full
    if (inplace) return true;
    const long long items = (long long)(P->H / 2) * (P->W / 8);
    return (items + SS_THREADS - 1) / SS_THREADS <= knob("CODEC_PEE_SS_OOP_MAXCH", 64);
}

static int pee_check(const codec_pee_params* P) {
    if (!P) return set_err(CODEC_EINVAL, "params is NULL");
    if (P->B < 1 || P->H < 1 || P->W < 1 || (long long)P->H * P->W > 0x7FFFFFFFLL)
        return set_err(CODEC_EINVAL, "bad shape");
    if (P->bytes != 1 && P->bytes != 2) return set_err(CODEC_EINVAL, "bytes must be 1 or 2");
    if (P->T < 1) return set_err(CODEC_EINVAL, "T must be >= 1");
    const int vmax = P->bytes == 2 ? 65535 : 255;
    if (P->maxval < 1 || P->maxval > vmax) return set_err(CODEC_EINVAL, "maxval out of range");
    if (P->payload_words < 1 || P->lm_words < 1) return set_err(CODEC_EINVAL, "payload_words/lm_words must be >= 1");
    const long long nc = (long long)(P->H / 2) * (P->W / 2);
    if ((long long)P->lm_words * 64 < nc) return set_err(CODEC_EINVAL, "lm_words must cover every candidate");
    return 0;
}

// up to three 8-byte-aligned regions zeroed by one launch (the look-back paths clear their
// status words, meta records, location map or payload rows before the pass: one dispatch
// instead of two or three hipMemsetAsync fills, which at C2 size cost more than the work)
struct ZeroSpans {
    u64* p[3];
    size_t n[3];   // 8-byte words
};
__global__ __launch_bounds__(256) void k_zero_spans(ZeroSpans z) {
    const size_t stride = (size_t)gridDim.x * 256;
#pragma unroll
    for (int r = 0; r < 3; ++r)
        for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < z.n[r]; i += stride) z.p[r][i] = 0ull;
}
static hipError_t pee_zero(hipStream_t st, void* a, size_t abytes, void* b = nullptr, size_t bbytes = 0,
                           void* c = nullptr, size_t cbytes = 0) {
    ZeroSpans z{{static_cast<u64*>(a), static_cast<u64*>(b), static_cast<u64*>(c)}, {abytes / 8, bbytes / 8, cbytes / 8}};
    const size_t tot = z.n[0] + z.n[1] + z.n[2];
    if (!tot) return hipSuccess;
    const unsigned g = (unsigned)std::min<size_t>(1024, (tot + 1023) / 1024);
    hipLaunchKernelGGL(k_zero_spans, dim3(g), dim3(256), 0, st, z);
    return hipGetLastError();
}

// ---- workspace registry.  Small out-of-place batches
// (PEE_MODE_SC) carry two status-word buffers and finished flags from call to call in the
// workspace, and the capacity pass leaves its bins clear for the next call, at offsets that
// depend on the shape.  The library remembers, per (device, workspace pointer), the shape of
// the last call that used it and the epoch of its self-cleaning calls: a call of another
// shape zeroes the workspace (one launch, the cumulative diagnostic counters kept) before it
// runs, so a workspace sized for the largest batch and reused for a smaller tail batch stays
// exact; the first self-cleaning call seen on a pointer zeroes its state region; and every
// self-cleaning call gets the next epoch (parity + tag, see PEE_MODE_SC).
struct PeeWsShape {
    int B, H, W, bytes;
    uint32_t epoch;   // self-cleaning calls issued on this workspace (their status-word epoch)
    bool sc_clean;    // the self-cleaning state region is known clean (zeroed here, or kept by SC calls)
    size_t diag;      // offset of the diagnostic counters in this shape's layout
    // a call on this workspace was captured into a graph: replays run without the
    // host, so they can rewrite the captured shape's state at any time.  Self-cleaning calls of
    // any OTHER shape then take the zeroing path (their finished flags could sit on the replay's
    // words); the captured shape itself stays exact through its epoch tags
    bool captured;
    int cB, cH, cW, cbytes;
};
static std::mutex g_pee_ws_mu;
static std::map<std::pair<int, uintptr_t>, PeeWsShape> g_pee_ws;
// the registry only remembers pointers: an unknown pointer is treated as a fresh workspace
// (its self-cleaning state zeroed on first use), so forgetting entries is always safe --
// bounded here so that a process allocating many workspaces does not grow it without end
constexpr size_t kPeeWsMax = 4096;
static std::pair<int, uintptr_t> pee_ws_key(const void* ws) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) dev = -1;
    return {dev, (uintptr_t)ws};
}
// the whole workspace but the diagnostic counters
static hipError_t pee_ws_zero(void* ws, const PeeWs& L, hipStream_t st) {
    char* w = static_cast<char*>(ws);
    return pee_zero(st, w, L.diag, w + L.hist, L.total - L.hist);
}
static bool pee_capturing(hipStream_t st) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    return hipStreamIsCapturing(st, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone;
}
// every workspace-taking PEE call, after its argument checks
static hipError_t pee_ws_enter(void* ws, const codec_pee_params* P, const PeeWs& L, hipStream_t st) {
    bool changed = false, moved_diag = false;
    {
        std::lock_guard<std::mutex> g(g_pee_ws_mu);
        auto k = pee_ws_key(ws);
        auto it = g_pee_ws.find(k);
        if (it == g_pee_ws.end() && g_pee_ws.size() >= kPeeWsMax) g_pee_ws.clear();
        PeeWsShape now{P->B, P->H, P->W, P->bytes, 0u, it != g_pee_ws.end(), L.diag, false, 0, 0, 0, 0};
        if (it == g_pee_ws.end()) {
            it = g_pee_ws.emplace(k, now).first;
        } else if (it->second.B != now.B || it->second.H != now.H || it->second.W != now.W ||
                   it->second.bytes != now.bytes) {
            // a shape change: zeroed below -- including the diagnostic counters when this
            // layout puts them elsewhere (they would start from the old shape's words)
            moved_diag = it->second.diag != L.diag;
            now.captured = it->second.captured;
            now.cB = it->second.cB; now.cH = it->second.cH; now.cW = it->second.cW; now.cbytes = it->second.cbytes;
            it->second = now;
            changed = true;
        }
        if (pee_capturing(st)) {
            it->second.captured = true;
            it->second.cB = P->B; it->second.cH = P->H; it->second.cW = P->W; it->second.cbytes = P->bytes;
        }
    }
    if (!changed) return hipSuccess;
    return moved_diag ? pee_zero(st, ws, L.total) : pee_ws_zero(ws, L, st);
}
// the self-cleaning words' unsafe-count field holds < 2^24 (LB_HI): bigger slices zero
// instead; so does a call being captured into a graph (a replay would repeat one epoch), and
// a call of another shape than a graph captured on this workspace (its replays may have
// written that shape's state over this one's)
static bool pee_sc_fits(const codec_pee_params* P, hipStream_t st, const void* ws) {
    if (pee_capturing(st)) return false;
    {
        std::lock_guard<std::mutex> g(g_pee_ws_mu);
        auto it = g_pee_ws.find(pee_ws_key(ws));
        if (it != g_pee_ws.end() && it->second.captured &&
            (it->second.cB != P->B || it->second.cH != P->H || it->second.cW != P->W || it->second.cbytes != P->bytes))
            return false;
    }
    return (long long)(P->H / 2) * (P->W / 2) <= PEE_SC_MAX_NC;
}
// this self-cleaning call's epoch (mod 126: parity and tag epoch % 63 + 1 both cycle in it);
// *fresh: the state region is not known clean (first self-cleaning call on a pointer never
// zeroed here): the caller zeroes it before the launch
static int pee_ws_epoch(const void* ws, bool* fresh) {
    std::lock_guard<std::mutex> g(g_pee_ws_mu);
    auto it = g_pee_ws.find(pee_ws_key(ws));
    if (it == g_pee_ws.end()) { *fresh = true; return 0; }   // not reached: pee_ws_enter registered it
    *fresh = !it->second.sc_clean;
    it->second.sc_clean = true;
    const uint32_t e = it->second.epoch;
    it->second.epoch = (e + 1u) % 126u;
    return (int)e;
}

// row H-1 of every slice, src -> dst (one strided 2-D copy)
static hipError_t pee_copy_last_rows(const codec_pee_params* P, const void* src, void* dst, hipStream_t st) {
    const size_t row = (size_t)P->W * P->bytes, pitch = (size_t)P->H * row, off = (size_t)(P->H - 1) * row;
    return hipMemcpy2DAsync(static_cast<char*>(dst) + off, pitch, static_cast<const char*>(src) + off, pitch, row,
                            (size_t)P->B, hipMemcpyDeviceToDevice, st);
}

extern "C" {

size_t codec_pee_workspace_bytes(const codec_pee_params* P) {
    if (pee_check(P)) return 0;
    return pee_ws(P).total;
}

size_t codec_pee_extract_flag_offset(const codec_pee_params* P) {
    if (pee_check(P)) return 0;
    return pee_ws(P).ctl + 4;   // ctl[1]: set when an extract chunk's look-back gave up
}

#ifdef PEE_LB_TRACE
int codec_debug_lb_trace(unsigned long long* out, int n) {   // diagnostic build only
    if (n > LB_TRACE_SLOTS * 12) n = LB_TRACE_SLOTS * 12;
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_lb_trace), (size_t)n * 8) == hipSuccess ? n : -1;
}
#endif
int codec_debug_res_trace(unsigned long long* out, int n) {   // CODEC_PEE_RES_TRACE=1 runs only
    if (!out || n < 0) return set_err(CODEC_EINVAL, "codec_debug_res_trace: bad arguments");
    if (n > RES_TRACE_WG * 5) n = RES_TRACE_WG * 5;
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_res_trace), (size_t)n * 8) == hipSuccess ? n : -1;
}
#ifdef PEE_SS_TRACE
int codec_debug_ss_trace(unsigned long long* out, int n) {   // diagnostic build only
    if (n > SS_TRACE_N) n = SS_TRACE_N;
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_ss_trace), (size_t)n * 8) == hipSuccess ? n : -1;
}
#endif

int codec_pee_capacity(const codec_pee_params* P, const void* cover, int32_t tmax, const int32_t* lengths,
                       int32_t* caps, int32_t* t_out, void* workspace, size_t workspace_bytes, void* stream) {
    int rc = pee_check(P);
    if (rc) return rc;
    if (!cover || !workspace) return set_err(CODEC_EINVAL, "codec_pee_capacity: NULL pointer argument");
    if (tmax < 1 || tmax > PEE_TMAX_MAX) return set_err(CODEC_EINVAL, "tmax must be in 1..64");
    if (t_out && !lengths) return set_err(CODEC_EINVAL, "codec_pee_capacity: t_out needs lengths");
    const PeeWs L = pee_ws(P);
    if (workspace_bytes < L.total) return set_err(CODEC_EINVAL, "workspace too small");
    HIP_TRY(pee_ws_enter(workspace, P, L, as_stream(stream)));   // another shape's state: zeroed first
    hipStream_t st = as_stream(stream);
    uint32_t* hist = reinterpret_cast<uint32_t*>(static_cast<char*>(workspace) + L.hist);
    // no memset: bins and arrival counters are zero on entry (zeroed workspace; each slice's
    // last workgroup clears them)
    const size_t va = P->bytes == 2 ? 16 : 8;
    const bool vec = (P->W % 8) == 0 && ((uintptr_t)cover % va) == 0;
    const long long units = vec ? (long long)(P->H / 2) * (P->W / 8) : (long long)(P->H / 2) * (P->W / 2);
    ProfScope prof(st, CODEC_K_PEE_CAPACITY);
    {   // launched even when there is nothing to count: the last workgroup writes caps / t_out
        const long long per = knob("CODEC_PEE_EHIST_PER_WG", 4096);
        const int dbg_delay = (int)debug_knob("CODEC_PEE_EHIST_DEBUG_DELAY", 0) - 1;
        dim3 grid((unsigned)max(1LL, (units + per - 1) / per), (unsigned)P->B);
        const size_t lds = (size_t)tmax * 256 * 4;   // lane-private counters
        uint32_t* arrivals = hist + (size_t)P->B * PEE_TMAX_MAX;
#define PEH(TT, VV) hipLaunchKernelGGL((k_pee_ehist<TT, VV>), grid, dim3(256), lds, st, static_cast<const TT*>(cover), P->H, \
                                       P->W, P->maxval, (int)tmax, (int)per, hist, arrivals, lengths, caps, t_out, dbg_delay)
        if (P->bytes == 2) { if (vec) PEH(uint16_t, true); else PEH(uint16_t, false); }
        else { if (vec) PEH(uint8_t, true); else PEH(uint8_t, false); }
#undef PEH
        LAUNCH_CHECK("k_pee_ehist");
    }
    return 0;
}

size_t codec_pee_diag_offset(const codec_pee_params* P) {
    if (pee_check(P)) return 0;
    return pee_ws(P).diag;
}

int codec_pee_reset(const codec_pee_params* P, void* workspace, size_t workspace_bytes, void* stream) {
    int rc = pee_check(P);
    if (rc) return rc;
    if (!workspace) return set_err(CODEC_EINVAL, "codec_pee_reset: NULL workspace");
    const PeeWs L = pee_ws(P);
    if (workspace_bytes < L.total) return set_err(CODEC_EINVAL, "workspace too small");
    hipStream_t st = as_stream(stream);
    HIP_TRY(pee_zero(st, workspace, L.total));   // diagnostics included: a fresh workspace
    std::lock_guard<std::mutex> g(g_pee_ws_mu);
    // (a graph captured on this workspace stays remembered: its replays may still run)
    auto& e = g_pee_ws[pee_ws_key(workspace)];
    const PeeWsShape prev = e;
    e = PeeWsShape{P->B, P->H, P->W, P->bytes, 0u, true, pee_ws(P).diag, prev.captured, prev.cB, prev.cH, prev.cW,
                   prev.cbytes};
    return 0;
}

int codec_pee_embed(const codec_pee_params* P, const void* cover, void* stego, const uint64_t* payload,
                    const int32_t* lengths, codec_pee_meta* meta, uint64_t* lm, void* workspace,
                    size_t workspace_bytes, void* stream) {
    return codec_pee_embed_ts(P, cover, stego, payload, lengths, nullptr, meta, lm, workspace, workspace_bytes, stream);
}

int codec_pee_embed_ts(const codec_pee_params* P, const void* cover, void* stego, const uint64_t* payload,
                       const int32_t* lengths, const int32_t* tps, codec_pee_meta* meta, uint64_t* lm, void* workspace,
                       size_t workspace_bytes, void* stream) {
    int rc = pee_check(P);
    if (rc) return rc;
    if (!cover || !stego || !payload || !lengths || !meta || !lm || !workspace)
        return set_err(CODEC_EINVAL, "codec_pee_embed: NULL pointer argument");
    const PeeWs L = pee_ws(P);
    if (workspace_bytes < L.total) return set_err(CODEC_EINVAL, "workspace too small");
    HIP_TRY(pee_ws_enter(workspace, P, L, as_stream(stream)));   // another shape's state: zeroed first
    hipStream_t st = as_stream(stream);
    uint32_t* cnt = reinterpret_cast<uint32_t*>(static_cast<char*>(workspace) + L.cnt);
    uint32_t* off = reinterpret_cast<uint32_t*>(static_cast<char*>(workspace) + L.off);
    const long long npx = (long long)P->H * P->W;
    const size_t va = P->bytes == 2 ? 16 : 8;
    const bool vec = (P->W % 8) == 0 && ((uintptr_t)cover % va) == 0 && ((uintptr_t)stego % va) == 0;
    const bool nt = knob("CODEC_NT", 1) != 0;
    const bool inplace = cover == stego;
    const long long items = (long long)(P->H / 2) * (P->W / 8);
    // single pass (default wherever W % 8 == 0 and the buffers are 16-B aligned): in place it
    // stops reading after `end`; out of place large batches walk chunk-major slot order (all
    // slices' chunk 0 first, then chunk 1 ...: every slice's look-back chain advances one hop
    // per generation of resident workgroups; slice-major order left whole generations
    // spinning on one slice's chain, 1.4 ms vs 0.82 ms at 256 x 2048^2, where the two-pass
    // scan + prefix embed takes 0.85 ms).
    // CODEC_PEE_ONEPASS: 0 forces the two-pass path; CODEC_PEE_1P_CHUNK_MAJOR=0: slice-major.
    // Out of place the chunk is the slot's own (CODEC_PEE_1P_NOTICKET=1, default): the per-slice
    // ticket atomic cost 2-3 % (0.78 -> 0.76 ms at 256 x 2048^2, tools/archive/tune_pee_mode2_cfg.json);
    // extract drops it too, and then loads the chunk's location-map words together with
    // its pixels (0.76 -> 0.74 ms).
    // CODEC_PEE_1P_GROUP (slices, multiple of 8; default 32): the batch is walked in groups of
    // that many slices, chunk-major inside a group -- 4 slices per XCD stream at once instead
    // of 32 (full chunk-major) or 1 (slice-major, whose look-back waits on the in-flight loads
    // of the 64 chunks before it): embed 0.81 -> 0.74 ms at 256 x 2048^2
    // (tools/tune_pee_group*_cfg.json); extract (CODEC_PEE_X_GROUP, default 32 as well)
    // 0.74 -> 0.73 ms (tools/archive/tune_pee_xnt_cfg.json).
    // Small out-of-place batches run the single pass too (one launch instead of scan + locate
    // + prefix embed, which are launch/latency bound there; tools/pee_small_batch.py, 2048²
    // embed+extract step: B=1 50 -> 32 us, B=4 65 -> 47, B=8 93 -> 74, B=31 229 -> 207).
    // B <= CODEC_PEE_FLAT_MAXB (7) uses flat slice-major slots over all XCDs (PEE_MODE_FLAT:
    // a lone slice's chunks would otherwise all sit on one XCD); no ticket by default (the
    // predecessors of a chunk have lower slot numbers, so in-order dispatch per XCD keeps the
    // look-back progressing, as in the lane order; 256 tickets on one line cost 8 us at B=1).
    const long long onepass = knob("CODEC_PEE_ONEPASS", -1);
    const bool flat = !inplace && P->B < 32 && P->B <= knob("CODEC_PEE_FLAT_MAXB", 7);
    if (vec && items > 0 && onepass != 0 && pee_use_slice_serial(P, inplace)) {
        // slice-serial single pass: one workgroup per slice, no look-back, no memsets
        ProfScope prof(st, CODEC_K_PEE_EMBED_SS);
        const bool pay_lds = P->payload_words <= SS_PAY_WORDS && knob("CODEC_PEE_SS_PAYLDS", 1) != 0;
#define PES1(TT, NTV, IP, PL) hipLaunchKernelGGL((k_pee_embed_ss<TT, NTV, IP, 4, PL>), dim3((unsigned)P->B), dim3(SS_THREADS), 0, st, \
            static_cast<const TT*>(cover), static_cast<TT*>(stego), P->H, P->W, P->T, P->maxval, lengths, tps, \
            reinterpret_cast<const u64*>(payload), P->payload_words, meta, reinterpret_cast<u64*>(lm), P->lm_words, \
            static_cast<char*>(workspace) + L.sink, 0, nullptr)
#define PES(TT, NTV, IP) do { if (pay_lds) PES1(TT, NTV, IP, true); else PES1(TT, NTV, IP, false); } while (0)
        // ring depth of the in-place embed: it does not know `end` in advance, so the D - 1
        // chunks it has in flight past it are wasted reads; at 256 x 2048^2 the steady state
        // is HBM-bound (~5 TB/s of reads + writes), and D = 2 keeps enough in flight:
        // 0.0825 -> 0.0789 ms (D = 3: 0.0824; tools/archive/ab_depth.sh).  D = 1 refills early (the
        // next chunk's loads go out before this chunk's barrier and compute): 0.0746 -> 0.0726
        // ms (profiles/r04/ip_early_ab.log).  CODEC_PEE_SS_D=2 / 4 restore the late refill.
        const long long ss_d = pay_lds ? knob("CODEC_PEE_SS_D", 1) : 4;
#define PES1D(TT, NTV, IP, DD) hipLaunchKernelGGL((k_pee_embed_ss<TT, NTV, IP, DD, true>), dim3((unsigned)P->B), dim3(SS_THREADS), 0, st, \
            static_cast<const TT*>(cover), static_cast<TT*>(stego), P->H, P->W, P->T, P->maxval, lengths, tps, \
            reinterpret_cast<const u64*>(payload), P->payload_words, meta, reinterpret_cast<u64*>(lm), P->lm_words, \
            static_cast<char*>(workspace) + L.sink, 0, nullptr)
        // in place, early ring of one: the load and store cache policies (CODEC_PEE_IP_NTL /
        // CODEC_PEE_IP_NTS; default non-temporal loads, plain stores, profiles/r05/ab_policy.txt)
        const bool ip_ntl = knob("CODEC_PEE_IP_NTL", 1) != 0, ip_nts = knob("CODEC_PEE_IP_NTS", 0) != 0;
#define PES1P(NTL, NTSV) hipLaunchKernelGGL((k_pee_embed_ss<uint16_t, NTL, true, 1, true, false, NTSV>), dim3((unsigned)P->B), \
            dim3(SS_THREADS), 0, st, static_cast<const uint16_t*>(cover), static_cast<uint16_t*>(stego), P->H, P->W, P->T, \
            P->maxval, lengths, tps, reinterpret_cast<const u64*>(payload), P->payload_words, meta, reinterpret_cast<u64*>(lm), \
            P->lm_words, static_cast<char*>(workspace) + L.sink, 0, nullptr)
        if (P->bytes == 2) {
            if (inplace) {
                if (ss_d == 2 && nt) PES1D(uint16_t, true, true, 2);
                else if (ss_d == 1 && nt) {
                    if (ip_ntl && ip_nts) PES1P(true, true);
                    else if (ip_ntl) PES1P(true, false);
                    else if (ip_nts) PES1P(false, true);
                    else PES1P(false, false);
                }
                else if (nt) PES(uint16_t, true, true); else PES(uint16_t, false, true);
            }
            else { if (nt) PES(uint16_t, true, false); else PES(uint16_t, false, false); }
        } else {
            if (inplace) { if (nt) PES(uint8_t, true, true); else PES(uint8_t, false, true); }
            else { if (nt) PES(uint8_t, true, false); else PES(uint8_t, false, false); }
        }
#undef PES
#undef PES1
#undef PES1D
#undef PES1P
        LAUNCH_CHECK("k_pee_embed_ss");
        if ((P->H & 1) && !inplace) HIP_TRY(pee_copy_last_rows(P, cover, stego, st));
        return 0;
    }
    if (vec && items > 0 && (long long)L.nchunks * P->B < 0x7FFFFFFFLL && onepass != 0) {
        u64* stw = reinterpret_cast<u64*>(static_cast<char*>(workspace) + L.st);
        uint32_t* ctl = reinterpret_cast<uint32_t*>(static_cast<char*>(workspace) + L.ctl);
        int mode = flat ? PEE_MODE_FLAT | (knob("CODEC_PEE_FLAT_TICKET", 0) ? 0 : PEE_MODE_NOTICKET)
                        : (knob("CODEC_PEE_1P_CHUNK_MAJOR", 1) ? PEE_MODE_CMAJOR : 0) |
                              (knob("CODEC_PEE_1P_NOTICKET", 1) ? PEE_MODE_NOTICKET : 0) |
                              ((int)(knob("CODEC_PEE_1P_GROUP", 32) / 8) << 8);
        // small out-of-place batches (flat slots, no ticket) clean up after themselves: no
        // zeroing launch (C2: one launch of ~2 us fewer per call); meta is written without
        // atomics out of place, so only in place (and the ticket modes) zero it
        if (flat && (mode & PEE_MODE_NOTICKET) && knob("CODEC_PEE_SELFCLEAN", 1) && pee_sc_fits(P, st, workspace)) mode |= PEE_MODE_SC;
        if (!(mode & PEE_MODE_SC))
            HIP_TRY(pee_zero(st, stw, L.ctl - L.st + PEE_CTL_WORDS(P->B, L.nchunks) * 4, meta, (size_t)P->B * sizeof(codec_pee_meta),
                             inplace ? lm : nullptr, inplace ? (size_t)P->B * P->lm_words * 8 : 0));
        bool sc_fresh = false;
        const int sc_epoch = (mode & PEE_MODE_SC) ? pee_ws_epoch(workspace, &sc_fresh) : 0;
        if (sc_fresh)   // a pointer never seen: start its self-cleaning state clean
            HIP_TRY(pee_zero(st, stw, L.ctl - L.st + PEE_CTL_WORDS(P->B, L.nchunks) * 4));
        ProfScope prof(st, CODEC_K_PEE_EMBED1);
        const long long total = pee_total_slots(P->B, L.nchunks, pee_group8(P->B, mode, inplace));
        long long g = knob(inplace ? "CODEC_PEE_IP_WGS" : "CODEC_PEE_1P_WGS", inplace ? 2048 : (1 << 30));
        if (g > total) g = total;
        g = (g + 7) / 8 * 8;   // keep every workgroup on one slot lane (pee_slot)
        const uint32_t spin_max = (uint32_t)debug_knob("CODEC_PEE_LB_SPINS", inplace ? (1 << 22) : (1 << 14));
        const int dbg_skip = (int)debug_knob("CODEC_PEE_DEBUG_SKIP", 0) - 1;
        const int dbg_stale = (int)debug_knob("CODEC_PEE_DEBUG_STALE", 0) - 1;
        uint32_t* diag = reinterpret_cast<uint32_t*>(static_cast<char*>(workspace) + L.diag);
#define PE1S(TT, NTV, IP, SCV) hipLaunchKernelGGL((k_pee_embed1<TT, NTV, IP, SCV>), dim3((unsigned)g), dim3(256), 0, st, \
            static_cast<const TT*>(cover), static_cast<TT*>(stego), P->H, P->W, P->T, P->maxval, lengths, \
            reinterpret_cast<const u64*>(payload), P->payload_words, L.nchunks, P->B, stw, ctl, meta, \
            reinterpret_cast<u64*>(lm), P->lm_words, mode, spin_max, dbg_skip, diag, tps, sc_epoch, dbg_stale)
#define PE1(TT, NTV, IP) do { if (!(IP) && (mode & PEE_MODE_SC)) PE1S(TT, NTV, false, true); else PE1S(TT, NTV, IP, false); } while (0)
        if (P->bytes == 2) {
            if (inplace) { if (nt) PE1(uint16_t, true, true); else PE1(uint16_t, false, true); }
            else { if (nt) PE1(uint16_t, true, false); else PE1(uint16_t, false, false); }
        } else {
            if (inplace) { if (nt) PE1(uint8_t, true, true); else PE1(uint8_t, false, true); }
            else { if (nt) PE1(uint8_t, true, false); else PE1(uint8_t, false, false); }
        }
#undef PE1
#undef PE1S
        LAUNCH_CHECK("k_pee_embed1");
        // odd H: the last row of each slice belongs to no row pair (no candidate, no MED
        // neighbour); out of place it is copied verbatim
        if ((P->H & 1) && !inplace) HIP_TRY(pee_copy_last_rows(P, cover, stego, st));
        return 0;
    }
    HIP_TRY(hipMemsetAsync(lm, 0, (size_t)P->B * P->lm_words * 8, st));
    {
        ProfScope prof(st, CODEC_K_PEE_SCAN);
        const int ntiles = L.ntiles_max;
        const long long target = knob("CODEC_PEE_SCAN_WGS", 32768);
        int per = (int)((ntiles * (long long)P->B + target - 1) / target);
        if (per < 1) per = 1;
        dim3 grid((ntiles + per - 1) / per, P->B);
        if (vec) {
            const long long tot = (long long)ntiles * P->B;
            long long gw = knob("CODEC_PEE_SCAN_GS_WGS", 32768);   // tools/tune_pee.py
            if (gw > (tot + 3) / 4) gw = (tot + 3) / 4;
            if (gw < 1) gw = 1;
#define PSCAN(TT, NTV) hipLaunchKernelGGL((k_pee_scan<TT, NTV>), dim3((unsigned)gw), dim3(256), 0, st, static_cast<const TT*>(cover), static_cast<TT*>(stego), P->H, P->W, P->T, P->maxval, cnt, L.ntiles_max, P->B, tps)
            if (P->bytes == 2) { if (nt) PSCAN(uint16_t, true); else PSCAN(uint16_t, false); }
            else { if (nt) PSCAN(uint8_t, true); else PSCAN(uint8_t, false); }
#undef PSCAN
            LAUNCH_CHECK("k_pee_scan");
        } else {
            if (!inplace) HIP_TRY(hipMemcpyAsync(stego, cover, (size_t)npx * P->B * P->bytes, hipMemcpyDeviceToDevice, st));
            if (P->bytes == 2)
                hipLaunchKernelGGL(k_pee_count<uint16_t>, grid, dim3(256), 0, st, static_cast<const uint16_t*>(cover),
                                   P->H, P->W, P->T, P->maxval, per, cnt, L.ntiles_max, tps);
            else
                hipLaunchKernelGGL(k_pee_count<uint8_t>, grid, dim3(256), 0, st, static_cast<const uint8_t*>(cover),
                                   P->H, P->W, P->T, P->maxval, per, cnt, L.ntiles_max, tps);
            LAUNCH_CHECK("k_pee_count");
        }
    }
    {
        ProfScope prof(st, CODEC_K_PEE_LOCATE);
        if (P->bytes == 2)
            hipLaunchKernelGGL(k_pee_locate<uint16_t>, dim3(P->B), dim3(256), 0, st, static_cast<const uint16_t*>(cover),
                               P->H, P->W, P->T, P->maxval, lengths, cnt, off, L.ntiles_max, meta, tps);
        else
            hipLaunchKernelGGL(k_pee_locate<uint8_t>, dim3(P->B), dim3(256), 0, st, static_cast<const uint8_t*>(cover),
                               P->H, P->W, P->T, P->maxval, lengths, cnt, off, L.ntiles_max, meta, tps);
        LAUNCH_CHECK("k_pee_locate");
    }
    {
        ProfScope prof(st, CODEC_K_PEE_EMBED);
        const int g = (int)knob("CODEC_PEE_EMBED_WGS", 64);
        dim3 grid(g < L.ntiles_max ? g : L.ntiles_max, P->B);
        if (vec && knob("CODEC_PEE_EMBED_V", 1)) {
            if (P->bytes == 2)
                hipLaunchKernelGGL(k_pee_embed_v<uint16_t>, grid, dim3(256), 0, st, static_cast<const uint16_t*>(cover),
                                   static_cast<uint16_t*>(stego), P->H, P->W, reinterpret_cast<const u64*>(payload),
                                   P->payload_words, off, L.ntiles_max, meta, reinterpret_cast<u64*>(lm), P->lm_words);
            else
                hipLaunchKernelGGL(k_pee_embed_v<uint8_t>, grid, dim3(256), 0, st, static_cast<const uint8_t*>(cover),
                                   static_cast<uint8_t*>(stego), P->H, P->W, reinterpret_cast<const u64*>(payload),
                                   P->payload_words, off, L.ntiles_max, meta, reinterpret_cast<u64*>(lm), P->lm_words);
            LAUNCH_CHECK("k_pee_embed_v");
            return 0;
        }
#define PEMB(TT, VV) hipLaunchKernelGGL((k_pee_embed<TT, VV>), grid, dim3(256), 0, st, static_cast<const TT*>(cover), \
                               static_cast<TT*>(stego), P->H, P->W, reinterpret_cast<const u64*>(payload), \
                               P->payload_words, off, L.ntiles_max, meta, reinterpret_cast<u64*>(lm), P->lm_words)
        if (P->bytes == 2) { if (vec) PEMB(uint16_t, true); else PEMB(uint16_t, false); }
        else { if (vec) PEMB(uint8_t, true); else PEMB(uint8_t, false); }
#undef PEMB
        LAUNCH_CHECK("k_pee_embed");
    }
    return 0;
}

int codec_pee_embed_auto(const codec_pee_params* P, const void* cover, void* stego, const uint64_t* payload,
                         const int32_t* lengths, int32_t tmax, int32_t* t_out, codec_pee_meta* meta, uint64_t* lm,
                         void* workspace, size_t workspace_bytes, void* stream) {
    int rc = pee_check(P);
    if (rc) return rc;
    if (!cover || !stego || !payload || !lengths || !t_out || !meta || !lm || !workspace)
        return set_err(CODEC_EINVAL, "codec_pee_embed_auto: NULL pointer argument");
    if (tmax < 1 || tmax > PEE_TMAX_MAX) return set_err(CODEC_EINVAL, "tmax must be in 1..64");
    const PeeWs L = pee_ws(P);
    if (workspace_bytes < L.total) return set_err(CODEC_EINVAL, "workspace too small");
    HIP_TRY(pee_ws_enter(workspace, P, L, as_stream(stream)));   // another shape's state: zeroed first
    hipStream_t st = as_stream(stream);
    const bool inplace = cover == stego;
    const bool vec = (P->W % 8) == 0 && ((uintptr_t)cover % 16) == 0 && ((uintptr_t)stego % 16) == 0;
    const long long items = (long long)(P->H / 2) * (P->W / 8);
    // fused single launch where the embed is slice-serial anyway (chip-filling batches of
    // <= 64-chunk slices, e.g. C3, or in place) and the counters fit beside the payload in
    // the LDS pad; elsewhere the capacity pass and the per-slice-T embed as two launches
    const bool fused = P->bytes == 2 && vec && items > 0 && knob("CODEC_PEE_ONEPASS", -1) != 0 &&
                       knob("CODEC_PEE_AUTO_FUSED", 1) != 0 && tmax <= SS_AUTO_TMAX &&
                       P->payload_words <= SS_PAY_WORDS && knob("CODEC_PEE_SS_PAYLDS", 1) != 0 &&
                       2LL * P->payload_words <= (long long)SS_AUTO_CNT_BASE(tmax) && pee_use_slice_serial(P, inplace);
    if (!fused) {
        rc = codec_pee_capacity(P, cover, tmax, lengths, nullptr, t_out, workspace, workspace_bytes, stream);
        if (rc) return rc;
        return codec_pee_embed_ts(P, cover, stego, payload, lengths, t_out, meta, lm, workspace, workspace_bytes, stream);
    }
    const bool nt = knob("CODEC_NT", 1) != 0;
    // resident variant (out of place, slices of <= 512 x 32 items, e.g. C3 / C4's 512^2): the
    // cover is read once and kept on the CU between the capacity and the embed phase
    // threads of the resident workgroup: 512 (two waves per SIMD, up to 32 items per lane in
    // 256 registers) or 1024 (four waves per SIMD, up to 16 items per lane in 128); 1024 where
    // it holds the slice (C3's 512^2, phase trace: last workgroup done at 55.4 -> 52.4 us, embed
    // phase 14.4 -> 12.8 us), else 512
    const long long kth = knob("CODEC_PEE_RES_THREADS", 0);
    auto res_fits = [&](int n) {   // items per lane in registers; payload below the counters / ranks
        return (items + n - 1) / n <= (n == 512 ? 32 : 16) && 2LL * P->payload_words + 2 <= RES_PAD_WORDS - 16LL * n;
    };
    auto lin_fits = [&]() {   // LIN layout: payload below the error words and the counters
        return 2LL * P->payload_words + 2 <= RES_PAD_WORDS_LIN - 24LL * 1024;
    };
    const int nth = kth == 512 ? 512 : kth == 1024 ? 1024 : res_fits(1024) ? 1024 : 512;
    const long long nres = (items + nth - 1) / nth;
    const long long CRl = P->W / 8;
    const bool lin = nth == 1024 && (items == 8 * 1024 || items == 16 * 1024) && 1024 % CRl == 0 && lin_fits() &&
                     knob("CODEC_PEE_RES_LIN", 1) != 0;
    if (!inplace && knob("CODEC_PEE_RES", 1) != 0 && res_fits(nth) && tmax <= SS_AUTO_TMAX) {
        ProfScope prof(st, CODEC_K_PEE_EMBED_RES);
#define PRES(NI, NTV, NTS, NTH, LN) hipLaunchKernelGGL((k_pee_embed_res<NI, NTV, NTS, NTH, LN>), dim3((unsigned)P->B), dim3(NTH), 0, st, \
            static_cast<const uint16_t*>(cover), static_cast<uint16_t*>(stego), P->H, P->W, P->maxval, lengths, \
            reinterpret_cast<const u64*>(payload), P->payload_words, meta, reinterpret_cast<u64*>(lm), P->lm_words, \
            static_cast<char*>(workspace) + L.sink, (int)tmax, t_out, trace)
        const int trace = (int)knob("CODEC_PEE_RES_TRACE", 0);
        // non-temporal loads, plain stores (nt stores: read phase 29.6 -> 32.5 us at C3);
        // CODEC_PEE_RES_NTS=1 / CODEC_NT=0 for A/B
        const bool nts = knob("CODEC_PEE_RES_NTS", 0) != 0;
#define PRESN(NI, NTH, LN) do { if (!nt) PRES(NI, false, false, NTH, LN); else if (nts) PRES(NI, true, true, NTH, LN); \
                                else PRES(NI, true, false, NTH, LN); } while (0)
        if (nth == 1024) {
            if (lin) { if (nres <= 8) PRESN(8, 1024, true); else PRESN(16, 1024, true); }
            else if (nres <= 8) PRESN(8, 1024, false);
            else PRESN(16, 1024, false);
        }
        else if (nres <= 8) PRESN(8, 512, false);
        else if (nres <= 16) PRESN(16, 512, false);
        else PRESN(32, 512, false);
#undef PRESN
#undef PRES
        LAUNCH_CHECK("k_pee_embed_res");
        if (P->H & 1) HIP_TRY(pee_copy_last_rows(P, cover, stego, st));
        return 0;
    }
    ProfScope prof(st, CODEC_K_PEE_EMBED_SS_AUTO);
#define PEA(NTV, IP, DD) hipLaunchKernelGGL((k_pee_embed_ss<uint16_t, NTV, IP, DD, true, true>), dim3((unsigned)P->B), \
            dim3(SS_THREADS), 0, st, static_cast<const uint16_t*>(cover), static_cast<uint16_t*>(stego), P->H, P->W, \
            P->T, P->maxval, lengths, nullptr, reinterpret_cast<const u64*>(payload), P->payload_words, meta, \
            reinterpret_cast<u64*>(lm), P->lm_words, static_cast<char*>(workspace) + L.sink, (int)tmax, t_out)
    // ring depths as in codec_pee_embed_ts (in place 2, out of place 4)
    if (inplace) { if (nt) PEA(true, true, 2); else PEA(false, true, 2); }
    else { if (nt) PEA(true, false, 4); else PEA(false, false, 4); }
#undef PEA
    LAUNCH_CHECK("k_pee_embed_ss(auto)");
    if ((P->H & 1) && !inplace) HIP_TRY(pee_copy_last_rows(P, cover, stego, st));
    return 0;
}

int codec_pee_extract(const codec_pee_params* P, const void* stego, const codec_pee_meta* meta, const uint64_t* lm,
                      void* cover_out, uint64_t* payload_out, void* workspace, size_t workspace_bytes, void* stream) {
    int rc = pee_check(P);
    if (rc) return rc;
    if (!stego || !meta || !lm || !cover_out || !payload_out || !workspace)
        return set_err(CODEC_EINVAL, "codec_pee_extract: NULL pointer argument");
    const PeeWs L = pee_ws(P);
    if (workspace_bytes < L.total) return set_err(CODEC_EINVAL, "workspace too small");
    HIP_TRY(pee_ws_enter(workspace, P, L, as_stream(stream)));   // another shape's state: zeroed first
    hipStream_t st = as_stream(stream);
    uint32_t* cnt = reinterpret_cast<uint32_t*>(static_cast<char*>(workspace) + L.cnt);
    uint32_t* off = reinterpret_cast<uint32_t*>(static_cast<char*>(workspace) + L.off);
    const long long nbytes = (long long)P->H * P->W * P->B * P->bytes;
    const bool nt = knob("CODEC_PEE_X_NT", knob("CODEC_NT", 1)) != 0;   // CODEC_PEE_X_NT: extract only (A/B)
    const size_t va = P->bytes == 2 ? 16 : 8;
    const bool vec = (P->W % 8) == 0 && ((uintptr_t)stego % va) == 0 && ((uintptr_t)cover_out % va) == 0;
    const long long items = (long long)(P->H / 2) * (P->W / 8);
    const bool inplace = stego == cover_out;
    const long long onepass = knob("CODEC_PEE_ONEPASS", -1);   // as in codec_pee_embed
    if (vec && items > 0 && onepass != 0 && pee_use_slice_serial(P, inplace)) {
        // slice-serial: writes every payload word itself (no memset) and never sets the flag
        uint32_t* ctl = reinterpret_cast<uint32_t*>(static_cast<char*>(workspace) + L.ctl);
        ProfScope prof(st, CODEC_K_PEE_EXTRACT_SS);
#define PXSD(TT, NTV, IP, DD) hipLaunchKernelGGL((k_pee_extract_ss<TT, NTV, IP, DD>), dim3((unsigned)P->B), dim3(SS_THREADS), 0, st, \
            static_cast<const TT*>(stego), static_cast<TT*>(cover_out), P->H, P->W, meta, reinterpret_cast<const u64*>(lm), \
            P->lm_words, reinterpret_cast<u64*>(payload_out), P->payload_words, ctl + 1, static_cast<char*>(workspace) + L.sink)
#define PXS(TT, NTV, IP) PXSD(TT, NTV, IP, 4)
        // ring depth (knob: 2, 4, 6).  Out of place (slices of <= 64 chunks, e.g. C3) 2: the
        // ring refills right behind the chunk, 0.0531 -> 0.0517 ms at 256 x 512^2; in place 4
        // (2: 0.0747 -> 0.0761 ms at 256 x 2048^2; 6 is slower everywhere, 0.064 / 0.086)
        const long long xd = knob("CODEC_PEE_SSX_D", inplace ? 4 : 2);
        // early refill (the slot reloaded as soon as its data is taken): in place a ring of one
        // refilled early beats the late ring of 4, 0.0752 -> 0.0726 ms (profiles/r04/ip_xearly_ab.log);
        // CODEC_PEE_SSX_EARLY=0 restores the late refill (then CODEC_PEE_SSX_D picks 2 / 4 / 6)
        const bool xe = knob("CODEC_PEE_SSX_EARLY", inplace ? 1 : 0) != 0;
        const long long xde = knob("CODEC_PEE_SSX_D", inplace ? 1 : 2);
#define PXSE(IP, DD) hipLaunchKernelGGL((k_pee_extract_ss<uint16_t, true, IP, DD, true>), dim3((unsigned)P->B), dim3(SS_THREADS), 0, st, \
            static_cast<const uint16_t*>(stego), static_cast<uint16_t*>(cover_out), P->H, P->W, meta, reinterpret_cast<const u64*>(lm), \
            P->lm_words, reinterpret_cast<u64*>(payload_out), P->payload_words, ctl + 1, static_cast<char*>(workspace) + L.sink)
        // in place, early ring of one: cache policies as for the in-place embed (CODEC_PEE_IP_NTL / _NTS)
        const bool xip_ntl = knob("CODEC_PEE_IP_NTL", 1) != 0, xip_nts = knob("CODEC_PEE_IP_NTS", 0) != 0;
#define PXSP(NTL, NTSV) hipLaunchKernelGGL((k_pee_extract_ss<uint16_t, NTL, true, 1, true, NTSV>), dim3((unsigned)P->B), \
            dim3(SS_THREADS), 0, st, static_cast<const uint16_t*>(stego), static_cast<uint16_t*>(cover_out), P->H, P->W, meta, \
            reinterpret_cast<const u64*>(lm), P->lm_words, reinterpret_cast<u64*>(payload_out), P->payload_words, ctl + 1, \
            static_cast<char*>(workspace) + L.sink)
        if (P->bytes == 2 && nt && xe) {
            if (inplace) {
                if (xde == 1) {
                    if (xip_ntl && xip_nts) PXSP(true, true);
                    else if (xip_ntl) PXSP(true, false);
                    else if (xip_nts) PXSP(false, true);
                    else PXSP(false, false);
                }
                else if (xde == 2) PXSE(true, 2); else PXSE(true, 4);
            }
            else { if (xde == 1) PXSE(false, 1); else if (xde == 2) PXSE(false, 2); else PXSE(false, 4); }
        } else if (P->bytes == 2 && nt && xd != 4) {
            if (inplace) { if (xd == 2) PXSD(uint16_t, true, true, 2); else PXSD(uint16_t, true, true, 6); }
            else { if (xd == 2) PXSD(uint16_t, true, false, 2); else PXSD(uint16_t, true, false, 6); }
        } else if (P->bytes == 2) {
            if (inplace) { if (nt) PXS(uint16_t, true, true); else PXS(uint16_t, false, true); }
            else { if (nt) PXS(uint16_t, true, false); else PXS(uint16_t, false, false); }
        } else {
            if (inplace) { if (nt) PXS(uint8_t, true, true); else PXS(uint8_t, false, true); }
            else { if (nt) PXS(uint8_t, true, false); else PXS(uint8_t, false, false); }
        }
#undef PXS
#undef PXSD
#undef PXSE
#undef PXSP
        LAUNCH_CHECK("k_pee_extract_ss");
        if ((P->H & 1) && !inplace) HIP_TRY(pee_copy_last_rows(P, stego, cover_out, st));
        return 0;
    }
    const bool flat = !inplace && P->B < 32 && P->B <= knob("CODEC_PEE_FLAT_MAXB", 7);
    if (vec && items > 0 && (long long)L.nchunks * P->B < 0x7FFFFFFFLL && onepass != 0) {
        u64* stw = reinterpret_cast<u64*>(static_cast<char*>(workspace) + L.st);
        uint32_t* ctl = reinterpret_cast<uint32_t*>(static_cast<char*>(workspace) + L.ctl);
        int mode = flat ? PEE_MODE_FLAT | (knob("CODEC_PEE_FLAT_TICKET", 0) ? 0 : PEE_MODE_NOTICKET)
                        : (knob("CODEC_PEE_X_CHUNK_MAJOR", knob("CODEC_PEE_1P_CHUNK_MAJOR", 1)) ? PEE_MODE_CMAJOR : 0) |
                              (knob("CODEC_PEE_X_NOTICKET", 1) ? PEE_MODE_NOTICKET : 0) |
                              ((int)(knob("CODEC_PEE_X_GROUP", 32) / 8) << 8);
        if (flat && (mode & PEE_MODE_NOTICKET) && knob("CODEC_PEE_SELFCLEAN", 1) && pee_sc_fits(P, st, workspace)) mode |= PEE_MODE_SC;
        if (!(mode & PEE_MODE_SC))
            HIP_TRY(pee_zero(st, payload_out, (size_t)P->B * P->payload_words * 8, stw, L.ctl - L.st + PEE_CTL_WORDS(P->B, L.nchunks) * 4));
        bool sc_fresh = false;
        const int sc_epoch = (mode & PEE_MODE_SC) ? pee_ws_epoch(workspace, &sc_fresh) : 0;
        if (sc_fresh)   // a pointer never seen: start its self-cleaning state clean
            HIP_TRY(pee_zero(st, stw, L.ctl - L.st + PEE_CTL_WORDS(P->B, L.nchunks) * 4));
        ProfScope prof(st, CODEC_K_PEE_EXTRACT1);
        const long long total = pee_total_slots(P->B, L.nchunks, pee_group8(P->B, mode, inplace));
        long long g = knob(inplace ? "CODEC_PEE_IP_WGS" : "CODEC_PEE_1P_WGS", inplace ? 2048 : (1 << 30));
        if (g > total) g = total;
        g = (g + 7) / 8 * 8;
        const uint32_t spin_max = (uint32_t)debug_knob("CODEC_PEE_LB_SPINS", inplace ? (1 << 22) : (1 << 14));
        const int dbg_skip = (int)debug_knob("CODEC_PEE_DEBUG_SKIP", 0) - 1;
        const int dbg_stale = (int)debug_knob("CODEC_PEE_DEBUG_STALE", 0) - 1;
        uint32_t* diag = reinterpret_cast<uint32_t*>(static_cast<char*>(workspace) + L.diag);
#define PX1S(TT, NTV, IP, SCV) hipLaunchKernelGGL((k_pee_extract1<TT, NTV, IP, SCV>), dim3((unsigned)g), dim3(256), 0, st, \
            static_cast<const TT*>(stego), static_cast<TT*>(cover_out), P->H, P->W, meta, reinterpret_cast<const u64*>(lm), \
            P->lm_words, L.nchunks, P->B, stw, ctl, reinterpret_cast<u64*>(payload_out), P->payload_words, mode, spin_max, \
            dbg_skip, diag, sc_epoch, dbg_stale)
#define PX1(TT, NTV, IP) do { if (!(IP) && (mode & PEE_MODE_SC)) PX1S(TT, NTV, false, true); else PX1S(TT, NTV, IP, false); } while (0)
        if (P->bytes == 2) {
            if (inplace) { if (nt) PX1(uint16_t, true, true); else PX1(uint16_t, false, true); }
            else { if (nt) PX1(uint16_t, true, false); else PX1(uint16_t, false, false); }
        } else {
            if (inplace) { if (nt) PX1(uint8_t, true, true); else PX1(uint8_t, false, true); }
            else { if (nt) PX1(uint8_t, true, false); else PX1(uint8_t, false, false); }
        }
#undef PX1
#undef PX1S
        LAUNCH_CHECK("k_pee_extract1");
        if ((P->H & 1) && !inplace) HIP_TRY(pee_copy_last_rows(P, stego, cover_out, st));
        return 0;
    }
    HIP_TRY(hipMemsetAsync(payload_out, 0, (size_t)P->B * P->payload_words * 8, st));
    {   // the single pass's look-back flag (codec_pee_extract_flag_offset) stays clear here
        uint32_t* ctl = reinterpret_cast<uint32_t*>(static_cast<char*>(workspace) + L.ctl);
        HIP_TRY(hipMemsetAsync(ctl + 1, 0, 4, st));
    }
    const bool fused = vec && knob("CODEC_PEE_FUSED", 1) != 0 && (P->W % 8) == 0 && items > 0 && (items % 256) == 0 &&
                       items * P->B < 0xFFFFFFFFLL;
    if (fused) {
        const int g = (int)knob("CODEC_PEE_EMBED_WGS", 64);
        dim3 grid(g < L.ntiles_max ? g : L.ntiles_max, P->B);
        {
            ProfScope prof(st, CODEC_K_PEE_DCOUNT);
            if (knob("CODEC_PEE_WAVE_TILES", 1)) {
                const int gw = (int)knob("CODEC_PEE_DCOUNT_W_WGS", 8);   // 4 waves (tiles) per workgroup
                dim3 gridw(gw, P->B);
#define PDCW(TT) hipLaunchKernelGGL((k_pee_dcount_w<TT>), gridw, dim3(256), 0, st, static_cast<const TT*>(stego), P->H, P->W, \
                               meta, reinterpret_cast<const u64*>(lm), P->lm_words, cnt, L.ntiles_max)
                if (P->bytes == 2) PDCW(uint16_t); else PDCW(uint8_t);
#undef PDCW
            } else {
#define PDC2(TT) hipLaunchKernelGGL((k_pee_dcount<TT, true>), grid, dim3(256), 0, st, static_cast<const TT*>(stego), P->H, P->W, \
                               meta, reinterpret_cast<const u64*>(lm), P->lm_words, cnt, L.ntiles_max)
                if (P->bytes == 2) PDC2(uint16_t); else PDC2(uint8_t);
#undef PDC2
            }
            LAUNCH_CHECK("k_pee_dcount");
            hipLaunchKernelGGL(k_pee_offsets, dim3(P->B), dim3(256), 0, st, meta, cnt, off, L.ntiles_max);
            LAUNCH_CHECK("k_pee_offsets");
        }
        ProfScope prof(st, CODEC_K_PEE_RECOVER);
        const uint32_t total = (uint32_t)(items * P->B);
        long long gg = (total + 1023) / 1024;
        const long long cap = knob("CODEC_PEE_RESTORE_WGS", 1 << 30);
        if (gg > cap) gg = cap;
#define PRG(TT, NTV) hipLaunchKernelGGL((k_pee_restore_gs<TT, NTV>), dim3((unsigned)gg), dim3(256), 0, st, static_cast<const TT*>(stego), \
                static_cast<TT*>(cover_out), P->H, P->W, (uint32_t)items, total, meta, reinterpret_cast<const u64*>(lm), P->lm_words, \
                off, L.ntiles_max, reinterpret_cast<u64*>(payload_out), P->payload_words)
        if (P->bytes == 2) { if (nt) PRG(uint16_t, true); else PRG(uint16_t, false); }
        else { if (nt) PRG(uint8_t, true); else PRG(uint8_t, false); }
#undef PRG
        LAUNCH_CHECK("k_pee_restore_gs");
        return 0;
    }
    {
        ProfScope prof(st, CODEC_K_PEE_COPY);
        if (((uintptr_t)stego % 16) == 0 && ((uintptr_t)cover_out % 16) == 0) {
            const int g = (int)knob("CODEC_PEE_COPY_WGS", 16384);
            if (P->bytes == 2) {
                if (nt) hipLaunchKernelGGL((k_pee_copy<uint16_t, true>), dim3(g), dim3(256), 0, st, static_cast<const uint16_t*>(stego), static_cast<uint16_t*>(cover_out), nbytes);
                else hipLaunchKernelGGL((k_pee_copy<uint16_t, false>), dim3(g), dim3(256), 0, st, static_cast<const uint16_t*>(stego), static_cast<uint16_t*>(cover_out), nbytes);
            } else {
                if (nt) hipLaunchKernelGGL((k_pee_copy<uint8_t, true>), dim3(g), dim3(256), 0, st, static_cast<const uint8_t*>(stego), static_cast<uint8_t*>(cover_out), nbytes);
                else hipLaunchKernelGGL((k_pee_copy<uint8_t, false>), dim3(g), dim3(256), 0, st, static_cast<const uint8_t*>(stego), static_cast<uint8_t*>(cover_out), nbytes);
            }
            LAUNCH_CHECK("k_pee_copy");
        } else {
            HIP_TRY(hipMemcpyAsync(cover_out, stego, (size_t)nbytes, hipMemcpyDeviceToDevice, st));
        }
    }
    const int g = (int)knob("CODEC_PEE_EMBED_WGS", 64);
    dim3 grid(g < L.ntiles_max ? g : L.ntiles_max, P->B);
    {
        ProfScope prof(st, CODEC_K_PEE_DCOUNT);
#define PDC(TT, VV) hipLaunchKernelGGL((k_pee_dcount<TT, VV>), grid, dim3(256), 0, st, static_cast<const TT*>(stego), P->H, P->W, \
                               meta, reinterpret_cast<const u64*>(lm), P->lm_words, cnt, L.ntiles_max)
        if (P->bytes == 2) { if (vec) PDC(uint16_t, true); else PDC(uint16_t, false); }
        else { if (vec) PDC(uint8_t, true); else PDC(uint8_t, false); }
#undef PDC
        LAUNCH_CHECK("k_pee_dcount");
        hipLaunchKernelGGL(k_pee_offsets, dim3(P->B), dim3(256), 0, st, meta, cnt, off, L.ntiles_max);
        LAUNCH_CHECK("k_pee_offsets");
    }
    {
        ProfScope prof(st, CODEC_K_PEE_RECOVER);
#define PREC(TT, VV) hipLaunchKernelGGL((k_pee_recover<TT, VV>), grid, dim3(256), 0, st, static_cast<const TT*>(stego), \
                               static_cast<TT*>(cover_out), P->H, P->W, meta, reinterpret_cast<const u64*>(lm), \
                               P->lm_words, off, L.ntiles_max, reinterpret_cast<u64*>(payload_out), P->payload_words)
        if (P->bytes == 2) { if (vec) PREC(uint16_t, true); else PREC(uint16_t, false); }
        else { if (vec) PREC(uint8_t, true); else PREC(uint8_t, false); }
#undef PREC
        LAUNCH_CHECK("k_pee_recover");
    }
    return 0;
}

}  // extern "C"

// ===================================================================== scheme 2: sublattices
// Four passes (oracle/pee_cpu.py, "Scheme 2"): pass p runs the scheme above on lattice p of
// the running image -- (odd, odd), (even, even), (odd, even), (even, odd) as (row, column)
// parities, y >= 1, x >= 1 -- taking the next min(remaining, capacity_p) payload bits; the
// decoder undoes them in reverse.  Each lattice's W / N / NW neighbours lie on the other
// three, so within a pass every candidate is independent and the pass runs in place: the
// tile kernels below read a candidate and its three neighbours and write only the candidate.
// The passes use tile counts (1024 candidates per tile, a workgroup of 256 lanes, 4
// consecutive candidates each) and a per-slice scan, as the two-pass scheme-1 path does;
// a pass with no bits left for a slice skips that slice's tiles (capacity reported as -1).
// Pass p's payload bits start at base_p = L_0 + ... + L_{p-1} of the slice (its earlier
// passes' records, `metas` = [passes][B]).
struct PeeLat {
    int y0, x0, hc, wc;
};
__host__ __device__ __forceinline__ PeeLat pee_lattice(int lat, int H, int W) {
    const bool ry = lat == 0 || lat == 2, rx = lat == 0 || lat == 3;
    PeeLat g;
    g.y0 = ry ? 1 : 2;
    g.x0 = rx ? 1 : 2;
    g.hc = H - g.y0 + 1 > 0 ? (H - g.y0 + 1) / 2 : 0;
    g.wc = W - g.x0 + 1 > 0 ? (W - g.x0 + 1) / 2 : 0;
    return g;
}

// the 4 candidates k0 .. k0 + 3 (those <= kmax) of a lane: pixel offsets, values, neighbours
template <typename T>
struct LatQuad {
    size_t o[4];
    int x[4], a[4], b[4], c[4];
    __device__ __forceinline__ void load(const T* img, int W, const PeeLat& g, int k0, int kmax) {
        int i = k0 / g.wc, j = k0 - (k0 / g.wc) * g.wc;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            // candidates past kmax load pixel (1, 1) instead (in bounds whenever a lattice has a
            // candidate) and are ignored by the caller: no divergent loads
            const bool ok = k0 + u <= kmax;
            const size_t oo = ok ? (size_t)(g.y0 + 2 * i) * W + (size_t)(g.x0 + 2 * j) : (size_t)W + 1;
            o[u] = oo;
            x[u] = img[oo]; a[u] = img[oo - 1]; b[u] = img[oo - W]; c[u] = img[oo - W - 1];
            const bool wrap = j + 1 == g.wc;   // branch-free step to candidate k0 + u + 1
            i += wrap ? 1 : 0;
            j = wrap ? 0 : j + 1;
        }
    }
};

__device__ __forceinline__ int pee_pass_base(const codec_pee_meta* metas, int pass, int B, int b) {
    int base = 0;
    for (int q = 0; q < pass; ++q) base += metas[(size_t)q * B + b].L;
    return base;
}

template <typename T>
__global__ __launch_bounds__(256) void k_pee_lat_count(const T* __restrict__ img, int H, int W, int lat, int T0,
                                                       int maxval, const int32_t* __restrict__ lengths,
                                                       const codec_pee_meta* __restrict__ metas, int pass, int B,
                                                       uint32_t* __restrict__ tile_cnt_all, int ntiles_max) {
    __shared__ uint32_t sh[8];
    const int b = blockIdx.y;
    if (lengths[b] - pee_pass_base(metas, pass, B, b) <= 0) return;   // nothing left: uniform
    const PeeLat g = pee_lattice(lat, H, W);
    const int nc = g.hc * g.wc, ntiles = (nc + PEE_TILE - 1) / PEE_TILE;
    const T* src = img + (size_t)b * H * W;
    for (int t = blockIdx.x; t < ntiles; t += gridDim.x) {
        const int k0 = t * PEE_TILE + 4 * threadIdx.x;
        LatQuad<T> q;
        q.load(src, W, g, k0, nc - 1);
        uint32_t cnt = 0;
#pragma unroll
        for (int u = 0; u < 4; ++u)
            if (k0 + u < nc) {
                const PeeCand pc = pee_classify(q.x[u], q.a[u], q.b[u], q.c[u], T0, maxval);
                cnt += (pc.expand && pc.safe) ? 1u : 0u;
            }
        const uint32_t tot = block_sum_u32<256>(cnt, sh);
        if (threadIdx.x == 0) tile_cnt_all[(size_t)b * ntiles_max + t] = tot;
    }
}

// per slice: tile offsets, this pass's L (min(remaining, capacity)), end, record
template <typename T>
__global__ __launch_bounds__(256) void k_pee_lat_locate(const T* __restrict__ img, int H, int W, int lat, int T0,
                                                        int maxval, const int32_t* __restrict__ lengths,
                                                        codec_pee_meta* __restrict__ metas, int pass, int B,
                                                        const uint32_t* __restrict__ tile_cnt_all,
                                                        uint32_t* __restrict__ tile_off_all, int ntiles_max) {
    __shared__ uint32_t sh[8];
    __shared__ int s_tile, s_end;
    __shared__ uint32_t s_base;
    const int b = blockIdx.x;
    const PeeLat g = pee_lattice(lat, H, W);
    const int nc = g.hc * g.wc, ntiles = (nc + PEE_TILE - 1) / PEE_TILE;
    const int rem = max(0, lengths[b] - pee_pass_base(metas, pass, B, b));
    codec_pee_meta* M = metas + (size_t)pass * B + b;
    if (rem == 0) {   // nothing left for this slice: the pass leaves it untouched
        if (threadIdx.x == 0) {
            M->T = T0; M->maxval = maxval; M->L = 0; M->end = -1; M->nc = nc; M->ntiles = ntiles; M->tile_end = -1;
            M->status = 0; M->capacity = -1; M->lm_count = 0; M->h = H; M->w = W; M->flags = 0;
            M->reserved[0] = lat; M->reserved[1] = 0; M->reserved[2] = 0;
        }
        return;
    }
    const uint32_t L = (uint32_t)rem;
    const uint32_t* cnt = tile_cnt_all + (size_t)b * ntiles_max;
    uint32_t* off = tile_off_all + (size_t)b * ntiles_max;
    if (threadIdx.x == 0) { s_tile = -1; s_end = -1; s_base = 0; }
    __syncthreads();
    uint32_t running = 0;
    for (int base = 0; base < ntiles; base += 256) {
        const int t = base + threadIdx.x;
        const uint32_t c = t < ntiles ? cnt[t] : 0u;
        uint32_t tot;
        const uint32_t ex = running + block_excl_scan<256>(c, sh, &tot);
        if (t < ntiles) off[t] = ex;
        if (t < ntiles && ex < L && ex + c >= L) { s_tile = t; s_base = ex; }
        running += tot;
    }
    __syncthreads();
    const int tile = s_tile;
    if (tile >= 0 && running >= L) {   // the L-th expandable candidate of `tile`
        const T* src = img + (size_t)b * H * W;
        const int k0 = tile * PEE_TILE + 4 * threadIdx.x;
        LatQuad<T> q;
        q.load(src, W, g, k0, nc - 1);
        uint32_t flags = 0, local = 0;
#pragma unroll
        for (int u = 0; u < 4; ++u)
            if (k0 + u < nc) {
                const PeeCand pc = pee_classify(q.x[u], q.a[u], q.b[u], q.c[u], T0, maxval);
                if (pc.expand && pc.safe) { flags |= 1u << u; ++local; }
            }
        uint32_t tot;
        const uint32_t pre = block_excl_scan<256>(local, sh, &tot);
        const uint32_t need = L - s_base;
        if (need > pre && need <= pre + local) {
            uint32_t r = pre;
#pragma unroll
            for (int u = 0; u < 4; ++u)
                if ((flags >> u) & 1u) {
                    ++r;
                    if (r == need) s_end = k0 + u;
                }
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        M->T = T0; M->maxval = maxval; M->nc = nc; M->ntiles = ntiles; M->capacity = (int)running;
        M->h = H; M->w = W; M->lm_count = 0; M->flags = 0;
        M->reserved[0] = lat; M->reserved[1] = 0; M->reserved[2] = 0;
        if (running < L) {   // the pass fills up: its capacity's bits, every candidate processed
            M->L = (int)running; M->end = nc - 1; M->tile_end = ntiles - 1; M->status = 1;
        } else {
            M->L = (int)L; M->end = s_end; M->tile_end = tile; M->status = 0;
        }
    }
}

// tiles <= tile_end, in place: expansion / shifting of the candidates, this pass's location map
template <typename T>
__global__ __launch_bounds__(256) void k_pee_lat_embed(T* __restrict__ img, int H, int W, int lat,
                                                       const u64* __restrict__ payload_all, int pw,
                                                       const uint32_t* __restrict__ tile_off_all, int ntiles_max,
                                                       codec_pee_meta* __restrict__ metas, int pass, int B,
                                                       u64* __restrict__ lm_all, int lmw) {
    __shared__ uint32_t sh[8];
    __shared__ uint32_t lm32[PEE_TILE / 32];
    const int b = blockIdx.y;
    codec_pee_meta* M = metas + (size_t)pass * B + b;
    const int tile_end = M->tile_end, end = M->end, Tthr = M->T, maxval = M->maxval;
    if (tile_end < 0) return;
    const uint32_t pbase = (uint32_t)pee_pass_base(metas, pass, B, b);
    const PeeLat g = pee_lattice(lat, H, W);
    T* dst = img + (size_t)b * H * W;
    const u64* payload = payload_all + (size_t)b * pw;
    u64* lm = lm_all + (size_t)b * lmw;
    const uint32_t* off = tile_off_all + (size_t)b * ntiles_max;
    for (int t = blockIdx.x; t <= tile_end; t += gridDim.x) {
        if (threadIdx.x < PEE_TILE / 32) lm32[threadIdx.x] = 0;
        const int k0 = t * PEE_TILE + 4 * threadIdx.x;
        LatQuad<T> q;
        q.load(dst, W, g, k0, end);
        PeeCand pc[4];
        uint32_t local = 0;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            pc[u].expand = pc[u].safe = pc[u].right = false;
            pc[u].x = pc[u].p = 0;
            if (k0 + u <= end) {
                pc[u] = pee_classify(q.x[u], q.a[u], q.b[u], q.c[u], Tthr, maxval);
                local += (pc[u].expand && pc[u].safe) ? 1u : 0u;
            }
        }
        uint32_t tot;
        uint32_t cur = pbase + off[t] + block_excl_scan<256>(local, sh, &tot);   // also orders lm32 zeroing
        uint32_t nib = 0, unsafe = 0;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            if (k0 + u > end) continue;
            if (!pc[u].safe) { nib |= 1u << u; ++unsafe; continue; }
            int nv;
            if (pc[u].expand) {
                const int bit = (int)(cur >> 6) < pw ? (int)((payload[cur >> 6] >> (cur & 63)) & 1ull) : 0;
                ++cur;
                nv = pc[u].p + 2 * (pc[u].x - pc[u].p) + bit;
            } else {
                nv = pc[u].right ? pc[u].x + Tthr : pc[u].x - Tthr;
            }
            dst[q.o[u]] = (T)nv;
        }
        if (nib) atomicOr(&lm32[(4 * threadIdx.x) >> 5], nib << ((4 * threadIdx.x) & 31));
        const uint32_t nun = block_sum_u32<256>(unsafe, sh);
        if (threadIdx.x < PEE_TILE / 64) {
            const int w = t * (PEE_TILE / 64) + threadIdx.x;
            if (w < lmw) lm[w] = (u64)lm32[2 * threadIdx.x] | ((u64)lm32[2 * threadIdx.x + 1] << 32);
        }
        if (threadIdx.x == 0 && nun) atomicAdd(&M->lm_count, (int)nun);
        __syncthreads();
    }
}

template <typename T>
__global__ __launch_bounds__(256) void k_pee_lat_dcount(const T* __restrict__ img, int H, int W, int lat,
                                                        const codec_pee_meta* __restrict__ metas, int pass, int B,
                                                        const u64* __restrict__ lm_all, int lmw,
                                                        uint32_t* __restrict__ tile_cnt_all, int ntiles_max) {
    __shared__ uint32_t sh[8];
    const int b = blockIdx.y;
    const codec_pee_meta* M = metas + (size_t)pass * B + b;
    const int tile_end = M->tile_end, end = M->end, Tthr = M->T;
    const PeeLat g = pee_lattice(lat, H, W);
    const T* src = img + (size_t)b * H * W;
    const u64* lm = lm_all + (size_t)b * lmw;
    for (int t = blockIdx.x; t <= tile_end; t += gridDim.x) {
        const int k0 = t * PEE_TILE + 4 * threadIdx.x;
        // the 4 candidates' location-map bits share one word (k0 % 4 == 0)
        const u64 lmw4 = (k0 >> 6) < lmw ? lm[k0 >> 6] : 0ull;
        LatQuad<T> q;
        q.load(src, W, g, k0, end);
        uint32_t local = 0;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int k = k0 + u;
            if (k <= end && !((lmw4 >> (k & 63)) & 1ull)) {
                const int e2 = q.x[u] - med3(q.a[u], q.b[u], q.c[u]);
                local += (e2 >= -2 * Tthr && e2 < 2 * Tthr) ? 1u : 0u;
            }
        }
        const uint32_t tot = block_sum_u32<256>(local, sh);
        if (threadIdx.x == 0) tile_cnt_all[(size_t)b * ntiles_max + t] = tot;
    }
}

// tiles <= tile_end, in place: the pass's bits (payload words OR-ed, zeroed by the caller)
// and the restored candidates
template <typename T>
__global__ __launch_bounds__(256) void k_pee_lat_recover(T* __restrict__ img, int H, int W, int lat,
                                                         const codec_pee_meta* __restrict__ metas, int pass, int B,
                                                         const u64* __restrict__ lm_all, int lmw,
                                                         const uint32_t* __restrict__ tile_off_all, int ntiles_max,
                                                         u64* __restrict__ payload_all, int pw) {
    __shared__ uint32_t sh[8];
    const int b = blockIdx.y;
    const codec_pee_meta* M = metas + (size_t)pass * B + b;
    const int tile_end = M->tile_end, end = M->end, Tthr = M->T;
    if (tile_end < 0) return;
    const uint32_t pbase = (uint32_t)pee_pass_base(metas, pass, B, b);
    const uint32_t plim = pbase + (uint32_t)max(0, M->L);
    const PeeLat g = pee_lattice(lat, H, W);
    T* dst = img + (size_t)b * H * W;
    const u64* lm = lm_all + (size_t)b * lmw;
    u64* payload = payload_all + (size_t)b * pw;
    const uint32_t* off = tile_off_all + (size_t)b * ntiles_max;
    for (int t = blockIdx.x; t <= tile_end; t += gridDim.x) {
        const int k0 = t * PEE_TILE + 4 * threadIdx.x;
        // the 4 candidates' location-map bits share one word (k0 % 4 == 0)
        const u64 lmw4 = (k0 >> 6) < lmw ? lm[k0 >> 6] : 0ull;
        LatQuad<T> q;
        q.load(dst, W, g, k0, end);
        int ps[4];
        bool act[4], inner[4];
        uint32_t local = 0;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int k = k0 + u;
            act[u] = k <= end && !((lmw4 >> (k & 63)) & 1ull);
            inner[u] = false;
            ps[u] = 0;
            if (act[u]) {
                ps[u] = med3(q.a[u], q.b[u], q.c[u]);
                const int e2 = q.x[u] - ps[u];
                inner[u] = e2 >= -2 * Tthr && e2 < 2 * Tthr;
                local += inner[u] ? 1u : 0u;
            }
        }
        uint32_t tot;
        uint32_t cur = pbase + off[t] + block_excl_scan<256>(local, sh, &tot);
        u64 word = 0;
        int wi = -1;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            if (!act[u]) continue;
            const int e2 = q.x[u] - ps[u];
            int x;
            if (inner[u]) {
                if ((e2 & 1) && cur < plim && (int)(cur >> 6) < pw) {   // consecutive bits: one atomic per word
                    if (wi != (int)(cur >> 6)) {
                        if (wi >= 0 && word) atomicOr(&payload[wi], word);
                        wi = (int)(cur >> 6);
                        word = 0;
                    }
                    word |= 1ull << (cur & 63);
                }
                ++cur;
                x = ps[u] + (e2 >> 1);
            } else {
                x = e2 >= 2 * Tthr ? q.x[u] - Tthr : q.x[u] + Tthr;
            }
            dst[q.o[u]] = (T)x;
        }
        if (wi >= 0 && word) atomicOr(&payload[wi], word);
    }
}

// ---- scheme 2, slice-serial: one 1024-thread workgroup per slice runs the (optional) copy and
// then every pass of the slice in one launch -- embed passes p_first..3 ascending, extract
// passes 3..0 descending -- with the payload cursor in a register.  The tile path above needs
// per pass a full-lattice count, a per-slice scan and the prefix pass (three launches) plus a
// stream copy; here a pass reads only the candidates up to its `end` (and the embed stops
// counting there: capacity is then the count through that chunk, flagged CODEC_PEE_PARTIAL
// like scheme 1's single pass).  Same records, pixels, maps and bits as the tile kernels
// (tests/test_pee.py runs both against the oracle).  A chunk = 4096 candidates, 4
// consecutive ones per lane (LatQuad's layout: lane t of chunk c holds candidates
// 4096 c + 4 t .. + 3, so the map's 64-candidate words are the 16-lane DPP rows); the next
// chunk's loads are issued before this one's scan (within a pass no candidate is a neighbour
// of another, so they never read a pixel the pass writes).  Passes are separated by a
// __syncthreads (workgroup-scope release/acquire: the next lattice reads this one's pixels).
#define LSS_THREADS 1024
#define LSS_CHUNK (4 * LSS_THREADS)
#define LSS_PAD_WORDS (21 * 1024)
   // 84 KB static LDS: one workgroup per CU, as k_pee_embed_ss

template <typename T>
__device__ __forceinline__ void lss_copy(const T* __restrict__ s, T* __restrict__ d, size_t npx, int mode) {
    const int tid = threadIdx.x;
    if (mode == 1) {   // 16-B vectors (slice bytes % 16 == 0, both bases aligned): 8 in flight per lane
        const size_t nv = npx * sizeof(T) / 16;
        const uint4* sv = reinterpret_cast<const uint4*>(s);
        uint4* dv = reinterpret_cast<uint4*>(d);
        size_t i = tid;
        for (; i + 7 * LSS_THREADS < nv; i += 8 * LSS_THREADS) {
            uint4 r[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) r[u] = ldv<true>(sv + i + u * LSS_THREADS);
#pragma unroll
            for (int u = 0; u < 8; ++u) dv[i + u * LSS_THREADS] = r[u];
        }
        for (; i < nv; i += LSS_THREADS) dv[i] = ldv<true>(sv + i);
    } else if (mode == 2) {
        for (size_t i = tid; i < npx; i += LSS_THREADS) d[i] = s[i];
    }
}

// PL: the slice's payload row staged in LDS (embed: read from it; extract: OR-ed into it, then
// written out whole) when 2 pw 32-bit words fit the pad; else global loads / atomics.  Every
// global store is unconditional -- a store that must not land goes to the wave's sink slot in
// the workspace, as in k_pee_embed_ss -- so hipcc's vmcnt counting stays exact and waiting for
// the next chunk's loads never drains this chunk's stores.
#define LSS_PAY_BASE 64
#define LSS_PAY_MAXW ((LSS_PAD_WORDS - LSS_PAY_BASE) / 2)
template <typename T, bool EXTRACT, bool PL, bool PF>
__global__ __launch_bounds__(LSS_THREADS) void k_pee_lat_ss(const T* __restrict__ src, T* dst, int H, int W, int T0,
                                                            int maxval, int copy_mode, int p_first,
                                                            u64* payload_all, int pw, const int32_t* __restrict__ lengths,
                                                            codec_pee_meta* metas, int B, u64* lm_all, int lmw,
                                                            char* __restrict__ sink) {
    __shared__ uint32_t pad[LSS_PAD_WORDS];   // [0..31]: wave totals (2 x 16), [32]: end, [33]: unsafe count
    uint32_t (*wtot)[16] = reinterpret_cast<uint32_t (*)[16]>(pad);
    uint32_t* pay32 = pad + LSS_PAY_BASE;
    const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63;
    const size_t npx = (size_t)H * W;
    T* img = dst + (size_t)b * npx;
    T* const sink_px = reinterpret_cast<T*>(sink + SS_SINK_SLOT(b, tid));
    u64* const sink_w = reinterpret_cast<u64*>(sink + SS_SINK_SLOT(b, tid) + 32);
    u64* payload = payload_all + (size_t)b * pw;
    if (PL) {   // embed: the payload row; extract: zeroed words the passes OR their bits into
        for (int w = tid; w < 2 * pw; w += LSS_THREADS)
            pay32[w] = EXTRACT ? 0u : reinterpret_cast<const uint32_t*>(payload)[w];
    } else if (EXTRACT) {
        for (int w = tid; w < pw; w += LSS_THREADS) payload[w] = 0ull;
    }
    if (copy_mode) lss_copy<T>(src + (size_t)b * npx, img, npx, copy_mode);
    __syncthreads();
    const uint32_t nbits = 64u * (uint32_t)pw;
    uint32_t base = 0;   // embed: payload bits taken by the passes before this one
    if (!EXTRACT && p_first == 1) {
        // pass 0 ran on scheme 1's kernels: its record is made scheme 2's here (k_pee_pass0_fix's
        // rule, idempotent -- L = the bits embedded, capacity when it filled up; lattice 0)
        codec_pee_meta* M0 = metas + b;
        const int L0 = M0->status == 1 ? M0->capacity : M0->L;
        base = (uint32_t)max(0, L0);
        if (tid == 0) { M0->L = L0; M0->reserved[0] = 0; }
    }
    int par = 0;
    for (int step = 0; step < (EXTRACT ? 4 : 4 - p_first); ++step) {
        const int p = EXTRACT ? 3 - step : p_first + step;
        const PeeLat g = pee_lattice(p, H, W);
        const int nc = g.hc * g.wc, ntiles = (nc + PEE_TILE - 1) / PEE_TILE;
        codec_pee_meta* M = metas + (size_t)p * B + b;
        u64* lm = lm_all + ((size_t)p * B + b) * lmw;
        int end, Tt;
        uint32_t pbase, lim;   // embed: lim = bits left; extract: lim = pbase + L
        if (EXTRACT) {
            if (M->tile_end < 0) continue;   // uniform
            end = M->end;
            Tt = M->T;
            pbase = 0;
            for (int q = 0; q < p; ++q) pbase += (uint32_t)max(0, metas[(size_t)q * B + b].L);
            lim = pbase + (uint32_t)max(0, M->L);
        } else {
            const int rem = lengths[b] - (int)base;
            if (rem <= 0) {   // nothing left: the pass leaves the slice untouched
                if (tid == 0) {
                    M->T = T0; M->maxval = maxval; M->L = 0; M->end = -1; M->nc = nc; M->ntiles = ntiles;
                    M->tile_end = -1; M->status = 0; M->capacity = -1; M->lm_count = 0; M->h = H; M->w = W;
                    M->flags = 0; M->reserved[0] = p; M->reserved[1] = 0; M->reserved[2] = 0;
                }
                continue;
            }
            end = nc - 1;   // until the chunk holding the rem-th expandable candidate is found
            Tt = T0;
            pbase = base;
            lim = (uint32_t)rem;
        }
        if (!EXTRACT && tid == 0) pad[33] = 0;
        const int kstop = EXTRACT ? end : nc - 1;   // last candidate a chunk may need
        const int nch = kstop >= 0 ? kstop / LSS_CHUNK + 1 : 0;
        uint32_t cursor = 0, unsafe = 0;   // rank of the chunk's first candidate (uniform); lane's unsafe count
        int c_done = nch;                  // embed: chunks walked
        bool found = false;
        // PF: the next chunk's loads are issued before this one is processed (one chunk in
        // flight; two in flight measured slower: 0.248 -> 0.324 ms C3 step).  extract: the 4
        // candidates' map word (k0 % 4 == 0) rides with the pixels; its index is clamped
        // (lmw * 64 >= nc > end: a lane past lmw has no active candidate)
        LatQuad<T> qa;
        u64 la = 0;
        auto request = [&](LatQuad<T>& qq, u64& ll, int c) {
            const int k0 = c * LSS_CHUNK + 4 * tid;
            qq.load(img, W, g, k0, kstop);   // clamped past kstop
            if (EXTRACT) ll = lm[min(k0 >> 6, lmw - 1)];
        };
        // one chunk; true when the embed has found `end` (the pass stops)
        auto chunk = [&](const LatQuad<T>& cur, const u64 lmw4, const int c) -> bool {
            const int k0 = c * LSS_CHUNK + 4 * tid;
                uint32_t n = 0, fl = 0;
                int ps[4];
    #pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const int k = k0 + u;
                    ps[u] = med3(cur.a[u], cur.b[u], cur.c[u]);
                    const int e = cur.x[u] - ps[u];
                    if (EXTRACT) {
                        const bool act = k <= end && !((lmw4 >> (k & 63)) & 1ull);
                        const bool inner = act && e >= -2 * Tt && e < 2 * Tt;
                        fl |= (act ? 1u : 0u) << u | (inner ? 16u : 0u) << u;
                        n += inner ? 1u : 0u;
                    } else {
                        const PeeCand pc = pee_classify(cur.x[u], cur.a[u], cur.b[u], cur.c[u], Tt, maxval);
                        const bool in = k < nc;
                        fl |= ((in & pc.expand & pc.safe) ? 1u : 0u) << u | ((in & pc.safe) ? 16u : 0u) << u |
                              ((in & pc.right) ? 256u : 0u) << u | (in ? 4096u : 0u) << u;
                        n += (in & pc.expand & pc.safe) ? 1u : 0u;
                    }
                }
                uint32_t ex, tot, wb;
                ss_scan_small(n, wtot, par, &ex, &tot, &wb);
                par ^= 1;
                const uint32_t r0 = cursor + ex;   // rank of this lane's first counted candidate
                if (EXTRACT) {
                    uint32_t r = pbase + r0;
                    uint32_t word = 0;
                    int wi = -1;
    #pragma unroll
                    for (int u = 0; u < 4; ++u) {
                        const bool act = (fl >> u) & 1u, inner = (fl >> (4 + u)) & 1u;
                        const int e2 = cur.x[u] - ps[u];
                        if (inner) {
                            if ((e2 & 1) && r < lim && r < nbits) {   // consecutive bits: one atomic per word
                                if (wi != (int)(r >> 5)) {
                                    if (wi >= 0 && word) {
                                        if (PL) atomicOr(&pay32[wi], word);
                                        else atomicOr(reinterpret_cast<uint32_t*>(payload) + wi, word);
                                    }
                                    wi = (int)(r >> 5);
                                    word = 0;
                                }
                                word |= 1u << (r & 31);
                            }
                            ++r;
                        }
                        const int x = inner ? ps[u] + (e2 >> 1) : (e2 >= 2 * Tt ? cur.x[u] - Tt : cur.x[u] + Tt);
                        *(act ? img + cur.o[u] : sink_px) = (T)x;
                    }
                    if (wi >= 0 && word) {
                        if (PL) atomicOr(&pay32[wi], word);
                        else atomicOr(reinterpret_cast<uint32_t*>(payload) + wi, word);
                    }
                    cursor += tot;
                    return false;
                }
                // embed: candidate k is processed iff fewer than lim expandable ones precede it
                const bool last = cursor + tot >= lim;   // this chunk holds the lim-th (uniform)
                uint32_t r = r0, nib = 0;
    #pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const bool proc = ((fl >> (12 + u)) & 1u) && r < lim;   // before nc and up to end
                    const bool safe = (fl >> (4 + u)) & 1u, es = (fl >> u) & 1u;
                    nib |= (proc && !safe) ? 1u << u : 0u;
                    unsafe += (proc && !safe) ? 1u : 0u;
                    const uint32_t bi = pbase + r;
                    uint32_t bit;
                    if (PL) {
                        const uint32_t wv = pay32[min(bi >> 5, (uint32_t)(2 * pw - 1))];
                        bit = bi < nbits ? (wv >> (bi & 31)) & 1u : 0u;
                    } else {
                        bit = (proc && es && bi < nbits) ? (uint32_t)((payload[bi >> 6] >> (bi & 63)) & 1ull) : 0u;
                    }
                    if (proc && es && r + 1 == lim) pad[32] = (uint32_t)(k0 + u);
                    const int nv = es ? ps[u] + 2 * (cur.x[u] - ps[u]) + (int)bit
                                      : (((fl >> (8 + u)) & 1u) ? cur.x[u] + Tt : cur.x[u] - Tt);
                    *(proc && safe ? img + cur.o[u] : sink_px) = (T)nv;
                    r += (proc && es) ? 1u : 0u;
                }
                // this chunk's map words (its 16-lane rows); in the chunk holding `end` only those of
                // tiles <= end's tile (the tile path writes whole tiles up to tile_end)
                const u64 word = row_or16_64((u64)nib << (4 * (lane & 15)));
                int tile_lim = ntiles - 1;
                if (last) {
                    lds_barrier();   // pad[32] (end) visible
                    end = (int)pad[32];
                    tile_lim = end / PEE_TILE;
                    found = true;
                }
                const int w = k0 >> 6;
                *((lane & 15) == 0 && w < lmw && (k0 / PEE_TILE) <= tile_lim ? lm + w : sink_w) = word;
                cursor += tot;
                if (last) { c_done = c + 1; return true; }
                return false;
        };
        if (PF && nch > 0) request(qa, la, 0);
        for (int c = 0; c < nch; ++c) {
            LatQuad<T> cur;
            u64 lw = 0;
            if (PF) {
                cur = qa;
                lw = la;
                request(qa, la, c + 1);
            } else {
                request(cur, lw, c);
            }
            if (chunk(cur, lw, c)) break;
        }
        if (EXTRACT) {
            __syncthreads();   // the next (lower) pass reads this lattice's restored pixels
            continue;
        }
        if (unsafe) atomicAdd(&pad[33], unsafe);   // rare: candidates whose transform would overflow
        __syncthreads();   // pad[33] complete; the next pass reads this lattice's pixels
        if (tid == 0) {
            M->T = T0; M->maxval = maxval; M->nc = nc; M->ntiles = ntiles; M->h = H; M->w = W;
            M->lm_count = (int)pad[33];
            M->reserved[0] = p; M->reserved[1] = 0; M->reserved[2] = 0;
            if (!found) {   // the pass fills up: its capacity's bits, every candidate processed
                M->L = (int)cursor; M->end = nc - 1; M->tile_end = ntiles - 1; M->status = 1;
                M->capacity = (int)cursor; M->flags = 0;
            } else {
                M->L = (int)lim; M->end = end; M->tile_end = end / PEE_TILE; M->status = 0;
                M->capacity = (int)cursor;   // counted through end's chunk: exact only if it is the last
                M->flags = c_done < (nc + LSS_CHUNK - 1) / LSS_CHUNK ? CODEC_PEE_PARTIAL : 0;
            }
        }
        base += found ? lim : cursor;
        __syncthreads();   // pad[32..33] reusable
    }
    if (EXTRACT && PL) {   // the payload row, whole (the passes' last barrier ordered the ORs)
        __syncthreads();
        for (int w = tid; w < pw; w += LSS_THREADS)
            payload[w] = (u64)pay32[2 * w] | ((u64)pay32[2 * w + 1] << 32);
    }
}

// pass 0 is scheme 1 on its own lattice: its record keeps the number of bits it embedded in L
// (scheme 1 keeps the requested length there and its capacity when it fills up)
__global__ __launch_bounds__(256) void k_pee_pass0_fix(codec_pee_meta* __restrict__ metas, int B) {
    const int b = blockIdx.x * 256 + threadIdx.x;
    if (b >= B) return;
    codec_pee_meta* M = metas + b;
    if (M->status == 1) M->L = M->capacity;
    M->reserved[0] = 0;
}

static int pee_multi_check(const codec_pee_params* P, int pass) {
    int rc = pee_check(P);
    if (rc) return rc;
    if (pass < 0 || pass > 3) return set_err(CODEC_EINVAL, "pass must be in 0..3");
    if ((long long)P->B * P->H * P->W * P->bytes > (1LL << 40)) return set_err(CODEC_EINVAL, "batch too large");
    return 0;
}

extern "C" {

int codec_pee_multi_embed_pass(const codec_pee_params* P, int32_t pass, const void* cover, void* stego,
                               const uint64_t* payload, const int32_t* lengths, codec_pee_meta* metas, uint64_t* lm,
                               void* workspace, size_t workspace_bytes, void* stream) {
    int rc = pee_multi_check(P, pass);
    if (rc) return rc;
    if (!cover || !stego || !payload || !lengths || !metas || !lm || !workspace)
        return set_err(CODEC_EINVAL, "codec_pee_multi_embed_pass: NULL pointer argument");
    const PeeWs L = pee_ws(P);
    if (workspace_bytes < L.total) return set_err(CODEC_EINVAL, "workspace too small");
    hipStream_t st = as_stream(stream);
    if (pass == 0 && knob("CODEC_PEE_MULTI_P0", 1) != 0) {
        // lattice 0 is scheme 1's: its embed paths (copy fused, 16-B items, look-back or
        // slice-serial) take the pass, and the records are made scheme 2's
        rc = codec_pee_embed_ts(P, cover, stego, payload, lengths, nullptr, metas, lm, workspace, workspace_bytes,
                                stream);
        if (rc) return rc;
        hipLaunchKernelGGL(k_pee_pass0_fix, dim3((unsigned)((P->B + 255) / 256)), dim3(256), 0, st, metas, P->B);
        LAUNCH_CHECK("k_pee_pass0_fix");
        return 0;
    }
    HIP_TRY(pee_ws_enter(workspace, P, L, st));
    uint32_t* cnt = reinterpret_cast<uint32_t*>(static_cast<char*>(workspace) + L.cnt);
    uint32_t* off = reinterpret_cast<uint32_t*>(static_cast<char*>(workspace) + L.off);
    if (cover != stego)   // the pass runs in place on the stego
        HIP_TRY(hipMemcpyAsync(stego, cover, (size_t)P->B * P->H * P->W * P->bytes, hipMemcpyDeviceToDevice, st));
    const PeeLat g = pee_lattice(pass, P->H, P->W);
    const int nc = g.hc * g.wc, ntiles = (nc + PEE_TILE - 1) / PEE_TILE;
    const int gx = std::max(1, std::min(ntiles, (int)knob("CODEC_PEE_LAT_WGS", 256)));
    dim3 grid(gx, P->B);
    {
        ProfScope prof(st, CODEC_K_PEE_LAT_COUNT);
#define PLC(TT) hipLaunchKernelGGL(k_pee_lat_count<TT>, grid, dim3(256), 0, st, static_cast<const TT*>(stego), P->H, P->W, \
                                   (int)pass, P->T, P->maxval, lengths, metas, (int)pass, P->B, cnt, L.ntiles_max)
        if (P->bytes == 2) PLC(uint16_t); else PLC(uint8_t);
#undef PLC
        LAUNCH_CHECK("k_pee_lat_count");
#define PLL(TT) hipLaunchKernelGGL(k_pee_lat_locate<TT>, dim3(P->B), dim3(256), 0, st, static_cast<const TT*>(stego), P->H, \
                                   P->W, (int)pass, P->T, P->maxval, lengths, metas, (int)pass, P->B, cnt, off, L.ntiles_max)
        if (P->bytes == 2) PLL(uint16_t); else PLL(uint8_t);
#undef PLL
        LAUNCH_CHECK("k_pee_lat_locate");
    }
    ProfScope prof(st, CODEC_K_PEE_LAT_EMBED);
#define PLE(TT) hipLaunchKernelGGL(k_pee_lat_embed<TT>, grid, dim3(256), 0, st, static_cast<TT*>(stego), P->H, P->W, \
                                   (int)pass, reinterpret_cast<const u64*>(payload), P->payload_words, off, L.ntiles_max, \
                                   metas, (int)pass, P->B, reinterpret_cast<u64*>(lm), P->lm_words)
    if (P->bytes == 2) PLE(uint16_t); else PLE(uint8_t);
#undef PLE
    LAUNCH_CHECK("k_pee_lat_embed");
    return 0;
}

int codec_pee_multi_extract_pass(const codec_pee_params* P, int32_t pass, const void* stego,
                                 const codec_pee_meta* metas, const uint64_t* lm, void* cover_out,
                                 uint64_t* payload_out, void* workspace, size_t workspace_bytes, void* stream) {
    int rc = pee_multi_check(P, pass);
    if (rc) return rc;
    if (!stego || !metas || !lm || !cover_out || !payload_out || !workspace)
        return set_err(CODEC_EINVAL, "codec_pee_multi_extract_pass: NULL pointer argument");
    const PeeWs L = pee_ws(P);
    if (workspace_bytes < L.total) return set_err(CODEC_EINVAL, "workspace too small");
    hipStream_t st = as_stream(stream);
    HIP_TRY(pee_ws_enter(workspace, P, L, st));
    uint32_t* cnt = reinterpret_cast<uint32_t*>(static_cast<char*>(workspace) + L.cnt);
    uint32_t* off = reinterpret_cast<uint32_t*>(static_cast<char*>(workspace) + L.off);
    if (cover_out != stego)   // the pass runs in place on cover_out
        HIP_TRY(hipMemcpyAsync(cover_out, stego, (size_t)P->B * P->H * P->W * P->bytes, hipMemcpyDeviceToDevice, st));
    const PeeLat g = pee_lattice(pass, P->H, P->W);
    const int nc = g.hc * g.wc, ntiles = (nc + PEE_TILE - 1) / PEE_TILE;
    const int gx = std::max(1, std::min(ntiles, (int)knob("CODEC_PEE_LAT_WGS", 256)));
    dim3 grid(gx, P->B);
    {
        ProfScope prof(st, CODEC_K_PEE_LAT_DCOUNT);
#define PLD(TT) hipLaunchKernelGGL(k_pee_lat_dcount<TT>, grid, dim3(256), 0, st, static_cast<const TT*>(cover_out), P->H, \
                                   P->W, (int)pass, metas, (int)pass, P->B, reinterpret_cast<const u64*>(lm), P->lm_words, \
                                   cnt, L.ntiles_max)
        if (P->bytes == 2) PLD(uint16_t); else PLD(uint8_t);
#undef PLD
        LAUNCH_CHECK("k_pee_lat_dcount");
        hipLaunchKernelGGL(k_pee_offsets, dim3(P->B), dim3(256), 0, st, metas + (size_t)pass * P->B, cnt, off, L.ntiles_max);
        LAUNCH_CHECK("k_pee_offsets");
    }
    ProfScope prof(st, CODEC_K_PEE_LAT_RECOVER);
#define PLR(TT) hipLaunchKernelGGL(k_pee_lat_recover<TT>, grid, dim3(256), 0, st, static_cast<TT*>(cover_out), P->H, P->W, \
                                   (int)pass, metas, (int)pass, P->B, reinterpret_cast<const u64*>(lm), P->lm_words, off, \
                                   L.ntiles_max, reinterpret_cast<u64*>(payload_out), P->payload_words)
    if (P->bytes == 2) PLR(uint16_t); else PLR(uint8_t);
#undef PLR
    LAUNCH_CHECK("k_pee_lat_recover");
    return 0;
}

}  // extern "C"

// the slice-serial scheme-2 launch (k_pee_lat_ss) where a chip-filling batch gives every CU a
// slice, as for scheme 1 (pee_use_slice_serial); slices up to CODEC_PEE_LAT_SS_MAXPX pixels (one
// CU streams its slice's copy).  CODEC_PEE_LAT_SS=0/1 forces the tile path / this one.
static bool pee_multi_use_ss(const codec_pee_params* P) {
    const long long k = knob("CODEC_PEE_LAT_SS", -1);
    if (k == 0) return false;
    if (k == 1) return true;
    const long long ncu = device_cu_count();
    if (P->B < ncu) return false;
    const long long rounds = (P->B + ncu - 1) / ncu;
    if ((double)P->B / (double)(rounds * ncu) < 0.85) return false;
    return (long long)P->H * P->W <= knob("CODEC_PEE_LAT_SS_MAXPX", 1LL << 20);
}
// 0: in place (no copy); 1: 16-B vector copy; 2: element copy (unaligned or ragged slices)
static int pee_lss_copy_mode(const codec_pee_params* P, const void* s, const void* d) {
    if (s == d) return 0;
    const size_t sb = (size_t)P->H * P->W * P->bytes;
    return (sb % 16 == 0 && (uintptr_t)s % 16 == 0 && (uintptr_t)d % 16 == 0) ? 1 : 2;
}

extern "C" {

int codec_pee_multi_embed(const codec_pee_params* P, const void* cover, void* stego, const uint64_t* payload,
                          const int32_t* lengths, codec_pee_meta* metas, uint64_t* lm, void* workspace,
                          size_t workspace_bytes, void* stream) {
    int rc = pee_multi_check(P, 0);
    if (rc) return rc;
    if (!cover || !stego || !payload || !lengths || !metas || !lm || !workspace)
        return set_err(CODEC_EINVAL, "codec_pee_multi_embed: NULL pointer argument");
    if (workspace_bytes < pee_ws(P).total) return set_err(CODEC_EINVAL, "workspace too small");
    const size_t lmp = (size_t)P->B * P->lm_words;   // one pass's map
    if (!pee_multi_use_ss(P)) {
        for (int p = 0; p < 4; ++p) {
            rc = codec_pee_multi_embed_pass(P, p, p == 0 ? cover : stego, stego, payload, lengths, metas, lm + p * lmp,
                                            workspace, workspace_bytes, stream);
            if (rc) return rc;
        }
        return 0;
    }
    hipStream_t st = as_stream(stream);
    // pass 0 through scheme 1's kernels (copy fused) unless CODEC_PEE_LAT_SS_P0=0, which runs the
    // copy and all four passes in the one slice-serial launch
    const bool p0s1 = knob("CODEC_PEE_LAT_SS_P0", 1) != 0 && knob("CODEC_PEE_MULTI_P0", 1) != 0;
    if (p0s1) {   // scheme 1's embed; the slice-serial launch below fixes pass 0's records
        rc = codec_pee_embed_ts(P, cover, stego, payload, lengths, nullptr, metas, lm, workspace, workspace_bytes,
                                stream);
        if (rc) return rc;
    }
    const int cm = p0s1 ? 0 : pee_lss_copy_mode(P, cover, stego);
    ProfScope prof(st, CODEC_K_PEE_LAT_SS_EMBED);
    char* sink = static_cast<char*>(workspace) + pee_ws(P).sink;
    const bool pl = P->payload_words <= LSS_PAY_MAXW && knob("CODEC_PEE_LAT_SS_PL", 1) != 0;
#define PLSE(TT, PLV) hipLaunchKernelGGL((k_pee_lat_ss<TT, false, PLV, true>), dim3((unsigned)P->B), dim3(LSS_THREADS), 0, st, \
                                    static_cast<const TT*>(cover), static_cast<TT*>(stego), P->H, P->W, P->T, P->maxval, cm, \
                                    p0s1 ? 1 : 0, const_cast<u64*>(reinterpret_cast<const u64*>(payload)), P->payload_words, \
                                    lengths, metas, P->B, reinterpret_cast<u64*>(lm), P->lm_words, sink)
    const bool pf = knob("CODEC_PEE_LAT_SS_PF", 1) != 0;
    if (P->bytes == 2) {
        if (!pf) hipLaunchKernelGGL((k_pee_lat_ss<uint16_t, false, true, false>), dim3((unsigned)P->B), dim3(LSS_THREADS), 0,
                                    st, static_cast<const uint16_t*>(cover), static_cast<uint16_t*>(stego), P->H, P->W, P->T,
                                    P->maxval, cm, p0s1 ? 1 : 0, const_cast<u64*>(reinterpret_cast<const u64*>(payload)),
                                    P->payload_words, lengths, metas, P->B, reinterpret_cast<u64*>(lm), P->lm_words, sink);
        else if (pl) PLSE(uint16_t, true);
        else PLSE(uint16_t, false);
    }
    else { if (pl) PLSE(uint8_t, true); else PLSE(uint8_t, false); }
#undef PLSE
    LAUNCH_CHECK("k_pee_lat_ss<embed>");
    return 0;
}

int codec_pee_multi_extract(const codec_pee_params* P, const void* stego, const codec_pee_meta* metas,
                            const uint64_t* lm, void* cover_out, uint64_t* payload_out, void* workspace,
                            size_t workspace_bytes, void* stream) {
    int rc = pee_multi_check(P, 0);
    if (rc) return rc;
    if (!stego || !metas || !lm || !cover_out || !payload_out || !workspace)
        return set_err(CODEC_EINVAL, "codec_pee_multi_extract: NULL pointer argument");
    if (workspace_bytes < pee_ws(P).total) return set_err(CODEC_EINVAL, "workspace too small");
    hipStream_t st = as_stream(stream);
    const size_t lmp = (size_t)P->B * P->lm_words;
    if (!pee_multi_use_ss(P)) {
        HIP_TRY(hipMemsetAsync(payload_out, 0, (size_t)P->B * P->payload_words * 8, st));
        for (int p = 3; p >= 0; --p) {
            rc = codec_pee_multi_extract_pass(P, p, p == 3 ? stego : cover_out, metas, lm + p * lmp, cover_out,
                                              payload_out, workspace, workspace_bytes, stream);
            if (rc) return rc;
        }
        return 0;
    }
    const int cm = pee_lss_copy_mode(P, stego, cover_out);
    ProfScope prof(st, CODEC_K_PEE_LAT_SS_EXTRACT);
    char* sink = static_cast<char*>(workspace) + pee_ws(P).sink;
    const bool pl = P->payload_words <= LSS_PAY_MAXW && knob("CODEC_PEE_LAT_SS_PL", 1) != 0;
#define PLSX(TT, PLV, PFV) hipLaunchKernelGGL((k_pee_lat_ss<TT, true, PLV, PFV>), dim3((unsigned)P->B), dim3(LSS_THREADS), 0, st, \
                                    static_cast<const TT*>(stego), static_cast<TT*>(cover_out), P->H, P->W, P->T, P->maxval, cm, \
                                    0, reinterpret_cast<u64*>(payload_out), P->payload_words, nullptr, \
                                    const_cast<codec_pee_meta*>(metas), P->B, const_cast<u64*>(reinterpret_cast<const u64*>(lm)), \
                                    P->lm_words, sink)
    const bool pf = knob("CODEC_PEE_LAT_SS_PF", 1) != 0;
    if (P->bytes == 2) {
        if (!pf) PLSX(uint16_t, true, false);
        else if (pl) PLSX(uint16_t, true, true);
        else PLSX(uint16_t, false, true);
    } else {
        if (pl) PLSX(uint8_t, true, true); else PLSX(uint8_t, false, true);
    }
#undef PLSX
    LAUNCH_CHECK("k_pee_lat_ss<extract>");
    return 0;
}

}  // extern "C"
