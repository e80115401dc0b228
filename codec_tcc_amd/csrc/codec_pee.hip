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

#define PEE_TILE 1024

struct PeeCand {
    int x, p;
    bool expand, right, safe;
};

__device__ __forceinline__ int med3(int a, int b, int c) {
    const int lo = min(a, b), hi = max(a, b);
    return c >= hi ? lo : (c <= lo ? hi : a + b - c);
}

__device__ __forceinline__ PeeCand pee_classify(int x, int a, int b, int c, int T, int maxval) {
    PeeCand r;
    r.x = x;
    r.p = med3(a, b, c);
    const int e = x - r.p;
    r.expand = (e >= -T) && (e < T);
    r.right = e >= T;
    if (r.expand) r.safe = (r.p + 2 * e >= 0) && (r.p + 2 * e + 1 <= maxval);
    else if (r.right) r.safe = x + T <= maxval;
    else r.safe = x - T >= 0;
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
template <typename T, bool NT>
__global__ __launch_bounds__(256) void k_pee_scan(const T* __restrict__ cover, T* __restrict__ stego, int H, int W,
                                                  int Tthr, int maxval, int tiles_per_wg,
                                                  uint32_t* __restrict__ tile_cnt_all, int ntiles_max) {
    typedef typename Vec8<T>::type V;
    __shared__ uint32_t sh[8];
    const int b = blockIdx.y;
    const size_t npx = (size_t)H * W;
    const T* src = cover + b * npx;
    T* dst = stego + b * npx;
    const int CR = W / 8, hc = H / 2;
    const long long items = (long long)hc * CR;
    const int ntiles = (int)((items + 255) / 256);
    uint32_t* tile_cnt = tile_cnt_all + (size_t)b * ntiles_max;
    const int t0 = blockIdx.x * tiles_per_wg;
    const int t1 = min(ntiles, t0 + tiles_per_wg);
    for (int t = t0; t < t1; ++t) {
        const long long it = (long long)t * 256 + threadIdx.x;
        uint32_t cnt = 0;
        if (it < items) {
            const int r = (int)(it / CR), c = (int)(it - (long long)r * CR);
            const size_t o0 = (size_t)(2 * r) * W + (size_t)c * 8, o1 = o0 + W;
            const V v0 = ldv<NT>(reinterpret_cast<const V*>(src + o0));
            const V v1 = ldv<NT>(reinterpret_cast<const V*>(src + o1));
            stv<NT>(reinterpret_cast<V*>(dst + o0), v0);
            stv<NT>(reinterpret_cast<V*>(dst + o1), v1);
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                int x, a, bb, cc;
                if constexpr (sizeof(T) == 2) {
                    x = (int)px16(v1, 2 * u + 1); a = (int)px16(v1, 2 * u); bb = (int)px16(v0, 2 * u + 1); cc = (int)px16(v0, 2 * u);
                } else {
                    x = (int)px8(v1, 2 * u + 1); a = (int)px8(v1, 2 * u); bb = (int)px8(v0, 2 * u + 1); cc = (int)px8(v0, 2 * u);
                }
                const PeeCand pc = pee_classify(x, a, bb, cc, Tthr, maxval);
                cnt += (pc.expand && pc.safe) ? 1u : 0u;
            }
        }
        const uint32_t tot = block_sum_u32<256>(cnt, sh);
        if (threadIdx.x == 0) tile_cnt[t] = tot;
    }
    // odd H: the last row belongs to no row pair; copy it
    if ((H & 1) && blockIdx.x == gridDim.x - 1) {
        const size_t o = (size_t)(H - 1) * W;
        for (int q = threadIdx.x; q < W; q += 256) dst[o + q] = src[o + q];
    }
}

// ---- scan for any shape: counts only (the copy is a separate stream copy)
template <typename T>
__global__ __launch_bounds__(256) void k_pee_count(const T* __restrict__ img, int H, int W, int Tthr, int maxval,
                                                   int tiles_per_wg, uint32_t* __restrict__ tile_cnt_all,
                                                   int ntiles_max) {
    __shared__ uint32_t sh[8];
    const int b = blockIdx.y;
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
__global__ __launch_bounds__(256) void k_pee_locate(const T* __restrict__ img, int H, int W, int Tthr, int maxval,
                                                    const int32_t* __restrict__ lengths,
                                                    const uint32_t* __restrict__ tile_cnt_all,
                                                    uint32_t* __restrict__ tile_off_all, int ntiles_max,
                                                    codec_pee_meta* __restrict__ meta_all) {
    __shared__ uint32_t sh[8];
    __shared__ int s_tile;
    __shared__ uint32_t s_base;
    __shared__ int s_end;
    const int b = blockIdx.x;
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
        } else if (running < L) {
            M->end = -1; M->tile_end = -1; M->status = 1;      // payload exceeds capacity
        } else {
            M->end = s_end; M->tile_end = tile; M->status = 0;
        }
        M->lm_count = 0;
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

// ====================================================================== host side
struct PeeWs {
    size_t cnt, off, total;
    int ntiles_max;
};

static PeeWs pee_ws(const codec_pee_params* P) {
    PeeWs L;
    const long long nc = (long long)(P->H / 2) * (P->W / 2);
    L.ntiles_max = (int)((nc + PEE_TILE - 1) / PEE_TILE);
    if (L.ntiles_max < 1) L.ntiles_max = 1;
    L.cnt = 0;
    L.off = align_up((size_t)P->B * L.ntiles_max * 4, 256);
    L.total = align_up(L.off + (size_t)P->B * L.ntiles_max * 4, 256);
    return L;
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

extern "C" {

size_t codec_pee_workspace_bytes(const codec_pee_params* P) {
    if (pee_check(P)) return 0;
    return pee_ws(P).total;
}

int codec_pee_embed(const codec_pee_params* P, const void* cover, void* stego, const uint64_t* payload,
                    const int32_t* lengths, codec_pee_meta* meta, uint64_t* lm, void* workspace,
                    size_t workspace_bytes, void* stream) {
    int rc = pee_check(P);
    if (rc) return rc;
    if (!cover || !stego || !payload || !lengths || !meta || !lm || !workspace)
        return set_err(CODEC_EINVAL, "codec_pee_embed: NULL pointer argument");
    const PeeWs L = pee_ws(P);
    if (workspace_bytes < L.total) return set_err(CODEC_EINVAL, "workspace too small");
    hipStream_t st = as_stream(stream);
    uint32_t* cnt = reinterpret_cast<uint32_t*>(static_cast<char*>(workspace) + L.cnt);
    uint32_t* off = reinterpret_cast<uint32_t*>(static_cast<char*>(workspace) + L.off);
    HIP_TRY(hipMemsetAsync(lm, 0, (size_t)P->B * P->lm_words * 8, st));
    const long long npx = (long long)P->H * P->W;
    const size_t va = P->bytes == 2 ? 16 : 8;
    const bool vec = (P->W % 8) == 0 && ((uintptr_t)cover % va) == 0 && ((uintptr_t)stego % va) == 0;
    const bool nt = knob("CODEC_NT", 1) != 0;
    {
        ProfScope prof(st, CODEC_K_PEE_SCAN);
        const int ntiles = L.ntiles_max;
        const long long target = knob("CODEC_PEE_SCAN_WGS", 32768);
        int per = (int)((ntiles * (long long)P->B + target - 1) / target);
        if (per < 1) per = 1;
        dim3 grid((ntiles + per - 1) / per, P->B);
        if (vec) {
#define PSCAN(TT, NTV) hipLaunchKernelGGL((k_pee_scan<TT, NTV>), grid, dim3(256), 0, st, static_cast<const TT*>(cover), static_cast<TT*>(stego), P->H, P->W, P->T, P->maxval, per, cnt, L.ntiles_max)
            if (P->bytes == 2) { if (nt) PSCAN(uint16_t, true); else PSCAN(uint16_t, false); }
            else { if (nt) PSCAN(uint8_t, true); else PSCAN(uint8_t, false); }
#undef PSCAN
            LAUNCH_CHECK("k_pee_scan");
        } else {
            HIP_TRY(hipMemcpyAsync(stego, cover, (size_t)npx * P->B * P->bytes, hipMemcpyDeviceToDevice, st));
            if (P->bytes == 2)
                hipLaunchKernelGGL(k_pee_count<uint16_t>, grid, dim3(256), 0, st, static_cast<const uint16_t*>(cover),
                                   P->H, P->W, P->T, P->maxval, per, cnt, L.ntiles_max);
            else
                hipLaunchKernelGGL(k_pee_count<uint8_t>, grid, dim3(256), 0, st, static_cast<const uint8_t*>(cover),
                                   P->H, P->W, P->T, P->maxval, per, cnt, L.ntiles_max);
            LAUNCH_CHECK("k_pee_count");
        }
    }
    {
        ProfScope prof(st, CODEC_K_PEE_LOCATE);
        if (P->bytes == 2)
            hipLaunchKernelGGL(k_pee_locate<uint16_t>, dim3(P->B), dim3(256), 0, st, static_cast<const uint16_t*>(cover),
                               P->H, P->W, P->T, P->maxval, lengths, cnt, off, L.ntiles_max, meta);
        else
            hipLaunchKernelGGL(k_pee_locate<uint8_t>, dim3(P->B), dim3(256), 0, st, static_cast<const uint8_t*>(cover),
                               P->H, P->W, P->T, P->maxval, lengths, cnt, off, L.ntiles_max, meta);
        LAUNCH_CHECK("k_pee_locate");
    }
    {
        ProfScope prof(st, CODEC_K_PEE_EMBED);
        const int g = (int)knob("CODEC_PEE_EMBED_WGS", 64);
        dim3 grid(g < L.ntiles_max ? g : L.ntiles_max, P->B);
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

int codec_pee_extract(const codec_pee_params* P, const void* stego, const codec_pee_meta* meta, const uint64_t* lm,
                      void* cover_out, uint64_t* payload_out, void* workspace, size_t workspace_bytes, void* stream) {
    int rc = pee_check(P);
    if (rc) return rc;
    if (!stego || !meta || !lm || !cover_out || !payload_out || !workspace)
        return set_err(CODEC_EINVAL, "codec_pee_extract: NULL pointer argument");
    const PeeWs L = pee_ws(P);
    if (workspace_bytes < L.total) return set_err(CODEC_EINVAL, "workspace too small");
    hipStream_t st = as_stream(stream);
    uint32_t* cnt = reinterpret_cast<uint32_t*>(static_cast<char*>(workspace) + L.cnt);
    uint32_t* off = reinterpret_cast<uint32_t*>(static_cast<char*>(workspace) + L.off);
    const long long nbytes = (long long)P->H * P->W * P->B * P->bytes;
    const bool nt = knob("CODEC_NT", 1) != 0;
    const size_t va = P->bytes == 2 ? 16 : 8;
    const bool vec = (P->W % 8) == 0 && ((uintptr_t)stego % va) == 0 && ((uintptr_t)cover_out % va) == 0;
    HIP_TRY(hipMemsetAsync(payload_out, 0, (size_t)P->B * P->payload_words * 8, st));
    const long long items = (long long)(P->H / 2) * (P->W / 8);
    const bool fused = vec && knob("CODEC_PEE_FUSED", 1) != 0 && (P->W % 8) == 0 && items > 0 && (items % 256) == 0 &&
                       items * P->B < 0xFFFFFFFFLL;
    if (fused) {
        const int g = (int)knob("CODEC_PEE_EMBED_WGS", 64);
        dim3 grid(g < L.ntiles_max ? g : L.ntiles_max, P->B);
        {
            ProfScope prof(st, CODEC_K_PEE_DCOUNT);
#define PDC2(TT) hipLaunchKernelGGL((k_pee_dcount<TT, true>), grid, dim3(256), 0, st, static_cast<const TT*>(stego), P->H, P->W, \
                               meta, reinterpret_cast<const u64*>(lm), P->lm_words, cnt, L.ntiles_max)
            if (P->bytes == 2) PDC2(uint16_t); else PDC2(uint8_t);
#undef PDC2
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
