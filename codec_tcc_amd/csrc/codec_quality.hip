// codec_quality.hip -- stego-quality moments for the metrics of the reference's
// src/mse.py (AnalisadorMSE: calcular_mse :74-117, calcular_psnr :119-133,
// calcular_ssim_simples :135-177, difference statistics :201-207).
//
// One read-only streaming pass over a (cover, stego) batch yields, per slice, EXACT integer
// moments: sum a, sum b, sum a^2, sum b^2, sum ab, sum |a-b|, max |a-b|, #(a != b), max a,
// max b.  Every metric of mse.py is a closed form of these (the host evaluates it in exact
// rational arithmetic, codec_tcc_amd/quality.py), so no float sum order has to be
// emulated and the only rounding is the final one.
//
// Launch: grid (regions per slice, B), 256 threads; a workgroup streams one contiguous
// region of one slice, 4 x 16-B vectors of each image per thread per iteration, keeps
// the moments in registers (32-bit sums, float64 FMAs for the products: QmAcc), reduces them across the wave
// with shuffles and adds them to the slice's record with 64-bit atomics (one set per
// wave), so HBM traffic is the two reads and nothing else.
#include "codec_common.h"

#define QM_WORDS 10

// per-thread accumulators, exact by bounds (the host caps a thread at QM_MAX_PX pixels):
// the linear sums in 32 bits (<= 2^16 px x 65535), the products in float64 FMAs (each product
// <= 2^32 is exact, every partial sum <= 2^16 x 2^32 < 2^53 is an exact integer) -- fewer,
// full-rate instructions instead of v_mad_u64_u32 and 64-bit adds (256 x 2048^2: 0.723 ->
// 0.719 ms; the pass is memory-bound either way, profiles/r04/quality_acc_ab.txt)
#define QM_MAX_PX 65536
struct QmAcc {
    uint32_t s[4];   // sum a, sum b, sum |a - b|, #(a != b)
    double q[3];     // sum a^2, sum b^2, sum ab
    uint32_t mx[3];  // max |a - b|, max a, max b
};

template <typename T>
__device__ __forceinline__ void qm_px(uint32_t a, uint32_t b, QmAcc& m) {
    m.s[0] += a;
    m.s[1] += b;
    const double fa = (double)a, fb = (double)b;
    m.q[0] = fma(fa, fa, m.q[0]);
    m.q[1] = fma(fb, fb, m.q[1]);
    m.q[2] = fma(fa, fb, m.q[2]);
    const uint32_t d = a > b ? a - b : b - a;
    m.s[2] += d;
    m.mx[0] = max(m.mx[0], d);
    m.s[3] += min(d, 1u);
    m.mx[1] = max(m.mx[1], a);
    m.mx[2] = max(m.mx[2], b);
}

template <typename T>
__device__ __forceinline__ void qm_vec(const typename Vec8<T>::type& va, const typename Vec8<T>::type& vb, QmAcc& m) {
    if constexpr (sizeof(T) == 2) {
        const uint32_t wa[4] = {va.x, va.y, va.z, va.w}, wb[4] = {vb.x, vb.y, vb.z, vb.w};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            qm_px<T>(wa[k] & 0xFFFFu, wb[k] & 0xFFFFu, m);
            qm_px<T>(wa[k] >> 16, wb[k] >> 16, m);
        }
    } else {
        const uint32_t wa[2] = {va.x, va.y}, wb[2] = {vb.x, vb.y};
#pragma unroll
        for (int k = 0; k < 2; ++k)
#pragma unroll
            for (int e = 0; e < 4; ++e) qm_px<T>((wa[k] >> (8 * e)) & 0xFFu, (wb[k] >> (8 * e)) & 0xFFu, m);
    }
}

template <typename T, bool VEC>
__global__ __launch_bounds__(256) void k_quality(const T* __restrict__ a_all, const T* __restrict__ b_all,
                                                 long long npx, long long per_wg, u64* __restrict__ out) {
    typedef typename Vec8<T>::type V;
    const int b = blockIdx.y;
    const T* A = a_all + (size_t)b * npx;
    const T* Bm = b_all + (size_t)b * npx;
    const long long p0 = (long long)blockIdx.x * per_wg;
    const long long p1 = min(npx, p0 + per_wg);
    QmAcc acc = {{0u, 0u, 0u, 0u}, {0.0, 0.0, 0.0}, {0u, 0u, 0u}};
    if (p0 < p1) {
        if constexpr (VEC) {
            // host guarantees: npx % 8 == 0, per_wg % 8 == 0, 16-B (8-B) aligned slices
            const V* va = reinterpret_cast<const V*>(A + p0);
            const V* vb = reinterpret_cast<const V*>(Bm + p0);
            const long long nv = (p1 - p0) / 8;
            long long i = threadIdx.x;
            for (; i + 3 * 256 < nv; i += 4 * 256) {
                V xa[4], xb[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) { xa[u] = ldv<true>(va + i + u * 256); xb[u] = ldv<true>(vb + i + u * 256); }
#pragma unroll
                for (int u = 0; u < 4; ++u) qm_vec<T>(xa[u], xb[u], acc);
            }
            for (; i < nv; i += 256) qm_vec<T>(ldv<true>(va + i), ldv<true>(vb + i), acc);
        } else {
            for (long long q = p0 + threadIdx.x; q < p1; q += 256) qm_px<T>(A[q], Bm[q], acc);
        }
    }
    // widen: the wave reduction sums 64 threads' values
    u64 m[8] = {acc.s[0], acc.s[1], (u64)acc.q[0], (u64)acc.q[1], (u64)acc.q[2], acc.s[2], 0ull, acc.s[3]};
    uint32_t mx[3] = {acc.mx[0], acc.mx[1], acc.mx[2]};
    // wave reduction, then one atomic set per wave
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
#pragma unroll
        for (int k = 0; k < 8; ++k) m[k] += __shfl_xor(m[k], o, 64);
#pragma unroll
        for (int k = 0; k < 3; ++k) mx[k] = max(mx[k], __shfl_xor(mx[k], o, 64));
    }
    if ((threadIdx.x & 63) == 0) {
        u64* o = out + (size_t)b * QM_WORDS;
        atomicAdd(&o[0], m[0]);
        atomicAdd(&o[1], m[1]);
        atomicAdd(&o[2], m[2]);
        atomicAdd(&o[3], m[3]);
        atomicAdd(&o[4], m[4]);
        atomicAdd(&o[5], m[5]);
        atomicMax(&o[6], (u64)mx[0]);
        atomicAdd(&o[7], m[7]);
        atomicMax(&o[8], (u64)mx[1]);
        atomicMax(&o[9], (u64)mx[2]);
    }
}

extern "C" {

int codec_quality_moments(int32_t B, int32_t H, int32_t W, int32_t bytes, const void* a, const void* b,
                          uint64_t* out, void* stream) {
    if (B < 1 || H < 1 || W < 1) return set_err(CODEC_EINVAL, "codec_quality_moments: bad shape B=%d H=%d W=%d", B, H, W);
    if (bytes != 1 && bytes != 2) return set_err(CODEC_EINVAL, "codec_quality_moments: bytes must be 1 or 2");
    if (!a || !b || !out) return set_err(CODEC_EINVAL, "codec_quality_moments: NULL pointer argument");
    const long long npx = (long long)H * W;
    if (npx > (1LL << 31)) return set_err(CODEC_EINVAL, "codec_quality_moments: slice too large");
    hipStream_t st = as_stream(stream);
    HIP_TRY(hipMemsetAsync(out, 0, (size_t)B * QM_WORDS * 8, st));
    const size_t va = bytes == 2 ? 16 : 8;
    const bool vec = (npx % 8) == 0 && ((uintptr_t)a % va) == 0 && ((uintptr_t)b % va) == 0;
    // ~256 KiB of each image per workgroup region (tools: one atomic set per wave)
    long long per = knob("CODEC_QUALITY_PX_PER_WG", 131072);
    per = (per + 7) / 8 * 8;
    if (per < 2048) per = 2048;
    if (per > 256LL * QM_MAX_PX) per = 256LL * QM_MAX_PX;   // the accumulators' exactness bound
    const long long wps = (npx + per - 1) / per;
    dim3 grid((unsigned)wps, B);
    ProfScope prof(st, CODEC_K_QUALITY);
#define QL(TT, VV) hipLaunchKernelGGL((k_quality<TT, VV>), grid, dim3(256), 0, st, static_cast<const TT*>(a), \
                                      static_cast<const TT*>(b), npx, per, reinterpret_cast<u64*>(out))
    if (bytes == 2) { if (vec) QL(uint16_t, true); else QL(uint16_t, false); }
    else { if (vec) QL(uint8_t, true); else QL(uint8_t, false); }
#undef QL
    LAUNCH_CHECK("k_quality");
    return 0;
}

}  // extern "C"
