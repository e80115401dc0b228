// Ceiling of the in-place MED-PEE access pattern (k_pee_embed_ss<..., INPLACE>), without its
// classification / scan work: 256 slices of 2048^2 uint16, one 1024-thread workgroup per
// slice (one per CU), each streams the items of its slice's first NCHUNK chunks (item = 8
// columns of a row pair: two 16-B loads) and stores the odd row back IN PLACE.  Variants:
//   ring D      : D chunks of loads in flight per thread (a register ring, refilled after use)
//   +barrier    : an LDS-only barrier per chunk (the embed's one scan barrier)
//   +valu N     : N dependent-free integer ops per candidate per chunk (the embed's VALU)
//   ntile       : the same bytes as 4 workgroups per CU (256 threads, a quarter slice each,
//                 contiguous quarters) -- more independent streams per CU
// Prints ms and GB/s of algorithmic bytes (2 rows read + 1 row written per item).
//   hipcc --offload-arch=gfx950 -O3 tools/ubench_inplace.hip -o tools/bin/ubench_inplace
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

typedef unsigned int v4u __attribute__((ext_vector_type(4)));
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

constexpr int H = 2048, W = 2048, CR = W / 8;
constexpr int NCHUNK = 24;   // ~ the chunks up to `end` (30 at 1 KB, T = 2); divisible by ring depths 1-4
constexpr int NT = 1024;

__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

// EARLY: the slot's refill is issued right after its data is taken (into temporaries), before
// the barrier and the compute -- D loads stay in flight through the barrier
template <int D, bool BAR, int VALU, bool EARLY = false, bool PS = false>
__global__ __launch_bounds__(NT) void inplace_stream(unsigned short* img, int nchunk, unsigned* sink) {
    __shared__ unsigned pad[21 * 1024];   // one workgroup per CU, as the embed's pad
    const size_t npx = (size_t)H * W;
    unsigned short* s = img + blockIdx.x * npx;
    if (threadIdx.x == 0) pad[0] = 0;
    v4u r0[D], r1[D];
    unsigned ro[D];
    unsigned acc = 0;
#pragma unroll
    for (int d = 0; d < D; ++d) {
        const unsigned it = d * NT + threadIdx.x;
        const unsigned r = it / CR, c = it - r * CR;
        ro[d] = 2u * r * W + 8u * c;
        r0[d] = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(s + ro[d]));
        r1[d] = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(s + ro[d] + W));
    }
    const int nfull = nchunk / D * D;
    for (int k0 = 0; k0 < nfull; k0 += D) {
#pragma unroll
        for (int d = 0; d < D; ++d) {
            const int k = k0 + d;
            v4u a = r0[d], b = r1[d];
            asm volatile("" ::"v"(a.x), "v"(b.x));
            const unsigned so = ro[d];
            if (EARLY) {
                const unsigned it = (unsigned)(k + D) * NT + threadIdx.x;
                const unsigned kk = k + D < nchunk ? it : threadIdx.x;
                const unsigned r = kk / CR, c = kk - r * CR;
                ro[d] = 2u * r * W + 8u * c;
                r0[d] = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(s + ro[d]));
                r1[d] = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(s + ro[d] + W));
            }
            unsigned x = a.x ^ b.y;
#pragma unroll
            for (int q = 0; q < VALU; ++q) x = (x * 0x9E37u + (b.z >> (q & 7))) ^ a.w;
            acc += x;
            b.x ^= (acc & 0u);
            if (BAR) lds_barrier();
            if (PS) *reinterpret_cast<v4u*>(s + so + W) = b;   // plain (cache-allocating) store: round 5's default
            else __builtin_nontemporal_store(b, reinterpret_cast<v4u*>(s + so + W));
            if (!EARLY) {
                const unsigned it = (unsigned)(k + D) * NT + threadIdx.x;
                const unsigned kk = k + D < nchunk ? it : threadIdx.x;
                const unsigned r = kk / CR, c = kk - r * CR;
                ro[d] = 2u * r * W + 8u * c;
                r0[d] = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(s + ro[d]));
                r1[d] = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(s + ro[d] + W));
            }
        }
    }
    if (acc == 0xFFFFFFFFu) sink[0] = acc + pad[threadIdx.x & 7];
}

// round 5: the embed's per-chunk scan barrier replaced by a chained
// wave scan -- per chunk every wave publishes its count in LDS (tagged with the chunk), then
// waits only for the LOWER waves' counts of this chunk and every wave's count of the previous
// chunk (the running total), read in one LDS load per lane and summed with DPP row scans.
// PAIR: the barrier kept, but one per two chunks (two chunks classified between scans).
__device__ __forceinline__ unsigned chain_tag(int k) { return ((unsigned)(k & 0x7FFF) | 0x8000u) << 16; }
template <int D, int VALU, bool EARLY, bool CHAIN, bool PAIR>
__global__ __launch_bounds__(NT) void inplace_chain(unsigned short* img, int nchunk, unsigned* sink) {
    __shared__ unsigned pad[21 * 1024 - 64];
    __shared__ unsigned agg[4][16];
    const size_t npx = (size_t)H * W;
    unsigned short* s = img + blockIdx.x * npx;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    if (threadIdx.x == 0) pad[0] = 0;
    if (threadIdx.x < 64) agg[threadIdx.x >> 4][threadIdx.x & 15] = 0u;
    __syncthreads();
    v4u r0[D], r1[D];
    unsigned ro[D];
    unsigned acc = 0, running = 0;
#pragma unroll
    for (int d = 0; d < D; ++d) {
        const unsigned it = d * NT + threadIdx.x;
        const unsigned r = it / CR, c = it - r * CR;
        ro[d] = 2u * r * W + 8u * c;
        r0[d] = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(s + ro[d]));
        r1[d] = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(s + ro[d] + W));
    }
    const int nfull = nchunk / D * D;
    for (int k0 = 0; k0 < nfull; k0 += D) {
#pragma unroll
        for (int d = 0; d < D; ++d) {
            const int k = k0 + d;
            v4u a = r0[d], b = r1[d];
            asm volatile("" ::"v"(a.x), "v"(b.x));
            const unsigned so = ro[d];
            if (EARLY) {
                const unsigned it = (unsigned)(k + D) * NT + threadIdx.x;
                const unsigned kk = k + D < nchunk ? it : threadIdx.x;
                const unsigned r = kk / CR, c = kk - r * CR;
                ro[d] = 2u * r * W + 8u * c;
                r0[d] = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(s + ro[d]));
                r1[d] = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(s + ro[d] + W));
            }
            unsigned x = a.x ^ b.y;
#pragma unroll
            for (int q = 0; q < VALU; ++q) x = (x * 0x9E37u + (b.z >> (q & 7))) ^ a.w;
            const unsigned n = x & 3u;
            const unsigned wt = (unsigned)__popcll(__ballot(n & 1u)) + 2u * (unsigned)__popcll(__ballot(n & 2u));
            if (CHAIN) {
                if (lane == 0)
                    __hip_atomic_store(&agg[k & 3][wv], chain_tag(k) | wt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                const bool prev = lane < 16 && k > 0, cur = lane >= 16 && lane < 16 + wv;
                unsigned* slot = prev ? &agg[(k - 1) & 3][lane] : &agg[k & 3][(lane - 16) & 15];
                const unsigned want = prev ? chain_tag(k - 1) : chain_tag(k);
                unsigned v = 0;
                for (;;) {
                    v = (prev || cur) ? __hip_atomic_load(slot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) : want;
                    if (!__ballot((v & 0xFFFF0000u) != want)) break;
                    __builtin_amdgcn_s_sleep(1);
                }
                int y = (prev || cur) ? (int)(v & 0xFFFFu) : 0;
                y += __builtin_amdgcn_update_dpp(0, y, 0x111, 0xF, 0xF, true);
                y += __builtin_amdgcn_update_dpp(0, y, 0x112, 0xF, 0xF, true);
                y += __builtin_amdgcn_update_dpp(0, y, 0x114, 0xF, 0xF, true);
                y += __builtin_amdgcn_update_dpp(0, y, 0x118, 0xF, 0xF, true);
                running += (unsigned)__builtin_amdgcn_readlane(y, 15);
                const unsigned pre = wv ? (unsigned)__builtin_amdgcn_readlane(y, 15 + wv) : 0u;
                acc += running + pre;
            } else if (!PAIR || (k & 1)) {
                lds_barrier();
                acc += wt;
            }
            acc += x;
            b.x ^= (acc & 0u);
            __builtin_nontemporal_store(b, reinterpret_cast<v4u*>(s + so + W));
            if (!EARLY) {
                const unsigned it = (unsigned)(k + D) * NT + threadIdx.x;
                const unsigned kk = k + D < nchunk ? it : threadIdx.x;
                const unsigned r = kk / CR, c = kk - r * CR;
                ro[d] = 2u * r * W + 8u * c;
                r0[d] = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(s + ro[d]));
                r1[d] = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(s + ro[d] + W));
            }
        }
    }
    if (acc == 0xFFFFFFFFu) sink[0] = acc + pad[threadIdx.x & 7];
}

// 4 workgroups of 256 threads per slice, each a contiguous quarter of the slice's chunks
template <int D>
__global__ __launch_bounds__(256) void inplace_quarters(unsigned short* img, int nchunk, unsigned* sink) {
    const size_t npx = (size_t)H * W;
    const int b = blockIdx.x >> 2, qt = blockIdx.x & 3;
    unsigned short* s = img + b * npx;
    const unsigned items = (unsigned)nchunk * NT, per = items / 4, it0 = qt * per;
    unsigned acc = 0;
    v4u r0[D], r1[D];
    unsigned ro[D];
#pragma unroll
    for (int d = 0; d < D; ++d) {
        const unsigned it = it0 + d * 256 + threadIdx.x;
        const unsigned r = it / CR, c = it - r * CR;
        ro[d] = 2u * r * W + 8u * c;
        r0[d] = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(s + ro[d]));
        r1[d] = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(s + ro[d] + W));
    }
    const unsigned steps = per / 256;
    for (unsigned k0 = 0; k0 + D <= steps; k0 += D) {
#pragma unroll
        for (int d = 0; d < D; ++d) {
            v4u a = r0[d], b2 = r1[d];
            acc += a.x ^ b2.y;
            __builtin_nontemporal_store(b2, reinterpret_cast<v4u*>(s + ro[d] + W));
            const unsigned kn = k0 + d + D < steps ? k0 + d + D : 0;
            const unsigned it = it0 + kn * 256 + threadIdx.x;
            const unsigned r = it / CR, c = it - r * CR;
            ro[d] = 2u * r * W + 8u * c;
            r0[d] = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(s + ro[d]));
            r1[d] = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(s + ro[d] + W));
        }
    }
    if (acc == 0xFFFFFFFFu) sink[0] = acc;
}

int main() {
    const int B = 256;
    const size_t bytes = (size_t)B * H * W * 2;
    unsigned short* img;
    unsigned* sink;
    CK(hipMalloc(&img, bytes));
    CK(hipMalloc(&sink, 256));
    CK(hipMemset(img, 1, bytes));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const double algo = (double)B * NCHUNK * NT * 48.0;   // 32 B read + 16 B written per item
    for (int pass = 0; pass < 2; ++pass) {
        for (int variant = 0; variant < 30; ++variant) {
            const char* name = "";
            float sum = 0.f, best = 1e9f;
            const int reps = 20;
            for (int r = 0; r < reps + 3; ++r) {
                CK(hipEventRecord(e0, 0));
                switch (variant) {
                case 0: name = "ring 1"; inplace_stream<1, false, 0><<<B, NT>>>(img, NCHUNK, sink); break;
                case 1: name = "ring 2"; inplace_stream<2, false, 0><<<B, NT>>>(img, NCHUNK, sink); break;
                case 2: name = "ring 3"; inplace_stream<3, false, 0><<<B, NT>>>(img, NCHUNK, sink); break;
                case 3: name = "ring 4"; inplace_stream<4, false, 0><<<B, NT>>>(img, NCHUNK, sink); break;
                case 4: name = "ring 2 +barrier"; inplace_stream<2, true, 0><<<B, NT>>>(img, NCHUNK, sink); break;
                case 5: name = "ring 3 +barrier"; inplace_stream<3, true, 0><<<B, NT>>>(img, NCHUNK, sink); break;
                case 6: name = "ring 2 +barrier +valu 16"; inplace_stream<2, true, 16><<<B, NT>>>(img, NCHUNK, sink); break;
                case 7: name = "ring 2 +barrier +valu 48"; inplace_stream<2, true, 48><<<B, NT>>>(img, NCHUNK, sink); break;
                case 8: name = "ring 3 +barrier +valu 48"; inplace_stream<3, true, 48><<<B, NT>>>(img, NCHUNK, sink); break;
                case 9: name = "ring 4 +barrier +valu 48"; inplace_stream<4, true, 48><<<B, NT>>>(img, NCHUNK, sink); break;
                case 10: name = "ring 2 +valu 48"; inplace_stream<2, false, 48><<<B, NT>>>(img, NCHUNK, sink); break;
                case 11: name = "quarters ring 2"; inplace_quarters<2><<<4 * B, 256>>>(img, NCHUNK, sink); break;
                case 12: name = "quarters ring 4"; inplace_quarters<4><<<4 * B, 256>>>(img, NCHUNK, sink); break;
                case 13: name = "ring 2 +barrier +valu 96"; inplace_stream<2, true, 96><<<B, NT>>>(img, NCHUNK, sink); break;
                case 14: name = "early ring 2 +barrier +valu 48"; inplace_stream<2, true, 48, true><<<B, NT>>>(img, NCHUNK, sink); break;
                case 15: name = "early ring 3 +barrier +valu 48"; inplace_stream<3, true, 48, true><<<B, NT>>>(img, NCHUNK, sink); break;
                case 16: name = "early ring 2 +barrier"; inplace_stream<2, true, 0, true><<<B, NT>>>(img, NCHUNK, sink); break;
                case 17: name = "early ring 1 +barrier +valu 48"; inplace_stream<1, true, 48, true><<<B, NT>>>(img, NCHUNK, sink); break;
                case 18: name = "early ring 4 +barrier +valu 48"; inplace_stream<4, true, 48, true><<<B, NT>>>(img, NCHUNK, sink); break;
                case 19: name = "early ring 1 +chain +valu 48"; inplace_chain<1, 48, true, true, false><<<B, NT>>>(img, NCHUNK, sink); break;
                case 20: name = "early ring 2 +chain +valu 48"; inplace_chain<2, 48, true, true, false><<<B, NT>>>(img, NCHUNK, sink); break;
                case 21: name = "ring 2 +chain +valu 48"; inplace_chain<2, 48, false, true, false><<<B, NT>>>(img, NCHUNK, sink); break;
                case 22: name = "early ring 1 +chain"; inplace_chain<1, 0, true, true, false><<<B, NT>>>(img, NCHUNK, sink); break;
                case 23: name = "early ring 2 +pair +valu 48"; inplace_chain<2, 48, true, false, true><<<B, NT>>>(img, NCHUNK, sink); break;
                case 24: name = "early ring 1 +bar2 +valu 48"; inplace_chain<1, 48, true, false, false><<<B, NT>>>(img, NCHUNK, sink); break;
                case 25: name = "early ring 2 +chain"; inplace_chain<2, 0, true, true, false><<<B, NT>>>(img, NCHUNK, sink); break;
                case 26: name = "early ring 4 +pair +valu 48"; inplace_chain<4, 48, true, false, true><<<B, NT>>>(img, NCHUNK, sink); break;
                case 27: name = "early ring 1 +bar +valu 48 +ps"; inplace_stream<1, true, 48, true, true><<<B, NT>>>(img, NCHUNK, sink); break;
                case 28: name = "early ring 2 +bar +valu 48 +ps"; inplace_stream<2, true, 48, true, true><<<B, NT>>>(img, NCHUNK, sink); break;
                case 29: name = "ring 2 +ps (no barrier, no valu)"; inplace_stream<2, false, 0, false, true><<<B, NT>>>(img, NCHUNK, sink); break;
                }
                CK(hipGetLastError());
                CK(hipEventRecord(e1, 0));
                CK(hipEventSynchronize(e1));
                float ms;
                CK(hipEventElapsedTime(&ms, e0, e1));
                if (r >= 3) { sum += ms; if (ms < best) best = ms; }
            }
            const float avg = sum / reps;
            printf("pass %d %-28s avg %.4f ms  best %.4f ms  %7.0f GB/s (algorithmic, avg)\n", pass, name, avg, best,
                   algo / avg / 1e6);
        }
    }
    return 0;
}
