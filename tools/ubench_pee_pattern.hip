// Access-pattern costs of k_pee_embed1's out-of-place sweep, separated from its scan work:
//   slot   : one 256-thread workgroup per 32 KiB chunk (4 row pairs of a 2048-wide slice),
//            slot v -> slice (v % 8) + 8 k, chunk-major or slice-major, plain copy
//   ticket : slot + the per-slice ticket atomic and done-flag load; the stores wait for the
//            ticket and use it as the chunk index (what k_pee_embed1 does on copy chunks)
//   region : 1024-thread workgroups streaming one contiguous region each (the copy ceiling)
//   hipcc --offload-arch=gfx950 -O3 tools/ubench_pee_pattern.hip -o tools/bin/ubench_pee_pattern
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

typedef unsigned int v4u __attribute__((ext_vector_type(4)));
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

constexpr int H = 2048, W = 2048, CR = W / 8;          // 16-B vectors per row
constexpr int CHUNK = 1024;                             // items (vector pairs) per chunk
constexpr int NCH = (H / 2) * CR / CHUNK;               // chunks per slice

__device__ __forceinline__ void slot_of(unsigned v, int B, int cmajor, int* b, int* j) {
    const int B8 = (B + 7) / 8, x = v & 7;
    const unsigned k = v >> 3;
    int bi;
    if (cmajor == 1) { *j = k / B8; bi = k - *j * B8; }
    else if (cmajor > 1) {   // skewed chunk-major: slice lane bi runs (bi % cmajor) chunks behind
        const int d = k / B8;
        bi = k - d * B8;
        *j = d - bi % cmajor;
    } else { bi = k / NCH; *j = k - bi * NCH; }
    *b = x + 8 * bi;
}

template <int CPW, bool TICKET>
__global__ __launch_bounds__(256) void slot_copy(const unsigned short* __restrict__ src, unsigned short* __restrict__ dst,
                                                 int B, int cmajor, unsigned* ctl) {
    __shared__ unsigned s_c;
    const size_t npx = (size_t)H * W;
    for (int q = 0; q < CPW; ++q) {
        const unsigned v = blockIdx.x * CPW + q;
        int b, j;
        slot_of(v, B, cmajor, &b, &j);
        if (j < 0 || j >= NCH) continue;
        const unsigned short* s = src + b * npx;
        unsigned short* d = dst + b * npx;
        v4u a0[4], a1[4];
        size_t o[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const unsigned it = (unsigned)j * CHUNK + u * 256 + threadIdx.x;
            const unsigned r = it / CR, c = it - r * CR;
            o[u] = (size_t)(2 * r) * W + (size_t)c * 8;
            a0[u] = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(s + o[u]));
            a1[u] = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(s + o[u] + W));
        }
        if (TICKET) {
            if (threadIdx.x == 0) {
                unsigned* t = ctl + 32 * b;
                const unsigned dn = __hip_atomic_load(t + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                s_c = atomicAdd(t, 1u) + (dn & 0u);
            }
            __syncthreads();
            const unsigned c = s_c;
            if (c != (unsigned)j) {
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const unsigned it = c * CHUNK + u * 256 + threadIdx.x;
                    const unsigned r = it / CR, cc = it - r * CR;
                    o[u] = (size_t)(2 * r) * W + (size_t)cc * 8;
                    a0[u] = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(s + o[u]));
                    a1[u] = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(s + o[u] + W));
                }
            }
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            __builtin_nontemporal_store(a0[u], reinterpret_cast<v4u*>(d + o[u]));
            __builtin_nontemporal_store(a1[u], reinterpret_cast<v4u*>(d + o[u] + W));
        }
        if (TICKET) __syncthreads();
    }
}

// each workgroup: `per` vectors, in steps of blockDim * 4
__global__ __launch_bounds__(1024) void region_copy(const v4u* __restrict__ src, v4u* __restrict__ dst, size_t per) {
    const size_t step = (size_t)blockDim.x * 4;
    const size_t r0 = (size_t)blockIdx.x * per;
    for (size_t i = 0; i < per; i += step) {
        const size_t base = r0 + i + threadIdx.x;
        v4u v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) v[u] = __builtin_nontemporal_load(src + base + (size_t)u * blockDim.x);
#pragma unroll
        for (int u = 0; u < 4; ++u) __builtin_nontemporal_store(v[u], dst + base + (size_t)u * blockDim.x);
    }
}

int main() {
    const int B = 256;
    const size_t bytes = (size_t)B * H * W * 2;
    unsigned short *src, *dst;
    unsigned* ctl;
    CK(hipMalloc(&src, bytes));
    CK(hipMalloc(&dst, bytes));
    CK(hipMalloc(&ctl, (size_t)B * 32 * 4 + 128));
    CK(hipMemset(src, 1, bytes));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const unsigned total = (unsigned)B * NCH;
    for (int pass = 0; pass < 2; ++pass) {
        for (int variant = 0; variant < 12; ++variant) {
            const char* name = "";
            float best = 1e9f, sum = 0.f;
            const int reps = 10;
            for (int r = 0; r < reps + 2; ++r) {
                CK(hipMemsetAsync(ctl, 0, (size_t)B * 32 * 4, 0));
                CK(hipEventRecord(e0, 0));
                switch (variant) {
                case 0: name = "slot cmajor 1 chunk/WG"; slot_copy<1, false><<<total, 256>>>(src, dst, B, 1, ctl); break;
                case 1: name = "slot smajor 1 chunk/WG"; slot_copy<1, false><<<total, 256>>>(src, dst, B, 0, ctl); break;
                case 2: name = "slot cmajor 2 chunk/WG"; slot_copy<2, false><<<total / 2, 256>>>(src, dst, B, 1, ctl); break;
                case 3: name = "slot cmajor 4 chunk/WG"; slot_copy<4, false><<<total / 4, 256>>>(src, dst, B, 1, ctl); break;
                case 4: name = "ticket cmajor 1 chunk/WG"; slot_copy<1, true><<<total, 256>>>(src, dst, B, 1, ctl); break;
                case 5: name = "ticket smajor 1 chunk/WG"; slot_copy<1, true><<<total, 256>>>(src, dst, B, 0, ctl); break;
                case 6: name = "region 1024 WGs x 1024"; region_copy<<<1024, 1024>>>((const v4u*)src, (v4u*)dst, bytes / 16 / 1024); break;
                case 8: name = "slot skew 4"; slot_copy<1, false><<<total + 3 * B, 256>>>(src, dst, B, 4, ctl); break;
                case 9: name = "slot skew 8"; slot_copy<1, false><<<total + 7 * B, 256>>>(src, dst, B, 8, ctl); break;
                case 10: name = "slot skew 16"; slot_copy<1, false><<<total + 15 * B, 256>>>(src, dst, B, 16, ctl); break;
                case 11: name = "slot skew 32"; slot_copy<1, false><<<total + 31 * B, 256>>>(src, dst, B, 32, ctl); break;
                case 7: name = "region 4096 WGs x 1024"; region_copy<<<4096, 1024>>>((const v4u*)src, (v4u*)dst, bytes / 16 / 4096); break;
                }
                CK(hipGetLastError());
                CK(hipEventRecord(e1, 0));
                CK(hipEventSynchronize(e1));
                float ms;
                CK(hipEventElapsedTime(&ms, e0, e1));
                if (r >= 2) { sum += ms; if (ms < best) best = ms; }
            }
            const float avg = sum / reps;
            printf("pass %d %-28s avg %.4f ms  best %.4f ms  %7.0f GB/s (r+w, avg)\n", pass, name, avg, best,
                   2.0 * bytes / avg / 1e6);
        }
    }
    return 0;
}
