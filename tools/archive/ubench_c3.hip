// C3-shape streaming ceilings (256 slices x 512^2 uint16 = 512 KiB per slice, one 1024-thread
// workgroup per slice and per CU, as k_pee_embed_ss): what a slice-serial workgroup can do
// per phase, and whether a second read of a slice it has just streamed is cheaper.
//   copy      : read slice -> write slice (the embed's traffic)
//   read      : read slice only (the capacity phase)
//   read+copy : read the slice, then copy it (the fused auto embed's traffic)
//   read+copy LDS k : the same, with the first k 32-KiB chunks kept in LDS by the read phase
//   write     : write only
// Each measurement alternates with a copy stego -> cover2 (as the bench's extract), so the
// Infinity Cache holds what the real step leaves in it.
//   hipcc --offload-arch=gfx950 -O3 tools/ubench_c3.hip -o tools/bin/ubench_c3
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

typedef unsigned int v4u __attribute__((ext_vector_type(4)));
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

constexpr int NT = 1024;
constexpr size_t SLICE = 512 * 512 * 2;             // bytes
constexpr size_t SVEC = SLICE / 16;                  // 16-B vectors per slice (32768)
constexpr int CHUNK = NT * 2;                        // vectors per chunk (2 per thread: 32 KiB)
constexpr int NCH = (int)(SVEC / CHUNK);             // 16 chunks

template <bool NTL> __device__ __forceinline__ v4u ld(const v4u* p) {
    if constexpr (NTL) return __builtin_nontemporal_load(p); else return *p;
}
template <bool NTS> __device__ __forceinline__ void st(v4u* p, v4u v) { if constexpr (NTS) __builtin_nontemporal_store(v, p); else *p = v; }

// mode 0 copy, 1 read, 2 read+copy, 3 write; hold = chunks kept in LDS by the read phase
template <int U, bool NTL, bool NTS = true>
__global__ __launch_bounds__(NT) void slice_kernel(const v4u* __restrict__ src, v4u* __restrict__ dst, int mode, int hold,
                                                   unsigned* sink) {
    extern __shared__ v4u lds[];                     // up to 4 chunks (128 KiB)
    const v4u* s = src + (size_t)blockIdx.x * SVEC;
    v4u* d = dst + (size_t)blockIdx.x * SVEC;
    const int t = threadIdx.x;
    unsigned acc = 0;
    if (mode == 1 || mode == 2) {                    // read phase
        for (int k0 = 0; k0 < NCH; k0 += U) {
            v4u a[U][2];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                a[u][0] = ld<false>(s + (size_t)(k0 + u) * CHUNK + t);
                a[u][1] = ld<false>(s + (size_t)(k0 + u) * CHUNK + NT + t);
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                acc ^= a[u][0].x ^ a[u][1].y ^ a[u][0].w ^ a[u][1].z;
                if (k0 + u < hold) { lds[(k0 + u) * CHUNK + t] = a[u][0]; lds[(k0 + u) * CHUNK + NT + t] = a[u][1]; }
            }
        }
        __syncthreads();
    }
    if (mode == 0 || mode == 2) {                    // copy phase
        for (int k0 = 0; k0 < NCH; k0 += U) {
            v4u a[U][2];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int k = k0 + u;
                if (mode == 2 && k < hold) {
                    a[u][0] = lds[k * CHUNK + t];
                    a[u][1] = lds[k * CHUNK + NT + t];
                } else {
                    a[u][0] = ld<NTL>(s + (size_t)k * CHUNK + t);
                    a[u][1] = ld<NTL>(s + (size_t)k * CHUNK + NT + t);
                }
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                st<NTS>(d + (size_t)(k0 + u) * CHUNK + t, a[u][0]);
                st<NTS>(d + (size_t)(k0 + u) * CHUNK + NT + t, a[u][1]);
            }
        }
    }
    if (mode == 3) {
        const v4u z = {(unsigned)t, 1u, 2u, 3u};
        for (int k = 0; k < NCH; ++k) { st<NTS>(d + (size_t)k * CHUNK + t, z); st<NTS>(d + (size_t)k * CHUNK + NT + t, z); }
    }
    if (acc == 0x9E3779B9u) sink[0] = acc;
}

int main() {
    const int B = 256;
    const size_t bytes = (size_t)B * SLICE;
    v4u *cov, *stg, *cov2; unsigned* sink;
    CK(hipMalloc(&cov, bytes)); CK(hipMalloc(&stg, bytes)); CK(hipMalloc(&cov2, bytes)); CK(hipMalloc(&sink, 64));
    CK(hipMemset(cov, 1, bytes)); CK(hipMemset(stg, 0, bytes)); CK(hipMemset(cov2, 0, bytes));
#define ATTR(...) CK(hipFuncSetAttribute((const void*)__VA_ARGS__, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024))
    ATTR(slice_kernel<4, true, true>); ATTR(slice_kernel<4, false, true>); ATTR(slice_kernel<4, false, false>);
    ATTR(slice_kernel<4, true, false>); ATTR(slice_kernel<2, false, true>); ATTR(slice_kernel<8, false, true>);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    const size_t lds = 128 * 1024;                    // one workgroup per CU
    auto run = [&](const char* name, int variant, int mode, int hold, double gb) {
        float tot = 0;
        const int reps = 20;
        for (int r = 0; r < reps + 3; ++r) {
            CK(hipEventRecord(e0));
            switch (variant) {
                case 0: slice_kernel<4, true, true><<<B, NT, lds>>>(cov, stg, mode, hold, sink); break;
                case 1: slice_kernel<4, false, true><<<B, NT, lds>>>(cov, stg, mode, hold, sink); break;
                case 2: slice_kernel<4, false, false><<<B, NT, lds>>>(cov, stg, mode, hold, sink); break;
                case 3: slice_kernel<4, true, false><<<B, NT, lds>>>(cov, stg, mode, hold, sink); break;
                case 4: slice_kernel<2, false, true><<<B, NT, lds>>>(cov, stg, mode, hold, sink); break;
                default: slice_kernel<8, false, true><<<B, NT, lds>>>(cov, stg, mode, hold, sink); break;
            }
            CK(hipEventRecord(e1));
            slice_kernel<4, true, true><<<B, NT, lds>>>(stg, cov2, 0, 0, sink);   // the "extract"
            CK(hipEventSynchronize(e1));
            float ms; CK(hipEventElapsedTime(&ms, e0, e1));
            if (r >= 3) tot += ms;
        }
        const float t = tot / reps;
        static const char* vn[] = {"U4 ntl nts", "U4 ld nts", "U4 ld st", "U4 ntl st", "U2 ld nts", "U8 ld nts"};
        printf("%-16s %-11s hold=%d  %.4f ms  %6.0f GB/s (of %.0f MB)\n", name, vn[variant], hold, t, gb / t / 1e-3 / 1e3, gb);
    };
    const double mb = bytes / 1e6;
    for (int pass = 0; pass < 2; ++pass) {
        for (int v = 0; v < 6; ++v) run("copy", v, 0, 0, 2 * mb);
        run("read", 1, 1, 0, mb);
        run("read", 5, 1, 0, mb);
        run("write", 0, 3, 0, mb);
        run("write", 2, 3, 0, mb);
        for (int v : {0, 1, 2}) run("read+copy", v, 2, 0, 3 * mb);
        run("read+copy LDS", 1, 2, 4, 3 * mb);
        run("read+copy LDS", 2, 2, 4, 3 * mb);
    }
    CK(hipGetLastError());
    return 0;
}
