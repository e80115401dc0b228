// Copy + LDS value-histogram sweep (the shape of k_scan_rows) on ct12-like data: does a
// smaller per-workgroup histogram (8-bit quarters, 64 KiB -> two workgroups per CU) stream
// better than the 16-bit halves (128 KiB, one workgroup per CU)?  Wrap bookkeeping is left
// out (it is rare); only the copy and the per-pixel LDS atomics are timed.
//   hipcc --offload-arch=gfx950 -O3 tools/ubench_hist.hip -o tools/bin/ubench_hist
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

typedef unsigned int v4u __attribute__((ext_vector_type(4)));
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

__global__ void fill_ct12(unsigned short* img, size_t n, int W) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const int x = (int)(i % W), y = (int)((i / W) % W);
        unsigned h = (unsigned)i * 2654435761u; h ^= h >> 15; h *= 2246822519u; h ^= h >> 13;
        const float noise = ((int)(h & 63) - 32) * 0.5f;
        float v = (sinf(x / 97.f) + cosf(y / 61.f) + 2.f) * 0.25f * 4095.f * 0.8f + noise;
        v = fminf(fmaxf(v, 0.f), 4095.f);
        img[i] = (unsigned short)v;
    }
}

// MODE 16: 16-bit halves (word v>>1); MODE 8: 8-bit quarters (word v>>2)
template <int MODE>
__global__ __launch_bounds__(1024) void copy_hist(const v4u* __restrict__ src, v4u* __restrict__ dst, size_t per,
                                                  unsigned* sink) {
    extern __shared__ unsigned lds[];
    const int words = MODE == 16 ? 32768 : 16384;
    for (int i = threadIdx.x; i < words; i += blockDim.x) lds[i] = 0;
    __syncthreads();
    const size_t step = (size_t)blockDim.x * 4;
    const size_t r0 = (size_t)blockIdx.x * per;
    unsigned acc = 0;
    for (size_t base = r0 + threadIdx.x; base + 3 * blockDim.x < r0 + per; base += step) {
        v4u v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) v[u] = __builtin_nontemporal_load(src + base + (size_t)u * blockDim.x);
#pragma unroll
        for (int u = 0; u < 4; ++u) __builtin_nontemporal_store(v[u], dst + base + (size_t)u * blockDim.x);
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            unsigned px[8] = {v[u].x & 0xFFFFu, v[u].x >> 16, v[u].y & 0xFFFFu, v[u].y >> 16,
                              v[u].z & 0xFFFFu, v[u].z >> 16, v[u].w & 0xFFFFu, v[u].w >> 16};
            unsigned old[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                if (MODE == 16) old[k] = atomicAdd(&lds[px[k] >> 1], 1u << (16 * (px[k] & 1)));
                else old[k] = atomicAdd(&lds[(px[k] >> 2) & 16383], 1u << (8 * (px[k] & 3)));
            }
#pragma unroll
            for (int k = 0; k < 8; ++k) acc += old[k] >> 31;
        }
    }
    __syncthreads();
    if (acc == 12345) sink[0] = lds[threadIdx.x];
}

template <class F>
static float timeit(F f, int reps) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    f(); f();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(a));
    for (int i = 0; i < reps; ++i) f();
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms; CK(hipEventElapsedTime(&ms, a, b));
    return ms / reps;
}

int main() {
    const int B = 256, W = 2048;
    const size_t n = (size_t)B * W * W, bytes = n * 2, nvec = bytes / 16;
    unsigned short* img; v4u* dst; unsigned* sink;
    CK(hipMalloc(&img, bytes)); CK(hipMalloc(&dst, bytes)); CK(hipMalloc(&sink, 64));
    fill_ct12<<<4096, 256>>>(img, n, W);
    CK(hipDeviceSynchronize());
    CK(hipFuncSetAttribute((const void*)copy_hist<16>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    CK(hipFuncSetAttribute((const void*)copy_hist<8>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    const v4u* src = reinterpret_cast<const v4u*>(img);
    for (int pass = 0; pass < 2; ++pass)
        for (int wgs : {512, 1024, 2048}) {
            const size_t per = nvec / wgs;
            float t16 = timeit([&] { copy_hist<16><<<wgs, 1024, 128 * 1024>>>(src, dst, per, sink); }, 5);
            float t8a = timeit([&] { copy_hist<8><<<wgs, 1024, 64 * 1024>>>(src, dst, per, sink); }, 5);
            float t8b = timeit([&] { copy_hist<8><<<wgs * 2, 512, 64 * 1024>>>(src, dst, per / 2, sink); }, 5);
            printf("pass %d wgs=%5d  16-bit/128KiB/1024thr %.3f ms   8-bit/64KiB/1024thr %.3f ms   8-bit/64KiB/512thr(x2 wgs) %.3f ms\n",
                   pass, wgs, t16, t8a, t8b);
        }
    CK(hipGetLastError());
    return 0;
}
