// Partition-camping test for region-per-workgroup sweeps: a workgroup that owns one
// contiguous region (as k_scan_fast must, for its LDS histogram) streams it either from
// its start (every resident workgroup then sits at the same offset of a region whose size
// is a power of two — same HBM channel) or from a per-workgroup rotated start.
//   hipcc --offload-arch=gfx950 -O3 tools/ubench_stagger.hip -o tools/bin/ubench_stagger
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

typedef unsigned int v4u __attribute__((ext_vector_type(4)));
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

// region of `per` vectors per WG; iteration i of the WG covers vectors
// [(i + rot) % niter * step, +step) with step = blockDim * U
template <int U>
__global__ __launch_bounds__(1024) void region_copy(const v4u* __restrict__ src, v4u* __restrict__ dst, size_t per,
                                                    int stagger, unsigned* sink) {
    extern __shared__ unsigned lds[];
    const size_t step = (size_t)blockDim.x * U;
    const size_t niter = per / step;
    const size_t r0 = (size_t)blockIdx.x * per;
    size_t rot = 0;
    if (stagger == 1) rot = ((size_t)blockIdx.x * 2654435761u) % niter;
    if (stagger == 2) rot = ((size_t)blockIdx.x * niter) / gridDim.x;   // spread evenly
    unsigned acc = 0;
    for (size_t i = 0; i < niter; ++i) {
        size_t it = i + rot; if (it >= niter) it -= niter;
        const size_t base = r0 + it * step + threadIdx.x;
        v4u v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = __builtin_nontemporal_load(src + base + (size_t)u * blockDim.x);
#pragma unroll
        for (int u = 0; u < U; ++u) { __builtin_nontemporal_store(v[u], dst + base + (size_t)u * blockDim.x); acc += v[u].x & 1u; }
    }
    if (acc == 0xFFFFFFFFu) { lds[threadIdx.x] = acc; sink[0] = lds[threadIdx.x ^ 1]; }
}

// band pattern of k_scan_fast (16-row bands, wave = 64 consecutive 16-B chunks of a band
// row, 4 rows per batch), region = bands_per_wg bands of one 2048x2048 slice, with the
// band order rotated per WG
template <int U>
__global__ __launch_bounds__(1024) void band_copy(const v4u* __restrict__ src, v4u* __restrict__ dst, int bands_per_wg,
                                                  int stagger, unsigned* __restrict__ sink) {
    extern __shared__ unsigned lds[];
    constexpr int H = 2048, W = 2048, SB = 16;
    const int b = blockIdx.y;
    const size_t vps = (size_t)H * W / 8;
    const v4u* s0 = src + b * vps;
    v4u* d0 = dst + b * vps;
    const int stride = W / 8, CR = W / 8;
    const int band0 = blockIdx.x * bands_per_wg, nitems = bands_per_wg * CR;
    const int lane = threadIdx.x & 63;
    const int wgid = blockIdx.y * gridDim.x + blockIdx.x;
    int rot = 0;
    const int nit = nitems / blockDim.x;
    if (stagger) rot = (int)(((unsigned)wgid * 2654435761u) % (unsigned)nit);
    unsigned acc = 0;
    for (int k = 0; k < nit; ++k) {
        int kk = k + rot; if (kk >= nit) kk -= nit;
        const int it = kk * blockDim.x + (threadIdx.x & ~63) + lane;
        const int band = band0 + it / CR, c = it % CR;
        const v4u* s = s0 + (size_t)band * SB * stride + c;
        v4u* d = d0 + (size_t)band * SB * stride + c;
        for (int r = 0; r < SB; r += U) {
            v4u v[U];
#pragma unroll
            for (int u = 0; u < U; ++u) v[u] = __builtin_nontemporal_load(s + (size_t)(r + u) * stride);
#pragma unroll
            for (int u = 0; u < U; ++u) { __builtin_nontemporal_store(v[u], d + (size_t)(r + u) * stride); acc += v[u].x & 1u; }
        }
    }
    if (acc == 0xFFFFFFFFu) { lds[threadIdx.x] = acc; sink[0] = lds[threadIdx.x ^ 1]; }
}


// interleaved regions: groups of P workgroups share P consecutive regions; workgroup j of a
// group takes blocks j, j+P, j+2P, ... of the group's span (P resident workgroups then read
// one moving window of the span instead of P separate streams)
template <int U>
__global__ __launch_bounds__(1024) void inter_copy(const v4u* __restrict__ src, v4u* __restrict__ dst, size_t per,
                                                   int P, unsigned* sink) {
    extern __shared__ unsigned lds[];
    const size_t step = (size_t)blockDim.x * U;
    const size_t niter = per / step;               // blocks per region
    const int grp = blockIdx.x / P, j = blockIdx.x % P;
    const size_t span0 = (size_t)grp * P * per;
    unsigned acc = 0;
    for (size_t i = 0; i < niter; ++i) {
        const size_t blk = i * P + j;
        const size_t base = span0 + blk * step + threadIdx.x;
        v4u v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = __builtin_nontemporal_load(src + base + (size_t)u * blockDim.x);
#pragma unroll
        for (int u = 0; u < U; ++u) { __builtin_nontemporal_store(v[u], dst + base + (size_t)u * blockDim.x); acc += v[u].x & 1u; }
    }
    if (acc == 0xFFFFFFFFu) { lds[threadIdx.x] = acc; sink[0] = lds[threadIdx.x ^ 1]; }
}

// grid-stride over the whole buffer in 64 KiB blocks (moving window of all resident WGs)
template <int U>
__global__ __launch_bounds__(1024) void gs_copy(const v4u* __restrict__ src, v4u* __restrict__ dst, size_t nvec,
                                                unsigned* sink) {
    extern __shared__ unsigned lds[];
    const size_t step = (size_t)blockDim.x * U;
    unsigned acc = 0;
    for (size_t blk = blockIdx.x; (blk + 1) * step <= nvec; blk += gridDim.x) {
        const size_t base = blk * step + threadIdx.x;
        v4u v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = __builtin_nontemporal_load(src + base + (size_t)u * blockDim.x);
#pragma unroll
        for (int u = 0; u < U; ++u) { __builtin_nontemporal_store(v[u], dst + base + (size_t)u * blockDim.x); acc += v[u].x & 1u; }
    }
    if (acc == 0xFFFFFFFFu) { lds[threadIdx.x] = acc; sink[0] = lds[threadIdx.x ^ 1]; }
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
    const int B = 256;
    const size_t bytes = (size_t)B * 2048 * 2048 * 2;
    const size_t nvec = bytes / 16;
    v4u *src, *dst; unsigned* sink;
    CK(hipMalloc(&src, bytes)); CK(hipMalloc(&dst, bytes)); CK(hipMalloc(&sink, 64));
    CK(hipMemset(src, 1, bytes)); CK(hipMemset(dst, 0, bytes));
    CK(hipFuncSetAttribute((const void*)region_copy<4>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    CK(hipFuncSetAttribute((const void*)band_copy<4>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    CK(hipFuncSetAttribute((const void*)inter_copy<4>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    CK(hipFuncSetAttribute((const void*)gs_copy<4>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    const int reps = 10;
    for (int pass = 0; pass < 2; ++pass) {
        for (int wgs : {512, 1024, 2048}) {
            const size_t per = nvec / wgs;
            float t = timeit([&] { region_copy<4><<<wgs, 1024, 128 * 1024>>>(src, dst, per, 0, sink); }, reps);
            printf("pass %d region      wgs=%5d        %.3f ms  %6.0f GB/s\n", pass, wgs, t, 2.0 * bytes / t / 1e6);
            for (int P : {2, 4, 8, 16}) {
                float t2 = timeit([&] { inter_copy<4><<<wgs, 1024, 128 * 1024>>>(src, dst, per, P, sink); }, reps);
                printf("pass %d interleave  wgs=%5d P=%2d   %.3f ms  %6.0f GB/s\n", pass, wgs, P, t2, 2.0 * bytes / t2 / 1e6);
            }
        }
        for (int wgs : {256, 512, 1024, 4096}) {
            float t = timeit([&] { gs_copy<4><<<wgs, 1024, 128 * 1024>>>(src, dst, nvec, sink); }, reps);
            printf("pass %d gridstride  wgs=%5d        %.3f ms  %6.0f GB/s\n", pass, wgs, t, 2.0 * bytes / t / 1e6);
        }
    }
    CK(hipGetLastError());
    return 0;
}
