// Scan-shaped streaming ceiling: the access pattern of k_scan_fast without its histogram
// (band of 16 rows per wave item, workgroup owns `bands_per_wg` bands of one slice, dynamic
// LDS reserved to pin occupancy).  Separates "one 1024-thread WG per CU" (the 128 KiB LDS
// histogram) from "large contiguous region per WG" as causes of the scan's gap to the
// grid-stride copy ceiling.
//   hipcc --offload-arch=gfx950 -O3 tools/ubench_scan.hip -o /tmp/ubench_scan && /tmp/ubench_scan
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

typedef unsigned int v4u __attribute__((ext_vector_type(4)));
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

constexpr int H = 2048, W = 2048, B = 256, SB = 16;

template <int U, int NT>
__global__ __launch_bounds__(1024) void scan_like(const v4u* __restrict__ src, v4u* __restrict__ dst, int bands_per_wg,
                                                  unsigned* __restrict__ sink) {
    extern __shared__ unsigned lds[];
    const int b = blockIdx.y;
    const size_t vps = (size_t)H * W / 8;   // 16-B vectors per slice
    const v4u* s0 = src + b * vps;
    v4u* d0 = dst + b * vps;
    const int stride = W / 8, CR = W / 8;
    const int band0 = blockIdx.x * bands_per_wg, nitems = bands_per_wg * CR;
    const int lane = threadIdx.x & 63;
    unsigned acc = 0;
    for (int base = (threadIdx.x & ~63); base < nitems; base += blockDim.x) {
        const int it = base + lane;
        const int band = band0 + it / CR, c = it % CR;
        const v4u* s = s0 + (size_t)band * SB * stride + c;
        v4u* d = d0 + (size_t)band * SB * stride + c;
        for (int r = 0; r < SB; r += U) {
            v4u v[U];
#pragma unroll
            for (int u = 0; u < U; ++u) v[u] = NT ? __builtin_nontemporal_load(s + (size_t)(r + u) * stride) : s[(size_t)(r + u) * stride];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                if (NT) __builtin_nontemporal_store(v[u], d + (size_t)(r + u) * stride); else d[(size_t)(r + u) * stride] = v[u];
                acc += v[u].x & 1u;
            }
        }
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
    const size_t bytes = (size_t)B * H * W * 2;
    v4u *src, *dst; unsigned* sink;
    CK(hipMalloc(&src, bytes)); CK(hipMalloc(&dst, bytes)); CK(hipMalloc(&sink, 64));
    CK(hipMemset(src, 1, bytes)); CK(hipMemset(dst, 0, bytes));
    CK(hipFuncSetAttribute((const void*)scan_like<4, 1>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    CK(hipFuncSetAttribute((const void*)scan_like<8, 1>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    CK(hipFuncSetAttribute((const void*)scan_like<4, 0>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    const int reps = 10;
    const int nbands = H / SB;
    for (int pass = 0; pass < 2; ++pass)
    for (int lds_kb : {128, 64, 40, 0})
        for (int threads : {1024, 512, 256})
            for (int wgs : {4, 16, 64}) {
                const int bpw = nbands / wgs;
                dim3 grid(wgs, B);
                const size_t sh = (size_t)lds_kb * 1024;
                float t4 = timeit([&] { scan_like<4, 1><<<grid, threads, sh>>>(src, dst, bpw, sink); }, reps);
                float t8 = timeit([&] { scan_like<8, 1><<<grid, threads, sh>>>(src, dst, bpw, sink); }, reps);
                float tp = timeit([&] { scan_like<4, 0><<<grid, threads, sh>>>(src, dst, bpw, sink); }, reps);
                printf("pass %d lds=%3dKB threads=%4d wgs/slice=%3d  U4nt %.3f ms (%6.0f GB/s)  U8nt %.3f  U4plain %.3f\n",
                       pass, lds_kb, threads, wgs, t4, 2.0 * bytes / t4 / 1e6, t8, tp);
            }
    CK(hipGetLastError());
    CK(hipFree(src)); CK(hipFree(dst));
    return 0;
}
