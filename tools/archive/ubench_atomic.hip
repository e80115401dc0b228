// Cost of the inter-workgroup primitives a look-back scan is built from, at the PEE
// chunk grid (65 536 workgroups of 256 threads): atomic-with-return tickets on one
// address / on 256 per-slice lines, agent-scope loads/stores of status words.
//   hipcc --offload-arch=gfx950 -O3 tools/ubench_atomic.hip -o /tmp/uba && /tmp/uba
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

__global__ __launch_bounds__(256) void k_empty(unsigned* sink) {
    if (threadIdx.x == 0 && blockIdx.x == 0xFFFFFFFu) sink[0] = 1;
}
// MODE 0: one address; 1: per-slice lines (blockIdx / 256, 128-B apart); 2: per-WG address
template <int MODE>
__global__ __launch_bounds__(256) void k_ticket(unsigned* ctr, unsigned* sink) {
    __shared__ unsigned s;
    if (threadIdx.x == 0) {
        unsigned* p = MODE == 0 ? ctr : (MODE == 1 ? ctr + 32 * (blockIdx.x / 256) : ctr + 32 * blockIdx.x);
        s = atomicAdd(p, 1u);
    }
    __syncthreads();
    if (s == 0xFFFFFFFFu) sink[threadIdx.x] = s;
}
template <int MODE>
__global__ __launch_bounds__(256) void k_noret(unsigned* ctr) {
    if (threadIdx.x == 0) {
        unsigned* p = MODE == 0 ? ctr : ctr + 32 * (blockIdx.x / 256);
        atomicAdd(p, 1u);
    }
}
// status publish + one 64-word look-back read by wave 0 (no waiting)
__global__ __launch_bounds__(256) void k_status(unsigned long long* st, unsigned* sink) {
    const int c = blockIdx.x & 255;
    unsigned long long* s = st + (blockIdx.x / 256) * 256;
    if (threadIdx.x == 0) __hip_atomic_store(s + c, 1ull << 62 | 5, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (threadIdx.x < 64) {
        const int idx = c - 1 - (int)threadIdx.x;
        unsigned long long w = idx >= 0 ? __hip_atomic_load(s + idx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0;
        if (w == 0xFFFFFFFFFFFFFFFFull) sink[0] = 1;
    }
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
    unsigned *ctr, *sink;
    unsigned long long* st;
    const int G = 65536;
    CK(hipMalloc(&ctr, (size_t)G * 32 * 4)); CK(hipMalloc(&sink, 4096)); CK(hipMalloc(&st, (size_t)G * 8));
    CK(hipMemset(ctr, 0, (size_t)G * 32 * 4)); CK(hipMemset(st, 0, (size_t)G * 8));
    const int reps = 10;
    for (int n : {8192, 65536}) {
        printf("grid %6d  empty          %.4f ms\n", n, timeit([&] { k_empty<<<n, 256>>>(sink); }, reps));
        printf("grid %6d  ticket 1 addr  %.4f ms\n", n, timeit([&] { k_ticket<0><<<n, 256>>>(ctr, sink); }, reps));
        printf("grid %6d  ticket /slice  %.4f ms\n", n, timeit([&] { k_ticket<1><<<n, 256>>>(ctr, sink); }, reps));
        printf("grid %6d  ticket /WG     %.4f ms\n", n, timeit([&] { k_ticket<2><<<n, 256>>>(ctr, sink); }, reps));
        printf("grid %6d  noret 1 addr   %.4f ms\n", n, timeit([&] { k_noret<0><<<n, 256>>>(ctr); }, reps));
        printf("grid %6d  noret /slice   %.4f ms\n", n, timeit([&] { k_noret<1><<<n, 256>>>(ctr); }, reps));
        printf("grid %6d  status+lookbk  %.4f ms\n", n, timeit([&] { k_status<<<n, 256>>>(st, sink); }, reps));
    }
    CK(hipGetLastError());
    return 0;
}
