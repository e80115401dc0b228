// Streaming-copy ceiling on this MI355X: what a read-B + write-B pass can reach, by
// load/store flavour, unroll and grid size.  Sets the target for k_scan_fast / k_restore.
//   hipcc --offload-arch=gfx950 -O3 tools/ubench_stream.hip -o /tmp/ubench && /tmp/ubench
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

typedef unsigned int v4u __attribute__((ext_vector_type(4)));
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

template <int U, int NT_LD, int NT_ST>
__global__ __launch_bounds__(256) void copy_gs(const v4u* __restrict__ src, v4u* __restrict__ dst, size_t n) {
    const size_t stride = (size_t)gridDim.x * 256 * U;
    for (size_t base = (size_t)blockIdx.x * 256 * U + threadIdx.x; base < n; base += stride) {
        v4u v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const size_t i = base + (size_t)u * 256;
            if (i < n) v[u] = NT_LD ? __builtin_nontemporal_load(src + i) : src[i];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const size_t i = base + (size_t)u * 256;
            if (i < n) {
                if (NT_ST) __builtin_nontemporal_store(v[u], dst + i); else dst[i] = v[u];
            }
        }
    }
}

// contiguous chunk per block (like k_restore / k_scan_fast: each WG owns a range)
template <int U>
__global__ __launch_bounds__(256) void copy_chunk(const v4u* __restrict__ src, v4u* __restrict__ dst, size_t n,
                                                  size_t per) {
    const size_t c0 = (size_t)blockIdx.x * per, c1 = c0 + per < n ? c0 + per : n;
    for (size_t base = c0 + threadIdx.x; base < c1; base += 256 * U) {
        v4u v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) if (base + u * 256 < c1) v[u] = src[base + u * 256];
#pragma unroll
        for (int u = 0; u < U; ++u) if (base + u * 256 < c1) dst[base + u * 256] = v[u];
    }
}

template <int U>
__global__ __launch_bounds__(256) void copy_chunk_nt(const v4u* __restrict__ src, v4u* __restrict__ dst, size_t n,
                                                     size_t per) {
    const size_t c0 = (size_t)blockIdx.x * per, c1 = c0 + per < n ? c0 + per : n;
    for (size_t base = c0 + threadIdx.x; base < c1; base += 256 * U) {
        v4u v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) if (base + u * 256 < c1) v[u] = __builtin_nontemporal_load(src + base + u * 256);
#pragma unroll
        for (int u = 0; u < U; ++u) if (base + u * 256 < c1) __builtin_nontemporal_store(v[u], dst + base + u * 256);
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
    const size_t bytes = (size_t)256 * 2048 * 2048 * 2;   // the benchmark's cover batch
    const size_t n = bytes / 16;
    v4u *src, *dst;
    CK(hipMalloc(&src, bytes)); CK(hipMalloc(&dst, bytes));
    CK(hipMemset(src, 1, bytes)); CK(hipMemset(dst, 0, bytes));
    const int reps = 10;
    auto report = [&](const char* name, float ms) {
        printf("%-44s %8.3f ms  %7.1f GB/s (r+w)\n", name, ms, 2.0 * bytes / ms / 1e6);
    };
    report("hipMemcpyAsync D2D", timeit([&] { (void)hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, 0); }, reps));
    for (int g : {1024, 2048, 4096, 8192, 16384}) {
        char nm[96];
        snprintf(nm, sizeof nm, "grid-stride U=4 plain grid=%d", g);
        report(nm, timeit([&] { copy_gs<4, 0, 0><<<g, 256>>>(src, dst, n); }, reps));
    }
    report("grid-stride U=1 plain grid=8192", timeit([&] { copy_gs<1, 0, 0><<<8192, 256>>>(src, dst, n); }, reps));
    report("grid-stride U=8 plain grid=4096", timeit([&] { copy_gs<8, 0, 0><<<4096, 256>>>(src, dst, n); }, reps));
    report("grid-stride U=4 nt-load grid=4096", timeit([&] { copy_gs<4, 1, 0><<<4096, 256>>>(src, dst, n); }, reps));
    report("grid-stride U=4 nt-store grid=4096", timeit([&] { copy_gs<4, 0, 1><<<4096, 256>>>(src, dst, n); }, reps));
    report("grid-stride U=4 nt-both grid=4096", timeit([&] { copy_gs<4, 1, 1><<<4096, 256>>>(src, dst, n); }, reps));
    for (int g : {256, 512, 2048, 8192, 32768}) {
        char nm[96];
        snprintf(nm, sizeof nm, "chunk-per-WG U=4 grid=%d", g);
        const size_t per = (n + g - 1) / g;
        report(nm, timeit([&] { copy_chunk<4><<<g, 256>>>(src, dst, n, per); }, reps));
    }
    for (int g : {2048, 8192, 16384, 32768}) {
        char nm[96];
        snprintf(nm, sizeof nm, "grid-stride U=4 nt-both grid=%d", g);
        report(nm, timeit([&] { copy_gs<4, 1, 1><<<g, 256>>>(src, dst, n); }, reps));
    }
    report("grid-stride U=2 nt-both grid=8192", timeit([&] { copy_gs<2, 1, 1><<<8192, 256>>>(src, dst, n); }, reps));
    report("grid-stride U=8 nt-both grid=8192", timeit([&] { copy_gs<8, 1, 1><<<8192, 256>>>(src, dst, n); }, reps));
    for (int g : {256, 2048, 8192, 32768}) {
        char nm[96];
        snprintf(nm, sizeof nm, "chunk-per-WG U=4 nt-both grid=%d", g);
        const size_t per = (n + g - 1) / g;
        report(nm, timeit([&] { copy_chunk_nt<4><<<g, 256>>>(src, dst, n, per); }, reps));
    }
    // repeat the baseline at the end (DVFS / drift check)
    report("grid-stride U=4 plain grid=4096 (again)", timeit([&] { copy_gs<4, 0, 0><<<4096, 256>>>(src, dst, n); }, reps));
    report("grid-stride U=4 nt-both grid=4096 (again)", timeit([&] { copy_gs<4, 1, 1><<<4096, 256>>>(src, dst, n); }, reps));
    CK(hipFree(src)); CK(hipFree(dst));
    return 0;
}
