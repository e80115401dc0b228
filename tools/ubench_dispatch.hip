// Workgroup dispatch spread of one-workgroup-per-CU launches (the C3 slice-serial kernels'
// shape): 256 workgroups, each stamps wall_clock64() (100 MHz) as its first instruction and
// then streams its own 512 KiB region (a copy, so that the launch is not empty).  Variants:
// workgroup size 1024 / 512 / 256 threads, static LDS 0 / 64 / 160 KiB.  Prints the start
// spread and the median start per XCD (workgroup b on XCD b % 8).
//   hipcc --offload-arch=gfx950 -O3 tools/ubench_dispatch.hip -o tools/r05/ubench_dispatch.bin
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

typedef unsigned int v4u __attribute__((ext_vector_type(4)));

template <int NT, int LDSW, int SCR = 0>
__global__ __launch_bounds__(NT) void k_disp(const v4u* __restrict__ src, v4u* __restrict__ dst, long long* st,
                                             long long* en, int nvec) {
    long long t0 = 0;
    if (threadIdx.x == 0) t0 = wall_clock64();
    unsigned scr_acc = 0;
    if (SCR > 0) {   // a dynamically indexed private array: forces scratch (SCR words per lane)
        volatile unsigned loc[SCR > 0 ? SCR : 1];
        for (int i = 0; i < SCR; ++i) loc[i] = threadIdx.x + i;
        scr_acc = loc[(threadIdx.x * 7) % (SCR > 0 ? SCR : 1)];
    }
    __shared__ unsigned lds[LDSW > 0 ? LDSW : 1];
    if (LDSW > 0) {
        for (int i = threadIdx.x; i < LDSW; i += NT) lds[i] = 0;
        __syncthreads();
    }
    const v4u* s = src + (size_t)blockIdx.x * nvec;
    v4u* d = dst + (size_t)blockIdx.x * nvec;
    unsigned acc = 0;
    for (int i = threadIdx.x; i < nvec; i += NT) {
        v4u v = __builtin_nontemporal_load(s + i);
        acc += v.x;
        __builtin_nontemporal_store(v, d + i);
    }
    if (LDSW > 0) {
        atomicAdd(&lds[threadIdx.x % (LDSW > 0 ? LDSW : 1)], acc);
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        st[blockIdx.x] = t0;
        en[blockIdx.x] = wall_clock64() + (LDSW > 0 ? (lds[0] & 0) : 0) + (scr_acc & 0);
    }
}

template <int NT, int LDSW, int SCR = 0>
void run(const char* name, const v4u* src, v4u* dst, long long* dst_st, long long* dst_en, int nvec) {
    const int G = 256;
    std::vector<long long> st(G), en(G);
    double best_spread = 1e30, med_len = 0, best_ms = 0;
    std::vector<double> xmed(8);
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int rep = 0; rep < 10; ++rep) {
        CK(hipEventRecord(a, 0));
        hipLaunchKernelGGL((k_disp<NT, LDSW, SCR>), dim3(G), dim3(NT), 0, 0, src, dst, dst_st, dst_en, nvec);
        CK(hipEventRecord(b, 0));
        CK(hipDeviceSynchronize());
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        CK(hipMemcpy(st.data(), dst_st, G * 8, hipMemcpyDeviceToHost));
        CK(hipMemcpy(en.data(), dst_en, G * 8, hipMemcpyDeviceToHost));
        const long long s0 = *std::min_element(st.begin(), st.end());
        const long long s1 = *std::max_element(st.begin(), st.end());
        if (rep >= 2 && (s1 - s0) * 0.01 < best_spread) {
            best_spread = (s1 - s0) * 0.01;
            best_ms = ms;
            std::vector<double> len(G);
            for (int i = 0; i < G; ++i) len[i] = (en[i] - st[i]) * 0.01;
            std::sort(len.begin(), len.end());
            med_len = len[G / 2];
            for (int x = 0; x < 8; ++x) {
                std::vector<double> v;
                for (int i = x; i < G; i += 8) v.push_back((st[i] - s0) * 0.01);
                std::sort(v.begin(), v.end());
                xmed[x] = v[v.size() / 2];
            }
        }
    }
    printf("%-26s kernel %.4f ms  start spread %.2f us  median workgroup %.2f us  starts by XCD:", name, best_ms,
           best_spread, med_len);
    for (int x = 0; x < 8; ++x) printf(" %.2f", xmed[x]);
    printf("\n");
}

int main() {
    const int nvec = 512 * 1024 / 16;   // 512 KiB per workgroup
    v4u *src, *dst;
    long long *st, *en;
    CK(hipMalloc(&src, (size_t)256 * nvec * 16));
    CK(hipMalloc(&dst, (size_t)256 * nvec * 16));
    CK(hipMemset(src, 1, (size_t)256 * nvec * 16));
    CK(hipMalloc(&st, 256 * 8));
    CK(hipMalloc(&en, 256 * 8));
    run<1024, 0>("1024 thr, no LDS", src, dst, st, en, nvec);
    run<1024, 16384>("1024 thr, 64 KiB LDS", src, dst, st, en, nvec);
    run<1024, 40960>("1024 thr, 160 KiB LDS", src, dst, st, en, nvec);
    run<512, 40960>("512 thr, 160 KiB LDS", src, dst, st, en, nvec);
    run<256, 40960>("256 thr, 160 KiB LDS", src, dst, st, en, nvec);
    run<256, 0>("256 thr, no LDS", src, dst, st, en, nvec);
    run<1024, 0>("1024 thr, no LDS (again)", src, dst, st, en, nvec);
    run<1024, 40960, 10>("1024 thr, 160 KiB, scratch 40 B", src, dst, st, en, nvec);
    run<1024, 0, 10>("1024 thr, no LDS, scratch 40 B", src, dst, st, en, nvec);
    run<1024, 40960, 64>("1024 thr, 160 KiB, scratch 256 B", src, dst, st, en, nvec);
    run<1024, 40960, 0>("1024 thr, 160 KiB (again)", src, dst, st, en, nvec);
    return 0;
}
