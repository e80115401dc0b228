// LDS atomic throughput on one CU (1024-thread workgroup, every CU busy): lane-ops per
// cycle for ds_add_u32 with / without return, by address pattern.  Bounds the value
// histogram of k_scan_rows / k_scan_fast (one LDS atomic per distinct pixel run).
//   hipcc --offload-arch=gfx950 -O3 tools/ubench_lds_atomic.hip -o tools/bin/ubench_lds_atomic
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

// pattern 0: lane-distinct consecutive words; 1: pseudo-random over 32768 words;
// 2: 64 lanes over 16 words (4-way same-address); 3: all lanes one word;
// 4: smooth ramp (lane/2 + noise over 8 words): neighbouring-pixel-like
template <bool RTN>
__global__ __launch_bounds__(1024) void lds_atomics(int pattern, int iters, unsigned* out) {
    __shared__ unsigned h[32768];
    for (int i = threadIdx.x; i < 32768; i += 1024) h[i] = 0;
    __syncthreads();
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    unsigned x = threadIdx.x * 2654435761u + blockIdx.x;
    unsigned acc = 0;
    for (int it = 0; it < iters; ++it) {
        unsigned a[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            x = x * 1664525u + 1013904223u;
            switch (pattern) {
                case 0: a[k] = (wv * 64 + lane + k * 1024 + it * 8) & 32767; break;
                case 1: a[k] = (x >> 7) & 32767; break;
                case 2: a[k] = (lane >> 2) + k * 64 + wv * 1024; break;
                case 3: a[k] = k + wv * 16; break;
                default: a[k] = ((lane >> 1) + ((x >> 20) & 7) + it * 3 + wv * 512 + k * 37) & 32767; break;
            }
        }
        if (RTN) {
            unsigned o[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) o[k] = atomicAdd(&h[a[k]], 1u);
#pragma unroll
            for (int k = 0; k < 8; ++k) acc += o[k] >> 31;
        } else {
#pragma unroll
            for (int k = 0; k < 8; ++k) atomicAdd(&h[a[k]], 1u);
        }
    }
    __syncthreads();
    if (acc == 12345) out[0] = h[threadIdx.x];
    if (threadIdx.x == 0) out[1 + blockIdx.x] = h[7];
}

int main() {
    int dev = 0, ncu = 0, clk = 0;
    CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
    CK(hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, dev));
    unsigned* out;
    CK(hipMalloc(&out, 4096 * 4));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    const int iters = 4096;
    const char* names[] = {"distinct", "random32K", "4-way-same", "all-same(16/wave)", "smooth"};
    for (int rtn = 0; rtn < 2; ++rtn)
        for (int p = 0; p < 5; ++p) {
            for (int rep = 0; rep < 2; ++rep) {
                CK(hipEventRecord(e0));
                if (rtn) lds_atomics<true><<<ncu, 1024>>>(p, iters, out);
                else lds_atomics<false><<<ncu, 1024>>>(p, iters, out);
                CK(hipEventRecord(e1));
                CK(hipEventSynchronize(e1));
                float ms; CK(hipEventElapsedTime(&ms, e0, e1));
                if (rep == 1) {
                    const double ops = 1024.0 * iters * 8;              // lane-ops per CU
                    const double cyc = ms * 1e-3 * clk * 1e3;            // clk in kHz
                    printf("%-4s %-18s %.3f ms  %.2f lane-ops/cycle/CU (clk %d MHz)  %.1f Gops/s chip\n",
                           rtn ? "rtn" : "nrtn", names[p], ms, ops / cyc, clk / 1000, ops * ncu / (ms * 1e-3) / 1e9);
                }
            }
        }
    return 0;
}
