// Microbenchmark: does a partially-masked global_load_dwordx4 cost the vector-memory
// path as much as a full one?  Random 16-B gathers from a 64 MB table (L2 / Infinity
// Cache resident), ITER dependent-free loads per lane, with only `active` lanes of each
// wave executing the load.  Prints ns per wave-level load instruction per CU.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__global__ void __launch_bounds__(256) gather(const float4* __restrict__ tab, uint32_t mask_n, int active, int iters,
                                              float* out) {
    const int lane = threadIdx.x & 63;
    uint32_t s = (blockIdx.x * 256u + threadIdx.x) * 2654435761u + 12345u;
    float acc = 0.0f;
    if (lane < active) {
        for (int i = 0; i < iters; ++i) {
            s = s * 1664525u + 1013904223u;
            const float4 v = tab[(s >> 4) & mask_n];
            acc += v.x + v.w;
        }
    }
    if (acc == 1234.5f) out[0] = acc;
}

int main() {
    const size_t n = (64u << 20) / 16;  // 64 MB of float4
    float4* tab;
    float* out;
    hipMalloc(&tab, n * 16);
    hipMalloc(&out, 4);
    hipMemset(tab, 0, n * 16);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const int blocks = 256 * 8, iters = 256;
    for (size_t tab_bytes : {(size_t)16 << 10, (size_t)1 << 20, (size_t)64 << 20}) {
    printf("table %zu KB\n", tab_bytes >> 10);
    for (int active : {64, 32, 16, 8, 1}) {
        for (int rep = 0; rep < 2; ++rep) {
            hipEventRecord(a);
            hipLaunchKernelGGL(gather, dim3(blocks), dim3(256), 0, 0, tab, (uint32_t)(tab_bytes / 16 - 1), active, iters, out);
            hipEventRecord(b);
            hipEventSynchronize(b);
            float ms = 0;
            hipEventElapsedTime(&ms, a, b);
            const double insts_per_cu = (double)blocks * 4 * iters / 256.0;
            if (rep) printf("active lanes %2d: %.3f ms, %.2f ns per wave load instruction per CU, %.1f GB/s useful\n",
                            active, ms, ms * 1e6 / insts_per_cu, (double)blocks * 4 * iters * active * 16 / (ms * 1e6));
        }
    }
    }
    return 0;
}
