// Microbenchmark: fetching one random 64-B record per lane (4 x global_load_dwordx4, quad j
// of the lane's own record in instruction j) against a cooperative fetch (in instruction j
// the four lanes of a quad group load the four 16-B quads of the record of group member j,
// so each instruction touches 16 records instead of 64).  Prints ns per record-fetch per CU.
#include <hip/hip_runtime.h>
#include <cstdio>

template <bool COOP>
__global__ void __launch_bounds__(256) fetch(const float4* __restrict__ tab, uint32_t nrec_mask, int iters, float* out) {
    const int lane = threadIdx.x & 63;
    uint32_t s = (blockIdx.x * 256u + threadIdx.x) * 2654435761u + 777u;
    float acc = 0.0f;
    for (int i = 0; i < iters; ++i) {
        s = s * 1664525u + 1013904223u;
        const uint32_t rec = (s >> 6) & nrec_mask;   // this lane's record
        if (!COOP) {
            const float4* r = tab + (size_t)rec * 4;
            const float4 a = r[0], b = r[1], c = r[2], d = r[3];
            acc += a.x + b.y + c.z + d.w;
        } else {
            const int base = lane & ~3, q = lane & 3;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const uint32_t rj = __shfl(rec, base + j);          // group member j's record
                const float4 v = tab[(size_t)rj * 4 + q];           // its quad q
                acc += v.x + v.w;
            }
        }
    }
    if (acc == 1234.5f) out[0] = acc;
}

int main() {
    const size_t max_bytes = (size_t)64 << 20;
    float4* tab;
    float* out;
    (void)hipMalloc(&tab, max_bytes);
    (void)hipMalloc(&out, 4);
    (void)hipMemset(tab, 0, max_bytes);
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    const int blocks = 256 * 8, iters = 128;
    for (size_t bytes : {(size_t)16 << 10, (size_t)1 << 20, (size_t)16 << 20, (size_t)64 << 20}) {
        const uint32_t mask = (uint32_t)(bytes / 64 - 1);
        for (int coop = 0; coop < 2; ++coop) {
            float ms = 0;
            for (int rep = 0; rep < 2; ++rep) {
                (void)hipEventRecord(a);
                if (coop) hipLaunchKernelGGL(fetch<true>, dim3(blocks), dim3(256), 0, 0, tab, mask, iters, out);
                else hipLaunchKernelGGL(fetch<false>, dim3(blocks), dim3(256), 0, 0, tab, mask, iters, out);
                (void)hipEventRecord(b);
                (void)hipEventSynchronize(b);
                (void)hipEventElapsedTime(&ms, a, b);
            }
            const double rec_per_cu = (double)blocks * 256 * iters / 256.0;
            printf("table %6zu KB %s: %.3f ms, %.3f ns per record per CU\n", bytes >> 10, coop ? "coop " : "plain",
                   ms, ms * 1e6 / rec_per_cu);
        }
    }
    return 0;
}
