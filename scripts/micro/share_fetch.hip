// Microbenchmark: cost of a 64-B record fetch (four global_load_dwordx4 per lane) when
// groups of G consecutive lanes want the same random record (G = 1: every lane its own,
// G = 64: the whole wave one record).  Tells whether lanes sharing records (coherent rays)
// make the vector-memory path cheaper.  Prints ns per lane-record per CU.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void __launch_bounds__(256) fetch(const float4* __restrict__ tab, uint32_t nrec_mask, int group, int iters,
                                             float* out) {
    const int lane = threadIdx.x & 63;
    const uint32_t gid = (blockIdx.x * 256u + (threadIdx.x & ~63u)) + (uint32_t)(lane / group);
    uint32_t s = gid * 2654435761u + 777u;
    float acc = 0.0f;
    for (int i = 0; i < iters; ++i) {
        s = s * 1664525u + 1013904223u;
        const float4* r = tab + (size_t)((s >> 6) & nrec_mask) * 4;
        const float4 a = r[0], b = r[1], c = r[2], d = r[3];
        acc += a.x + b.y + c.z + d.w;
    }
    if (acc == 1234.5f) out[0] = acc;
}

int main() {
    const size_t max_bytes = (size_t)16 << 20;
    float4* tab;
    float* out;
    (void)hipMalloc(&tab, max_bytes);
    (void)hipMalloc(&out, 4);
    (void)hipMemset(tab, 0, max_bytes);
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    const int blocks = 256 * 8, iters = 128;
    for (size_t bytes : {(size_t)1 << 20, (size_t)16 << 20}) {
        for (int g : {1, 2, 4, 8, 16, 64}) {
            float ms = 0;
            for (int rep = 0; rep < 2; ++rep) {
                (void)hipEventRecord(a);
                hipLaunchKernelGGL(fetch, dim3(blocks), dim3(256), 0, 0, tab, (uint32_t)(bytes / 64 - 1), g, iters, out);
                (void)hipEventRecord(b);
                (void)hipEventSynchronize(b);
                (void)hipEventElapsedTime(&ms, a, b);
            }
            printf("table %5zu KB, %2d lanes per record: %.3f ms, %.3f ns per lane-record per CU\n", bytes >> 10, g, ms,
                   ms * 1e6 / ((double)blocks * 256 * iters / 256.0));
        }
    }
    return 0;
}
