// td_active.hip -- micro-benchmark: does a record gather cost per
// wave instruction or per active lane?  Every CU runs 8 waves per SIMD; in each wave only
// the first `active` lanes loop over `iters` inner-record-shaped fetches (three 16-B loads
// + one 8-B load of a 64-B record) from a table of `nrec` records; `dep` makes each fetch's
// address depend on the previous record (the traversal's pointer chase).
//   hipcc --offload-arch=gfx950 -O3 -o td_active td_active.hip && ./td_active
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__global__ void __launch_bounds__(256) gather(const float4* __restrict__ table, uint32_t nrec, uint32_t iters,
                                              uint32_t active, uint32_t dep, uint32_t* __restrict__ sink) {
    const uint32_t lane = threadIdx.x & 63u;
    uint32_t x = (blockIdx.x * 256u + threadIdx.x) * 2654435761u + 0x9E3779B9u;
    uint32_t acc = 0;
    if (lane < active) {
        for (uint32_t i = 0; i < iters; ++i) {
            x ^= x << 13; x ^= x >> 17; x ^= x << 5;
            const uint32_t idx = (dep ? (x ^ acc) : x) % nrec;
            const float4* p = table + (size_t)idx * 4;
            const float4 q0 = p[0], q1 = p[1], q2 = p[2];
            const float2 r = *reinterpret_cast<const float2*>(p + 3);
            acc += __float_as_uint(q0.x) ^ __float_as_uint(q1.y) ^ __float_as_uint(q2.z) ^ __float_as_uint(r.y);
        }
    }
    if (acc == 0x9E3779B9u) sink[blockIdx.x] = acc;
}

int main() {
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    const uint32_t blocks = cus * 8;
    const uint32_t maxrec = 1u << 20;
    float4* table;
    uint32_t* sink;
    hipMalloc(&table, (size_t)maxrec * 64);
    hipMalloc(&sink, blocks * 4);
    std::vector<float4> h((size_t)maxrec * 4);
    for (size_t i = 0; i < h.size(); ++i) h[i] = make_float4((float)(i & 7), 1.f, 2.f, 3.f);
    hipMemcpy(table, h.data(), h.size() * 16, hipMemcpyHostToDevice);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const uint32_t iters = 256;
    printf("nrec     KiB  dep active  ms      ns/wave-iter/CU  ns/lane-iter/CU\n");
    for (uint32_t nrec : {256u, 16384u, 262144u})
        for (uint32_t dep : {0u, 1u})
            for (uint32_t active : {64u, 48u, 32u, 16u, 4u}) {
                hipLaunchKernelGGL(gather, dim3(blocks), dim3(256), 0, 0, table, nrec, iters, active, dep, sink);
                hipEventRecord(e0, 0);
                for (int k = 0; k < 4; ++k)
                    hipLaunchKernelGGL(gather, dim3(blocks), dim3(256), 0, 0, table, nrec, iters, active, dep, sink);
                hipEventRecord(e1, 0);
                hipEventSynchronize(e1);
                float ms = 0;
                hipEventElapsedTime(&ms, e0, e1);
                ms /= 4;
                const double wave_iters = (double)blocks * 4 * iters;
                printf("%7u %6u  %u   %3u   %.4f   %8.3f         %8.3f\n", nrec, nrec * 64 / 1024, dep, active, ms,
                       ms * 1e6 / wave_iters * cus, ms * 1e6 / (wave_iters * active) * cus);
            }
    return 0;
}
