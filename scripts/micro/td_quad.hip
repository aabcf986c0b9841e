// td_quad.hip -- micro-benchmark: is a vector-memory gather charged per
// active LANE or per active QUAD (group of 4 lanes)?  Every CU runs 8 waves per SIMD; each
// active lane loops over `iters` inner-record-shaped fetches (three 16-B loads + one 8-B
// load of a 64-B record, the address depending on the previous record) from a table of
// `nrec` records.  Lane patterns (which lanes are active, which record each reads):
//   all64-quad  : 64 lanes, the 4 lanes of a quad read the same record (16 records / wave)
//   lead16      : lane 0 of every quad only (16 lanes in 16 quads), one record each
//   all64-lane  : 64 lanes, every lane its own record
//   pack16-lane : lanes 0..15 (16 lanes in 4 quads), every lane its own record
//   pack16-quad : lanes 0..15, the 4 lanes of a quad read the same record (4 records)
//   lead4       : lane 0 of quads 0..3 only (4 lanes in 4 quads)
//   hipcc --offload-arch=gfx950 -O3 -o td_quad td_quad.hip && ./td_quad
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

enum { ALL64_QUAD, LEAD16, ALL64_LANE, PACK16_LANE, PACK16_QUAD, LEAD4, NPAT };
static const char* kName[NPAT] = {"all64-quad", "lead16", "all64-lane", "pack16-lane", "pack16-quad", "lead4"};

__global__ void __launch_bounds__(256) gather(const float4* __restrict__ table, uint32_t nrec, uint32_t iters,
                                              int pat, uint32_t* __restrict__ sink) {
    const uint32_t lane = threadIdx.x & 63u;
    bool act;
    uint32_t key;   // lanes with the same key read the same record sequence
    switch (pat) {
        case ALL64_QUAD: act = true; key = lane >> 2; break;
        case LEAD16: act = (lane & 3u) == 0; key = lane >> 2; break;
        case ALL64_LANE: act = true; key = lane; break;
        case PACK16_LANE: act = lane < 16; key = lane; break;
        case PACK16_QUAD: act = lane < 16; key = lane >> 2; break;
        default: act = (lane & 3u) == 0 && lane < 16; key = lane >> 2; break;
    }
    uint32_t x = ((blockIdx.x * 4u + (threadIdx.x >> 6)) * 64u + key) * 2654435761u + 0x9E3779B9u;
    uint32_t acc = 0;
    if (act) {
        for (uint32_t i = 0; i < iters; ++i) {
            x ^= x << 13; x ^= x >> 17; x ^= x << 5;
            const uint32_t idx = (x ^ (acc & 1u)) % nrec;   // depends on the previous record
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
    const uint32_t blocks = cus * 8;   // 8 blocks of 4 waves per CU = 8 waves per SIMD
    const uint32_t maxrec = 1u << 14;
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
    printf("nrec    KiB  pattern       ms       ns/wave-iter/CU\n");
    for (uint32_t nrec : {256u, 16384u})
        for (int pat = 0; pat < NPAT; ++pat) {
            hipLaunchKernelGGL(gather, dim3(blocks), dim3(256), 0, 0, table, nrec, iters, pat, sink);
            hipEventRecord(e0, 0);
            for (int k = 0; k < 4; ++k) hipLaunchKernelGGL(gather, dim3(blocks), dim3(256), 0, 0, table, nrec, iters, pat, sink);
            hipEventRecord(e1, 0);
            hipEventSynchronize(e1);
            float ms = 0;
            hipEventElapsedTime(&ms, e0, e1);
            ms /= 4;
            const double wave_iters = (double)blocks * 4 * iters;
            printf("%6u %5u  %-12s  %.4f   %8.3f\n", nrec, nrec * 64 / 1024, kName[pat], ms, ms * 1e6 / wave_iters * cus);
        }
    return 0;
}
