// quad_coop.hip -- micro-benchmark: the traversal's lanes mostly read ONE
// record per quad (2.6 lanes per quad request on C3).  Today each lane fetches the whole
// 56-B record itself with four loads (3 x 16 B + 8 B).  Alternative: the quad fetches the
// 64-B record cooperatively -- lane q loads 16-B chunk q, ONE load instruction -- and DPP
// quad broadcasts hand every lane all four chunks.  8 waves per SIMD on every CU, each lane
// chasing its own (or its quad's) random records.
//   mode 0: every lane its own record, 4 loads         (distinct per lane)
//   mode 1: one record per quad, every lane 4 loads    (today's traversal, coherent quads)
//   mode 2: one record per quad, 1 cooperative load + 12 DPP moves
//   hipcc --offload-arch=gfx950 -O3 -o quad_coop quad_coop.hip && ./quad_coop
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__device__ __forceinline__ float bq(float v, int c) {   // value of lane c of this quad
    const int ctrl = c * 0x55;                          // quad_perm [c, c, c, c]
    switch (c) {
        case 0: return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x00, 0xF, 0xF, false));
        case 1: return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x55, 0xF, 0xF, false));
        case 2: return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xAA, 0xF, 0xF, false));
        default: return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xFF, 0xF, 0xF, false));
    }
    (void)ctrl;
}

template <int MODE>
__global__ void __launch_bounds__(256) chase(const float4* __restrict__ table, uint32_t nrec, uint32_t iters,
                                             uint32_t* __restrict__ sink) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t key = MODE == 0 ? (blockIdx.x * 256u + threadIdx.x) : ((blockIdx.x * 256u + threadIdx.x) >> 2);
    uint32_t x = key * 2654435761u + 0x9E3779B9u;
    uint32_t acc = 0;
    for (uint32_t i = 0; i < iters; ++i) {
        x ^= x << 13; x ^= x >> 17; x ^= x << 5;
        const uint32_t idx = (x ^ (acc & 1u)) % nrec;   // dependent on the last record
        const float4* p = table + (size_t)idx * 4;
        float a, b, c, d;
        if (MODE == 2) {
            const float4 m = p[lane & 3u];               // chunk (lane & 3) of the quad's record
            a = bq(m.x, 0); b = bq(m.y, 1); c = bq(m.z, 2); d = bq(m.y, 3);
            const float e = bq(m.w, 0) + bq(m.x, 1) + bq(m.w, 1) + bq(m.x, 2) + bq(m.y, 2) + bq(m.w, 2)
                          + bq(m.x, 3) + bq(m.z, 3);
            a += e;
        } else {
            const float4 q0 = p[0], q1 = p[1], q2 = p[2];
            const float2 r = *reinterpret_cast<const float2*>(p + 3);
            a = q0.x + q0.w + q1.x + q1.w + q2.x + q2.w; b = q1.y + q0.y; c = q2.z + q0.z; d = r.y + r.x + q1.z + q2.y;
        }
        acc += __float_as_uint(a) ^ __float_as_uint(b) ^ __float_as_uint(c) ^ __float_as_uint(d);
    }
    if (acc == 0x9E3779B9u) sink[blockIdx.x] = acc;
}

template <int MODE>
static float run(const float4* t, uint32_t nrec, uint32_t iters, uint32_t blocks, uint32_t* sink) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    hipLaunchKernelGGL(chase<MODE>, dim3(blocks), dim3(256), 0, 0, t, nrec, iters, sink);
    (void)hipEventRecord(e0, 0);
    for (int k = 0; k < 4; ++k) hipLaunchKernelGGL(chase<MODE>, dim3(blocks), dim3(256), 0, 0, t, nrec, iters, sink);
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    return ms / 4;
}

int main() {
    int cus = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    const uint32_t blocks = cus * 8, iters = 256, maxrec = 1u << 20;
    float4* table;
    uint32_t* sink;
    (void)hipMalloc(&table, (size_t)maxrec * 64);
    (void)hipMalloc(&sink, blocks * 4);
    std::vector<float4> h((size_t)maxrec * 4, make_float4(1.f, 2.f, 3.f, 4.f));
    (void)hipMemcpy(table, h.data(), h.size() * 16, hipMemcpyHostToDevice);
    const double lane_iters = (double)blocks * 256 * iters;
    printf("nrec    KiB   mode  ms       ns/lane-iter/CU\n");
    for (uint32_t nrec : {256u, 16384u, 262144u, 1u << 20}) {
        const float m0 = run<0>(table, nrec, iters, blocks, sink);
        const float m1 = run<1>(table, nrec, iters, blocks, sink);
        const float m2 = run<2>(table, nrec, iters, blocks, sink);
        const float ms[3] = {m0, m1, m2};
        for (int m = 0; m < 3; ++m)
            printf("%7u %6u  %d   %.4f   %.3f\n", nrec, nrec * 64 / 1024, m, ms[m], ms[m] * 1e6 / lane_iters * cus);
    }
    return 0;
}
