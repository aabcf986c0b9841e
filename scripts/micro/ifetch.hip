// Microbenchmark: what a LONE wave pays per instruction when its loop does not fit the
// instruction buffer (the traversal main loop is 1,040 bytes; the lone-block SQ
// counters show ~31 instruction fetches per trip and 2/3 of the wave's cycles not issuing).
// One wave (or one wave per SIMD of one CU) runs a loop whose body is N independent VALU adds
// over 8 accumulators, in the 4-byte (VOP2, _e32) or the 8-byte (VOP3, _e64) encoding, with or
// without a taken s_branch after every 8 instructions; prints ns and shader cycles per
// instruction (s_memrealtime 100 MHz; s_memtime).
#include <hip/hip_runtime.h>
#include <cstdio>

#define R8(x) x x x x x x x x
#define ADD4 "v_add_f32_e32 %0, %8, %0\n v_add_f32_e32 %1, %8, %1\n v_add_f32_e32 %2, %8, %2\n v_add_f32_e32 %3, %8, %3\n" \
             "v_add_f32_e32 %4, %8, %4\n v_add_f32_e32 %5, %8, %5\n v_add_f32_e32 %6, %8, %6\n v_add_f32_e32 %7, %8, %7\n"
#define ADD8 "v_add_f32_e64 %0, %8, %0\n v_add_f32_e64 %1, %8, %1\n v_add_f32_e64 %2, %8, %2\n v_add_f32_e64 %3, %8, %3\n" \
             "v_add_f32_e64 %4, %8, %4\n v_add_f32_e64 %5, %8, %5\n v_add_f32_e64 %6, %8, %6\n v_add_f32_e64 %7, %8, %7\n"
#define JMP "s_branch 1f\n 1:\n"
// a taken branch over 64 / 256 / 1024 bytes of never-executed s_nop: the target is not in the
// instruction bytes already fetched
#define JMP64 "s_branch 1f\n .fill 16, 4, 0xBF800000\n 1:\n"
#define JMP256 "s_branch 1f\n .fill 64, 4, 0xBF800000\n 1:\n"
#define JMP1K "s_branch 1f\n .fill 256, 4, 0xBF800000\n 1:\n"
// a VALU compare into an SGPR pair, a SALU op on it, a VALU select by it (x4): the VALU -> SALU
// -> VALU mask hand-offs of the traversal loop's branch-free steps
#define HOFF1(i, j) "v_cmp_lt_f32_e64 s[40:41], %" #i ", %8\n s_and_b64 s[42:43], s[40:41], exec\n v_cndmask_b32_e64 %" #j ", %" #j ", %8, s[42:43]\n"
#define MASK HOFF1(0, 1) HOFF1(2, 3) HOFF1(4, 5) HOFF1(6, 7)
// exec saved, narrowed to all lanes, one add, restored (x4): the if-blocks' exec dance
#define EXEC1(i) "s_and_saveexec_b64 s[40:41], s[42:43]\n v_add_f32_e32 %" #i ", %8, %" #i "\n s_or_b64 exec, exec, s[40:41]\n"
#define EXEC EXEC1(0) EXEC1(1) EXEC1(2) EXEC1(3)

// V: 0 = 4-byte adds, 1 = 8-byte adds, 2 = 4-byte adds + a taken branch per 8, 3 = 8-byte + branch,
// 4/5/6 = 4-byte adds + a taken branch over 64 B / 256 B / 1 KB per 8, 7 = MASK, 8 = EXEC
// (7 and 8 count each group of 8 as 8: divide by 12/8 or 13/8 for per-instruction figures)
// N8: the body is N8 x 8 adds (N8 = 1, 8, 32)
template <int V, int N8>
__global__ void __launch_bounds__(256) body(int iters, float b, unsigned long long* t) {
    float a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    const unsigned long long r0 = __builtin_amdgcn_s_memrealtime(), c0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int k = 0; k < N8; ++k) {
            if (V == 0) asm volatile(ADD4 : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b));
            if (V == 1) asm volatile(ADD8 : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b));
            if (V == 2) asm volatile(ADD4 JMP : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b));
            if (V == 3) asm volatile(ADD8 JMP : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b));
            if (V == 4) asm volatile(ADD4 JMP64 : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b));
            if (V == 5) asm volatile(ADD4 JMP256 : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b));
            if (V == 7) asm volatile(MASK : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b) : "s40", "s41", "s42", "s43", "scc");
            if (V == 8) asm volatile("s_mov_b64 s[42:43], -1\n" EXEC : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b) : "s40", "s41", "s42", "s43", "scc");
            if (V == 6) asm volatile(ADD4 JMP1K : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b));
        }
    }
    const unsigned long long r1 = __builtin_amdgcn_s_memrealtime(), c1 = __builtin_amdgcn_s_memtime();
    const float s = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
    if ((threadIdx.x & 63) == 0) {
        const int w = threadIdx.x >> 6;
        t[2 * w] = r1 - r0;
        t[2 * w + 1] = c1 - c0;
    }
    if (s == 1234.5f) t[15] = 1;
}

template <int V, int N8>
void run(const char* name, int waves, unsigned long long* d) {
    const int iters = 20000 / N8;
    const long insts = (long)iters * N8 * 8;
    unsigned long long h[16];
    for (int rep = 0; rep < 3; ++rep) {
        hipLaunchKernelGGL((body<V, N8>), dim3(1), dim3(64 * waves), 0, 0, iters, 1e-7f, d);
        (void)hipDeviceSynchronize();
    }
    (void)hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    printf("{\"variant\": \"%s\", \"body_insts\": %d, \"waves\": %d, \"ns_per_inst\": %.3f, \"cycles_per_inst\": %.3f}\n",
           name, N8 * 8, waves, h[0] * 10.0 / insts, (double)h[1] / insts);
}

int main(int argc, char** argv) {
    unsigned long long* d;
    (void)hipMalloc(&d, 16 * sizeof(unsigned long long));
    const int only1 = argc > 1;   // under rocprofv3 --pmc: one wave only, one dispatch set per kernel
    for (int waves : {1, 4}) {
        if (only1 && waves != 1) continue;
        run<0, 1>("add_4B", waves, d);
        run<0, 8>("add_4B", waves, d);
        run<0, 32>("add_4B", waves, d);
        run<1, 1>("add_8B", waves, d);
        run<1, 8>("add_8B", waves, d);
        run<1, 32>("add_8B", waves, d);
        run<2, 8>("add_4B_branch_per_8", waves, d);
        run<2, 32>("add_4B_branch_per_8", waves, d);
        run<3, 8>("add_8B_branch_per_8", waves, d);
        run<3, 32>("add_8B_branch_per_8", waves, d);
        run<4, 8>("add_4B_branch_over_64B_per_8", waves, d);
        run<5, 8>("add_4B_branch_over_256B_per_8", waves, d);
        run<6, 4>("add_4B_branch_over_1KB_per_8", waves, d);
        run<7, 8>("mask_handoff_12_insts_per_8", waves, d);     // per 8 "insts": 12 instructions
        run<8, 8>("exec_dance_13_insts_per_8", waves, d);       // 1 + 12 instructions

    }
    return 0;
}
