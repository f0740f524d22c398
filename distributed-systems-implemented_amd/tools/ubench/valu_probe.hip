// valu_probe.hip — issue cost of the integer VALU instructions the wc map
// kernel's per-word path uses (gfx950), at the map kernel's occupancy (16 waves
// per CU, 256 workgroups x 1024 threads): cycles per wave-instruction per SIMD
// for 8 independent chains of one instruction.
// Build: hipcc -O3 --offload-arch=gfx950 valu_probe.hip -o valu_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CHK(x)                                                                        \
    do {                                                                              \
        hipError_t e_ = (x);                                                          \
        if (e_ != hipSuccess) {                                                       \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                  \
        }                                                                             \
    } while (0)

#define OP8(INS)                                                                                                  \
    asm volatile(INS " %0, %0, %8\n\t" INS " %1, %1, %8\n\t" INS " %2, %2, %8\n\t" INS " %3, %3, %8\n\t" INS          \
                     " %4, %4, %8\n\t" INS " %5, %5, %8\n\t" INS " %6, %6, %8\n\t" INS " %7, %7, %8"                \
                 : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)                   \
                 : "v"(k))
#define OP8_3(INS)                                                                                                \
    asm volatile(INS " %0, %0, %8, 3\n\t" INS " %1, %1, %8, 3\n\t" INS " %2, %2, %8, 3\n\t" INS " %3, %3, %8, 3\n\t" \
                 INS " %4, %4, %8, 3\n\t" INS " %5, %5, %8, 3\n\t" INS " %6, %6, %8, 3\n\t" INS " %7, %7, %8, 3"     \
                 : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)                   \
                 : "v"(k))

#define BOP3(INS) asm volatile("v_bitop3_b32 %0, %0, %8, %0 bitop3:0x96\n\tv_bitop3_b32 %1, %1, %8, %1 bitop3:0x96\n\tv_bitop3_b32 %2, %2, %8, %2 bitop3:0x96\n\tv_bitop3_b32 %3, %3, %8, %3 bitop3:0x96\n\tv_bitop3_b32 %4, %4, %8, %4 bitop3:0x96\n\tv_bitop3_b32 %5, %5, %8, %5 bitop3:0x96\n\tv_bitop3_b32 %6, %6, %8, %6 bitop3:0x96\n\tv_bitop3_b32 %7, %7, %8, %7 bitop3:0x96" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(k))
#define UN(INS) asm volatile(INS " %0, %0\n\t" INS " %1, %1\n\t" INS " %2, %2\n\t" INS " %3, %3\n\t" INS " %4, %4\n\t" INS " %5, %5\n\t" INS " %6, %6\n\t" INS " %7, %7" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(k))
#define CMPV(INS) asm volatile(INS " vcc, %0, %8\n\t" INS " vcc, %1, %8\n\t" INS " vcc, %2, %8\n\t" INS " vcc, %3, %8\n\t" INS " vcc, %4, %8\n\t" INS " vcc, %5, %8\n\t" INS " vcc, %6, %8\n\t" INS " vcc, %7, %8" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(k) : "vcc")
#define CMPS(INS) asm volatile(INS " s[40:41], %0, %8\n\t" INS " s[42:43], %1, %8\n\t" INS " s[44:45], %2, %8\n\t" INS " s[46:47], %3, %8\n\t" INS " s[48:49], %4, %8\n\t" INS " s[50:51], %5, %8\n\t" INS " s[52:53], %6, %8\n\t" INS " s[54:55], %7, %8" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(k) : "s40","s41","s42","s43","s44","s45","s46","s47","s48","s49","s50","s51","s52","s53","s54","s55")
#define FFBL(INS) asm volatile("v_ffbl_b32 %0, %0\n\tv_ffbl_b32 %1, %1\n\tv_ffbl_b32 %2, %2\n\tv_ffbl_b32 %3, %3\n\tv_ffbl_b32 %4, %4\n\tv_ffbl_b32 %5, %5\n\tv_ffbl_b32 %6, %6\n\tv_ffbl_b32 %7, %7" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(k))
#define CND(INS) asm volatile("s_mov_b64 s[40:41], 0x5555\n\tv_cndmask_b32_e64 %0, %0, %8, s[40:41]\n\tv_cndmask_b32_e64 %1, %1, %8, s[40:41]\n\tv_cndmask_b32_e64 %2, %2, %8, s[40:41]\n\tv_cndmask_b32_e64 %3, %3, %8, s[40:41]\n\tv_cndmask_b32_e64 %4, %4, %8, s[40:41]\n\tv_cndmask_b32_e64 %5, %5, %8, s[40:41]\n\tv_cndmask_b32_e64 %6, %6, %8, s[40:41]\n\tv_cndmask_b32_e64 %7, %7, %8, s[40:41]" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(k) : "s40", "s41")
#define CNDV(INS) asm volatile("s_mov_b64 vcc, 0x5555\n\tv_cndmask_b32 %0, %0, %8, vcc\n\tv_cndmask_b32 %1, %1, %8, vcc\n\tv_cndmask_b32 %2, %2, %8, vcc\n\tv_cndmask_b32 %3, %3, %8, vcc\n\tv_cndmask_b32 %4, %4, %8, vcc\n\tv_cndmask_b32 %5, %5, %8, vcc\n\tv_cndmask_b32 %6, %6, %8, vcc\n\tv_cndmask_b32 %7, %7, %8, vcc" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(k) : "vcc")
#define CMP64(INS) asm volatile("v_cmp_eq_u64 s[40:41], %0, %1\n\tv_cmp_eq_u64 s[42:43], %2, %3\n\tv_cmp_eq_u64 s[44:45], %4, %5\n\tv_cmp_eq_u64 s[46:47], %6, %7\n\tv_cmp_eq_u64 s[48:49], %0, %2\n\tv_cmp_eq_u64 s[50:51], %4, %6\n\tv_cmp_eq_u64 s[52:53], %1, %3\n\tv_cmp_eq_u64 s[54:55], %5, %7" : "+v"(q0), "+v"(q1), "+v"(q2), "+v"(q3), "+v"(q4), "+v"(q5), "+v"(q6), "+v"(q7) : : "s40","s41","s42","s43","s44","s45","s46","s47","s48","s49","s50","s51","s52","s53","s54","s55","scc")

template <int M>
__global__ void __launch_bounds__(1024) probe(unsigned* out, int iters) {
    unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6,
             a7 = a0 + 7, k = 0x9E3779B1u ^ blockIdx.x;
    unsigned long long q0 = a0, q1 = a1 + 9, q2 = a2, q3 = a3 + 9, q4 = a4, q5 = a5 + 9, q6 = a6, q7 = a7 + 9;
    for (int it = 0; it < iters; it++) {
        if constexpr (M == 0) OP8("v_add_u32");
        if constexpr (M == 1) OP8("v_lshrrev_b32");
        if constexpr (M == 2) OP8("v_lshlrev_b32");
        if constexpr (M == 3) OP8("v_or_b32");
        if constexpr (M == 4) OP8("v_xor_b32");
        if constexpr (M == 5) OP8("v_ashrrev_i32");
        if constexpr (M == 6) OP8("v_subrev_u32");
        if constexpr (M == 7) OP8("v_min_u32");
        if constexpr (M == 8) OP8("v_max_i32");
        if constexpr (M == 9) OP8("v_mul_u32_u24");
        if constexpr (M == 10) OP8("v_lshlrev_b32_e64");
        if constexpr (M == 11) OP8("v_lshrrev_b32_e64");
        if constexpr (M == 12) OP8_3("v_bfi_b32");
        if constexpr (M == 13) OP8_3("v_or3_b32");
        if constexpr (M == 14) OP8_3("v_mad_u32_u24");
        if constexpr (M == 15) OP8_3("v_alignbyte_b32");
        if constexpr (M == 16) OP8_3("v_and_or_b32");
        if constexpr (M == 17) BOP3("v_bitop3_b32");
        if constexpr (M == 18) CMPV("v_cmp_gt_u32");
        if constexpr (M == 19) CMPS("v_cmp_gt_u32_e64");
        if constexpr (M == 20) OP8("v_mbcnt_lo_u32_b32");
        if constexpr (M == 21) OP8("v_mbcnt_hi_u32_b32");
        if constexpr (M == 22) UN("v_not_b32");
        if constexpr (M == 23) UN("v_mov_b32");
        if constexpr (M == 24) UN("v_ffbl_b32");
        if constexpr (M == 25) CND("v_cndmask_b32_e64");
    }
    a0 ^= (unsigned)(q0 ^ q1 ^ q2 ^ q3 ^ q4 ^ q5 ^ q6 ^ q7);
    if ((a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7) == 0x12345) out[0] = 1;
}

template <int M>
static void run(const char* name, unsigned* d) {
    const int iters = 20000;
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0));
    CHK(hipEventCreate(&e1));
    probe<M><<<256, 1024>>>(d, 100);
    CHK(hipDeviceSynchronize());
    CHK(hipEventRecord(e0));
    probe<M><<<256, 1024>>>(d, iters);
    CHK(hipEventRecord(e1));
    CHK(hipEventSynchronize(e1));
    float ms = 0;
    CHK(hipEventElapsedTime(&ms, e0, e1));
    // per SIMD: 4 waves x iters x 8 instructions; at an assumed 2.4 GHz clock
    const double cyc = ms * 1e-3 * 2.4e9 / (4.0 * iters * 8);
    printf("%-16s %8.3f ms  %5.2f cyc per wave-instruction per SIMD (2.4 GHz)\n", name, ms, cyc);
    fflush(stdout);
}

int main() {
    unsigned* d;
    CHK(hipMalloc(&d, 64));
    run<0>("v_add_u32", d);
    run<1>("v_lshrrev_b32", d);
    run<2>("v_lshlrev_b32", d);
    run<3>("v_or_b32", d);
    run<4>("v_xor_b32", d);
    run<5>("v_ashrrev_i32", d);
    run<6>("v_subrev_u32", d);
    run<7>("v_min_u32", d);
    run<8>("v_max_i32", d);
    run<9>("v_mul_u32_u24", d);
    run<10>("v_lshlrev_b32_e64", d);
    run<11>("v_lshrrev_b32_e64", d);
    run<12>("v_bfi_b32", d);
    run<13>("v_or3_b32", d);
    run<14>("v_mad_u32_u24", d);
    run<15>("v_alignbyte_b32", d);
    run<16>("v_and_or_b32", d);
    run<17>("v_bitop3_b32", d);
    run<18>("v_cmp_gt_u32", d);
    run<19>("v_cmp_gt_u32_e64", d);
    run<20>("v_mbcnt_lo_u32_b32", d);
    run<21>("v_mbcnt_hi_u32_b32", d);
    run<22>("v_not_b32", d);
    run<23>("v_mov_b32", d);
    run<24>("v_ffbl_b32", d);
    run<25>("v_cndmask_b32_e64", d);
    return 0;
}
