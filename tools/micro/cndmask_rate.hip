// Microbenchmark (dev only): what an s_nop between VALU instructions costs,
// and is a VOP2 v_cndmask_b32 that reads VCC slow on
// gfx950?  valu_rate.hip measured ~23.6 SIMD-cycles per instruction for
// back-to-back `v_cndmask_b32 vX, vX, vY, vcc` with VCC never written in the
// loop, against ~4.4 for the VOP3 form reading an SGPR pair.  Here: the same
// with VCC set by SALU before the loop, with VCC set by a VALU compare before
// the loop, the compiler's usual pair (v_cmp_*_e32 vcc then v_cndmask_b32_e32
// reading it), and the VOP3 pair on s[12:13], at 5 waves per SIMD.
//   hipcc --offload-arch=gfx950 -O3 tools/micro/cndmask_rate.hip -o /tmp/cndmask_rate
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

constexpr int ITER = 2048;
#define R8(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)
#define REP4(S) S S S S

template <int OP>
__global__ __launch_bounds__(64) void k(uint32_t seed, uint32_t* out) {
    uint32_t a0 = seed ^ threadIdx.x, a1 = a0 * 3, a2 = a0 * 5, a3 = a0 * 7, a4 = a0 * 9, a5 = a0 * 11, a6 = a0 * 13,
             a7 = a0 * 15;
    const uint32_t c = seed * 0x9E3779B1u + 1;
    if (OP == 1) asm volatile("s_mov_b64 vcc, -1" ::: "vcc");
    if (OP == 2) asm volatile("v_cmp_gt_u32 vcc, %0, %1" ::"v"(a0), "v"(c) : "vcc");
    for (int it = 0; it < ITER; ++it) {
        if (OP == 0 || OP == 1 || OP == 2) {   // 32 selects reading VCC
#define X(i) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(a##i) : "v"(c) : "vcc");
            REP4(R8(X))
#undef X
        } else if (OP == 3) {   // 16 pairs: VOP2 compare into VCC, VOP2 select reading it
#define X(i) asm volatile("v_cmp_gt_i32 vcc, %0, %1\n v_cndmask_b32 %0, %0, %1, vcc" : "+v"(a##i) : "v"(c) : "vcc");
            REP4(X(0) X(1) X(2) X(3))
#undef X
        } else if (OP == 4) {   // 16 pairs on an SGPR pair (VOP3)
#define X(i) asm volatile("v_cmp_gt_i32_e64 s[12:13], %0, %1\n v_cndmask_b32_e64 %0, %0, %1, s[12:13]" : "+v"(a##i) : "v"(c) : "s12", "s13");
            REP4(X(0) X(1) X(2) X(3))
#undef X
        } else if (OP == 6) {   // 32 adds, each followed by s_nop 0
#define X(i) asm volatile("v_add_u32 %0, %0, %1\n s_nop 0" : "+v"(a##i) : "v"(c));
            REP4(R8(X))
#undef X
        } else if (OP == 7) {   // 32 adds, each followed by s_nop 1
#define X(i) asm volatile("v_add_u32 %0, %0, %1\n s_nop 1" : "+v"(a##i) : "v"(c));
            REP4(R8(X))
#undef X
        } else if (OP == 8) {   // a dependent DPP add chain (row_shr:1), as the compiler emits it (s_nop 1 before each)
#define X(i) asm volatile("s_nop 1\n v_add_u32_dpp %0, %0, %0 row_shr:1 row_mask:0xf bank_mask:0xf" : "+v"(a##i));
            REP4(R8(X))
#undef X
        } else if (OP == 9) {   // eight independent DPP add chains interleaved, no s_nop (no hazard: the source was written 8 VALU back)
#define X(i) asm volatile("v_add_u32_dpp %0, %0, %0 row_shr:1 row_mask:0xf bank_mask:0xf" : "+v"(a##i));
            REP4(R8(X))
#undef X
        } else if (OP == 10) {   // one compare into VCC, then 7 VOP2 selects reading it, one asm block (no s_nop between)
            asm volatile("v_cmp_gt_i32 vcc, %0, %8\n v_cndmask_b32 %1, %1, %8, vcc\n v_cndmask_b32 %2, %2, %8, vcc\n"
                         " v_cndmask_b32 %3, %3, %8, vcc\n v_cndmask_b32 %4, %4, %8, vcc\n v_cndmask_b32 %5, %5, %8, vcc\n"
                         " v_cndmask_b32 %6, %6, %8, vcc\n v_cndmask_b32 %7, %7, %8, vcc"
                         : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(c) : "vcc");
            asm volatile("v_cmp_gt_i32 vcc, %0, %8\n v_cndmask_b32 %1, %1, %8, vcc\n v_cndmask_b32 %2, %2, %8, vcc\n"
                         " v_cndmask_b32 %3, %3, %8, vcc\n v_cndmask_b32 %4, %4, %8, vcc\n v_cndmask_b32 %5, %5, %8, vcc\n"
                         " v_cndmask_b32 %6, %6, %8, vcc\n v_cndmask_b32 %7, %7, %8, vcc"
                         : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(c) : "vcc");
            asm volatile("v_cmp_gt_i32 vcc, %0, %8\n v_cndmask_b32 %1, %1, %8, vcc\n v_cndmask_b32 %2, %2, %8, vcc\n"
                         " v_cndmask_b32 %3, %3, %8, vcc\n v_cndmask_b32 %4, %4, %8, vcc\n v_cndmask_b32 %5, %5, %8, vcc\n"
                         " v_cndmask_b32 %6, %6, %8, vcc\n v_cndmask_b32 %7, %7, %8, vcc"
                         : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(c) : "vcc");
            asm volatile("v_cmp_gt_i32 vcc, %0, %8\n v_cndmask_b32 %1, %1, %8, vcc\n v_cndmask_b32 %2, %2, %8, vcc\n"
                         " v_cndmask_b32 %3, %3, %8, vcc\n v_cndmask_b32 %4, %4, %8, vcc\n v_cndmask_b32 %5, %5, %8, vcc\n"
                         " v_cndmask_b32 %6, %6, %8, vcc\n v_cndmask_b32 %7, %7, %8, vcc"
                         : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(c) : "vcc");
        } else if (OP == 11) {   // the same with the VOP3 select reading an SGPR pair
            asm volatile("v_cmp_gt_i32_e64 s[12:13], %0, %8\n v_cndmask_b32_e64 %1, %1, %8, s[12:13]\n v_cndmask_b32_e64 %2, %2, %8, s[12:13]\n"
                         " v_cndmask_b32_e64 %3, %3, %8, s[12:13]\n v_cndmask_b32_e64 %4, %4, %8, s[12:13]\n v_cndmask_b32_e64 %5, %5, %8, s[12:13]\n"
                         " v_cndmask_b32_e64 %6, %6, %8, s[12:13]\n v_cndmask_b32_e64 %7, %7, %8, s[12:13]"
                         : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(c) : "s12", "s13");
            asm volatile("v_cmp_gt_i32_e64 s[12:13], %0, %8\n v_cndmask_b32_e64 %1, %1, %8, s[12:13]\n v_cndmask_b32_e64 %2, %2, %8, s[12:13]\n"
                         " v_cndmask_b32_e64 %3, %3, %8, s[12:13]\n v_cndmask_b32_e64 %4, %4, %8, s[12:13]\n v_cndmask_b32_e64 %5, %5, %8, s[12:13]\n"
                         " v_cndmask_b32_e64 %6, %6, %8, s[12:13]\n v_cndmask_b32_e64 %7, %7, %8, s[12:13]"
                         : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(c) : "s12", "s13");
            asm volatile("v_cmp_gt_i32_e64 s[12:13], %0, %8\n v_cndmask_b32_e64 %1, %1, %8, s[12:13]\n v_cndmask_b32_e64 %2, %2, %8, s[12:13]\n"
                         " v_cndmask_b32_e64 %3, %3, %8, s[12:13]\n v_cndmask_b32_e64 %4, %4, %8, s[12:13]\n v_cndmask_b32_e64 %5, %5, %8, s[12:13]\n"
                         " v_cndmask_b32_e64 %6, %6, %8, s[12:13]\n v_cndmask_b32_e64 %7, %7, %8, s[12:13]"
                         : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(c) : "s12", "s13");
            asm volatile("v_cmp_gt_i32_e64 s[12:13], %0, %8\n v_cndmask_b32_e64 %1, %1, %8, s[12:13]\n v_cndmask_b32_e64 %2, %2, %8, s[12:13]\n"
                         " v_cndmask_b32_e64 %3, %3, %8, s[12:13]\n v_cndmask_b32_e64 %4, %4, %8, s[12:13]\n v_cndmask_b32_e64 %5, %5, %8, s[12:13]\n"
                         " v_cndmask_b32_e64 %6, %6, %8, s[12:13]\n v_cndmask_b32_e64 %7, %7, %8, s[12:13]"
                         : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(c) : "s12", "s13");
        } else if (OP == 12) {   // one compare into VCC, then 7 VOP3 selects reading VCC
            asm volatile("v_cmp_gt_i32 vcc, %0, %8\n v_cndmask_b32_e64 %1, %1, %8, vcc\n v_cndmask_b32_e64 %2, %2, %8, vcc\n"
                         " v_cndmask_b32_e64 %3, %3, %8, vcc\n v_cndmask_b32_e64 %4, %4, %8, vcc\n v_cndmask_b32_e64 %5, %5, %8, vcc\n"
                         " v_cndmask_b32_e64 %6, %6, %8, vcc\n v_cndmask_b32_e64 %7, %7, %8, vcc"
                         : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(c) : "vcc");
            asm volatile("v_cmp_gt_i32 vcc, %0, %8\n v_cndmask_b32_e64 %1, %1, %8, vcc\n v_cndmask_b32_e64 %2, %2, %8, vcc\n"
                         " v_cndmask_b32_e64 %3, %3, %8, vcc\n v_cndmask_b32_e64 %4, %4, %8, vcc\n v_cndmask_b32_e64 %5, %5, %8, vcc\n"
                         " v_cndmask_b32_e64 %6, %6, %8, vcc\n v_cndmask_b32_e64 %7, %7, %8, vcc"
                         : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(c) : "vcc");
            asm volatile("v_cmp_gt_i32 vcc, %0, %8\n v_cndmask_b32_e64 %1, %1, %8, vcc\n v_cndmask_b32_e64 %2, %2, %8, vcc\n"
                         " v_cndmask_b32_e64 %3, %3, %8, vcc\n v_cndmask_b32_e64 %4, %4, %8, vcc\n v_cndmask_b32_e64 %5, %5, %8, vcc\n"
                         " v_cndmask_b32_e64 %6, %6, %8, vcc\n v_cndmask_b32_e64 %7, %7, %8, vcc"
                         : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(c) : "vcc");
            asm volatile("v_cmp_gt_i32 vcc, %0, %8\n v_cndmask_b32_e64 %1, %1, %8, vcc\n v_cndmask_b32_e64 %2, %2, %8, vcc\n"
                         " v_cndmask_b32_e64 %3, %3, %8, vcc\n v_cndmask_b32_e64 %4, %4, %8, vcc\n v_cndmask_b32_e64 %5, %5, %8, vcc\n"
                         " v_cndmask_b32_e64 %6, %6, %8, vcc\n v_cndmask_b32_e64 %7, %7, %8, vcc"
                         : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(c) : "vcc");
        } else if (OP == 13) {   // compare into VCC, one add between, then one VOP2 select reading VCC, 5 adds
            asm volatile("v_cmp_gt_i32 vcc, %0, %8\n v_add_u32 %1, %1, %8\n v_cndmask_b32 %2, %2, %8, vcc\n"
                         " v_add_u32 %3, %3, %8\n v_add_u32 %4, %4, %8\n v_add_u32 %5, %5, %8\n"
                         " v_add_u32 %6, %6, %8\n v_add_u32 %7, %7, %8"
                         : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(c) : "vcc");
            asm volatile("v_cmp_gt_i32 vcc, %0, %8\n v_add_u32 %1, %1, %8\n v_cndmask_b32 %2, %2, %8, vcc\n"
                         " v_add_u32 %3, %3, %8\n v_add_u32 %4, %4, %8\n v_add_u32 %5, %5, %8\n"
                         " v_add_u32 %6, %6, %8\n v_add_u32 %7, %7, %8"
                         : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(c) : "vcc");
            asm volatile("v_cmp_gt_i32 vcc, %0, %8\n v_add_u32 %1, %1, %8\n v_cndmask_b32 %2, %2, %8, vcc\n"
                         " v_add_u32 %3, %3, %8\n v_add_u32 %4, %4, %8\n v_add_u32 %5, %5, %8\n"
                         " v_add_u32 %6, %6, %8\n v_add_u32 %7, %7, %8"
                         : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(c) : "vcc");
            asm volatile("v_cmp_gt_i32 vcc, %0, %8\n v_add_u32 %1, %1, %8\n v_cndmask_b32 %2, %2, %8, vcc\n"
                         " v_add_u32 %3, %3, %8\n v_add_u32 %4, %4, %8\n v_add_u32 %5, %5, %8\n"
                         " v_add_u32 %6, %6, %8\n v_add_u32 %7, %7, %8"
                         : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(c) : "vcc");
        } else if (OP == 14) {   // 64-bit add pairs: v_add_co (writes VCC) + v_addc_co (reads it)
            asm volatile("v_add_co_u32 %0, vcc, %0, %8\n v_addc_co_u32 %1, vcc, %1, %8, vcc\n v_add_co_u32 %2, vcc, %2, %8\n v_addc_co_u32 %3, vcc, %3, %8, vcc\n"
                         " v_add_co_u32 %4, vcc, %4, %8\n v_addc_co_u32 %5, vcc, %5, %8, vcc\n v_add_co_u32 %6, vcc, %6, %8\n v_addc_co_u32 %7, vcc, %7, %8, vcc"
                         : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(c) : "vcc");
            asm volatile("v_add_co_u32 %0, vcc, %0, %8\n v_addc_co_u32 %1, vcc, %1, %8, vcc\n v_add_co_u32 %2, vcc, %2, %8\n v_addc_co_u32 %3, vcc, %3, %8, vcc\n"
                         " v_add_co_u32 %4, vcc, %4, %8\n v_addc_co_u32 %5, vcc, %5, %8, vcc\n v_add_co_u32 %6, vcc, %6, %8\n v_addc_co_u32 %7, vcc, %7, %8, vcc"
                         : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(c) : "vcc");
            asm volatile("v_add_co_u32 %0, vcc, %0, %8\n v_addc_co_u32 %1, vcc, %1, %8, vcc\n v_add_co_u32 %2, vcc, %2, %8\n v_addc_co_u32 %3, vcc, %3, %8, vcc\n"
                         " v_add_co_u32 %4, vcc, %4, %8\n v_addc_co_u32 %5, vcc, %5, %8, vcc\n v_add_co_u32 %6, vcc, %6, %8\n v_addc_co_u32 %7, vcc, %7, %8, vcc"
                         : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(c) : "vcc");
            asm volatile("v_add_co_u32 %0, vcc, %0, %8\n v_addc_co_u32 %1, vcc, %1, %8, vcc\n v_add_co_u32 %2, vcc, %2, %8\n v_addc_co_u32 %3, vcc, %3, %8, vcc\n"
                         " v_add_co_u32 %4, vcc, %4, %8\n v_addc_co_u32 %5, vcc, %5, %8, vcc\n v_add_co_u32 %6, vcc, %6, %8\n v_addc_co_u32 %7, vcc, %7, %8, vcc"
                         : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(c) : "vcc");
        } else if (OP == 5) {   // 32 plain adds (reference)
#define X(i) asm volatile("v_add_u32 %0, %0, %1" : "+v"(a##i) : "v"(c));
            REP4(R8(X))
#undef X
        }
    }
    out[blockIdx.x * 64 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

template <int OP>
static void run(const char* name, uint32_t* out) {
    const int wps = 5, nwg = 256 * 4 * wps;
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    k<OP><<<nwg, 64>>>(1, out);
    hipEventRecord(e0);
    k<OP><<<nwg, 64>>>(2, out);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    printf("%-44s %.3f ms = %.2f SIMD-cycles per instruction at 2.4 GHz\n", name, ms,
           ms * 1e-3 * 2.4e9 / ((double)ITER * 32 * wps));
    hipEventDestroy(e0);
    hipEventDestroy(e1);
}

int main() {
    uint32_t* out;
    hipMalloc(&out, sizeof(uint32_t) * 256 * 4 * 5 * 64);
    run<5>("v_add_u32 (reference)", out);
    run<0>("v_cndmask_b32 vcc, VCC never written", out);
    run<1>("v_cndmask_b32 vcc, VCC set by s_mov before", out);
    run<2>("v_cndmask_b32 vcc, VCC set by v_cmp before", out);
    run<3>("v_cmp_e32 vcc + v_cndmask_b32_e32 vcc pairs", out);
    run<4>("v_cmp_e64 s[12:13] + v_cndmask_e64 pairs", out);
    run<6>("v_add_u32 + s_nop 0 (per VALU)", out);
    run<7>("v_add_u32 + s_nop 1 (per VALU)", out);
    run<8>("s_nop 1 + v_add_u32_dpp (per VALU)", out);
    run<9>("v_add_u32_dpp, 8 chains interleaved", out);
    run<10>("v_cmp_e32 vcc + 7 v_cndmask_b32_e32 vcc", out);
    run<11>("v_cmp_e64 s[12:13] + 7 v_cndmask_e64 s[12:13]", out);
    run<12>("v_cmp_e32 vcc + 7 v_cndmask_b32_e64 vcc", out);
    run<13>("v_cmp vcc, add, v_cndmask_e32 vcc, 5 adds", out);
    run<14>("v_add_co_u32 vcc + v_addc_co_u32 vcc pairs", out);
    hipFree(out);
    return 0;
}
