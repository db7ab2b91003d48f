// Microbenchmark (dev only): issue cost of the integer VALU instructions the
// row executor is made of, on gfx950, by occupancy.  Every wave of W waves per
// SIMD runs ITER x 32 independent instructions of one kind (8 accumulators,
// each written every 8th instruction); the kernel's HIP-event time and the
// waves' own s_memtime spans give SIMD-cycles per wave-instruction.
//   hipcc --offload-arch=gfx950 -O3 tools/micro/valu_rate.hip -o /tmp/valu_rate
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

constexpr int ITER = 2048;

#define R8(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)
#define REP4(S) S S S S

template <int OP>
__global__ __launch_bounds__(64) void k(uint32_t seed, uint32_t* out, unsigned long long* span) {
    uint32_t a0 = seed ^ threadIdx.x, a1 = a0 * 3, a2 = a0 * 5, a3 = a0 * 7, a4 = a0 * 9, a5 = a0 * 11, a6 = a0 * 13,
             a7 = a0 * 15;
    uint64_t b0 = a0, b1 = a1, b2 = a2, b3 = a3;
    const uint32_t c = seed * 0x9E3779B1u + 1;
    const unsigned long long t0 = clock64();
    for (int it = 0; it < ITER; ++it) {
        if (OP == 0) {
#define X(i) asm volatile("v_add_u32 %0, %0, %1" : "+v"(a##i) : "v"(c));
            REP4(R8(X))
#undef X
        } else if (OP == 1) {
#define X(i) asm volatile("v_perm_b32 %0, %0, %1, %1" : "+v"(a##i) : "v"(c));
            REP4(R8(X))
#undef X
        } else if (OP == 2) {
#define X(i) asm volatile("v_alignbyte_b32 %0, %0, %1, %1" : "+v"(a##i) : "v"(c));
            REP4(R8(X))
#undef X
        } else if (OP == 3) {
#define X(i) asm volatile("v_mov_b32_dpp %0, %0 row_shr:1 row_mask:0xf bank_mask:0xf" : "+v"(a##i));
            REP4(R8(X))
#undef X
        } else if (OP == 4) {
#define X(i) asm volatile("v_max_i32_dpp %0, %0, %0 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1" : "+v"(a##i));
            REP4(R8(X))
#undef X
        } else if (OP == 5) {
#define X(i) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(a##i) : "v"(c) : "vcc");
            REP4(R8(X))
#undef X
        } else if (OP == 6) {
#define Y(i) asm volatile("v_lshlrev_b64 %0, 1, %0" : "+v"(b##i));
            REP4(REP4(Y(0) Y(1)) REP4(Y(2) Y(3)))
#undef Y
        } else if (OP == 7) {
#define X(i) asm volatile("v_bfe_u32 %0, %0, 3, 5" : "+v"(a##i));
            REP4(R8(X))
#undef X
        } else if (OP == 8) {
#define X(i) asm volatile("v_cmp_gt_i32 vcc, %0, %1" ::"v"(a##i), "v"(c) : "vcc");
            REP4(R8(X))
#undef X
        } else if (OP == 9) {
#define X(i) asm volatile("v_mad_u32_u24 %0, %0, %1, %1" : "+v"(a##i) : "v"(c));
            REP4(R8(X))
#undef X
        } else if (OP == 10) {
#define X(i) asm volatile("v_lshl_add_u32 %0, %0, 2, %1" : "+v"(a##i) : "v"(c));
            REP4(R8(X))
#undef X
        } else if (OP == 11) {
#define X(i) asm volatile("v_add_co_u32 %0, vcc, %0, %1" : "+v"(a##i) : "v"(c) : "vcc");
            REP4(R8(X))
#undef X
        } else if (OP == 12) {   // a 50/50 mix of v_add_u32 and v_and_b32 with an SGPR-free VOP2
#define X(i) asm volatile("v_add_u32 %0, %0, %1\n v_and_b32 %0, %0, %1" : "+v"(a##i) : "v"(c));
            REP4(X(0) X(1) X(2) X(3))
#undef X
        } else if (OP == 14) {   // the select form the compiler emits: VOP3 with an SGPR-pair mask
#define X(i) asm volatile("v_cndmask_b32_e64 %0, %0, %1, s[10:11]" : "+v"(a##i) : "v"(c) : "s10", "s11");
            REP4(R8(X))
#undef X
        } else if (OP == 15) {   // v_add_u32 in its VOP3 encoding
#define X(i) asm volatile("v_add_u32_e64 %0, %0, %1" : "+v"(a##i) : "v"(c));
            REP4(R8(X))
#undef X
        } else if (OP == 16) {
#define X(i) asm volatile("v_or3_b32 %0, %0, %1, %1" : "+v"(a##i) : "v"(c));
            REP4(R8(X))
#undef X
        } else if (OP == 17) {   // compare to an SGPR pair, then select on it (pairs)
#define X(i) asm volatile("v_cmp_gt_i32_e64 s[12:13], %0, %1\n v_cndmask_b32_e64 %0, %0, %1, s[12:13]" : "+v"(a##i) : "v"(c) : "s12", "s13");
            REP4(X(0) X(1) X(2) X(3))
#undef X
        } else if (OP == 18) {   // v_and_b32 (VOP2)
#define X(i) asm volatile("v_and_b32 %0, %0, %1" : "+v"(a##i) : "v"(c));
            REP4(R8(X))
#undef X
        } else if (OP == 13) {   // ds_read-free scalar op mix: s_add per 2 VALU (SALU co-issue)
#define X(i) asm volatile("v_add_u32 %0, %0, %1\n s_add_u32 s40, s40, 1" : "+v"(a##i) : "v"(c) : "s40", "scc");
            REP4(R8(X))
#undef X
        }
    }
    const unsigned long long t1 = clock64();
    out[blockIdx.x * 64 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7 ^ (uint32_t)(b0 ^ b1 ^ b2 ^ b3);
    if (threadIdx.x == 0) span[blockIdx.x] = t1 - t0;
}

template <int OP>
static void run(const char* name, int wps, uint32_t* out, unsigned long long* span, unsigned long long* hspan) {
    const int nwg = 256 * 4 * wps;   // wps waves per SIMD on 256 CUs
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    k<OP><<<nwg, 64>>>(1, out, span);
    hipEventRecord(e0);
    k<OP><<<nwg, 64>>>(2, out, span);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    hipMemcpy(hspan, span, sizeof(unsigned long long) * nwg, hipMemcpyDeviceToHost);
    double avg = 0;
    for (int i = 0; i < nwg; ++i) avg += (double)hspan[i];
    avg /= nwg;
    const double instrs = (double)ITER * 32;   // per wave
    // s_memtime span per wave / (instructions per wave x waves per SIMD) = cycles per instruction per SIMD
    const double cyc_span = avg / (instrs * wps);
    const double cyc_evt = ms * 1e-3 * 2.4e9 / (instrs * wps);
    printf("%-22s waves/SIMD %d  span %.2f cyc/instr  event %.3f ms = %.2f cyc/instr at 2.4 GHz\n", name, wps, cyc_span,
           ms, cyc_evt);
    hipEventDestroy(e0);
    hipEventDestroy(e1);
}

int main() {
    uint32_t* out;
    unsigned long long* span;
    hipMalloc(&out, sizeof(uint32_t) * 256 * 4 * 8 * 64);
    hipMalloc(&span, sizeof(unsigned long long) * 256 * 4 * 8);
    static unsigned long long hspan[256 * 4 * 8];
    for (int w : {2, 5, 8}) {
        run<0>("v_add_u32", w, out, span, hspan);
        run<1>("v_perm_b32", w, out, span, hspan);
        run<2>("v_alignbyte_b32", w, out, span, hspan);
        run<3>("v_mov_b32_dpp", w, out, span, hspan);
        run<4>("v_max_i32_dpp", w, out, span, hspan);
        run<5>("v_cndmask_b32", w, out, span, hspan);
        run<6>("v_lshlrev_b64", w, out, span, hspan);
        run<7>("v_bfe_u32", w, out, span, hspan);
        run<8>("v_cmp_gt_i32 (vcc)", w, out, span, hspan);
        run<9>("v_mad_u32_u24", w, out, span, hspan);
        run<10>("v_lshl_add_u32", w, out, span, hspan);
        run<11>("v_add_co_u32", w, out, span, hspan);
        run<12>("add+and", w, out, span, hspan);
        run<13>("add + s_add", w, out, span, hspan);
        run<14>("v_cndmask_b32_e64 sgpr", w, out, span, hspan);
        run<15>("v_add_u32_e64", w, out, span, hspan);
        run<16>("v_or3_b32", w, out, span, hspan);
        run<17>("v_cmp_e64 + v_cndmask", w, out, span, hspan);
        run<18>("v_and_b32", w, out, span, hspan);
    }
    hipFree(out);
    hipFree(span);
    return 0;
}
