// Dev check (r05ap): VOP3 select helpers on a ballot mask (sel_m / sel2_m /
// sel4_m, the round-5 attempt to avoid back-to-back VOP2 selects reading VCC,
// tools/micro/cndmask_rate.hip) against plain ternaries, in full and
// divergent exec.  Each asm starts and ends with `s_nop 1`: a VALU write of
// the mask SGPR and a VALU reading it as a lane mask need two wait states,
// which the compiler inserts for its own instructions only.  All cases
// matched; in the row decoder the helpers were 0.7 % slower (r05ar) and one
// site decoded wrong bytes (r05aq), so the decoder keeps plain ternaries.
// Prints the mismatch count per case (0 expected).
//   hipcc --offload-arch=gfx950 -O3 tools/micro/sel_check.hip -o tools/micro/sel_check.bin
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
#define LZ4M_MASK(c) ((uint64_t)__ballot(c))
__device__ __forceinline__ uint32_t sel_m(uint64_t m, bool, uint32_t a, uint32_t b) {
    uint32_t r;
    asm volatile("s_nop 1\n\tv_cndmask_b32_e64 %0, %1, %2, %3\n\ts_nop 1" : "=v"(r) : "v"(b), "v"(a), "s"(m));
    return r;
}
__device__ __forceinline__ void sel2_m(uint64_t m, bool, uint32_t a0, uint32_t b0, uint32_t a1, uint32_t b1,
                                       uint32_t& r0, uint32_t& r1) {
    asm volatile("s_nop 1\n\tv_cndmask_b32_e64 %0, %2, %4, %6\n\tv_cndmask_b32_e64 %1, %3, %5, %6\n\ts_nop 1"
                 : "=&v"(r0), "=&v"(r1)
                 : "v"(b0), "v"(b1), "v"(a0), "v"(a1), "s"(m));
}
__device__ __forceinline__ u32x4 sel4_m(uint64_t m, bool, u32x4 a, u32x4 b) {
    uint32_t r0, r1, r2, r3;
    asm volatile("s_nop 1\n\tv_cndmask_b32_e64 %0, %4, %8, %12\n\tv_cndmask_b32_e64 %1, %5, %9, %12\n\t"
                 "v_cndmask_b32_e64 %2, %6, %10, %12\n\tv_cndmask_b32_e64 %3, %7, %11, %12\n\ts_nop 1"
                 : "=&v"(r0), "=&v"(r1), "=&v"(r2), "=&v"(r3)
                 : "v"(b.x), "v"(b.y), "v"(b.z), "v"(b.w), "v"(a.x), "v"(a.y), "v"(a.z), "v"(a.w), "s"(m));
    return u32x4{r0, r1, r2, r3};
}

__global__ __launch_bounds__(64) void k(const uint32_t* in, uint32_t* bad) {
    const uint32_t t = blockIdx.x * 64 + threadIdx.x;
    const uint32_t a = in[4 * t], b = in[4 * t + 1], x = in[4 * t + 2], y = in[4 * t + 3];
    uint32_t nb[6] = {0, 0, 0, 0, 0, 0};
    // 1: one select, full exec
    {
        const bool c = (x & 4) != 0;
        const uint32_t r = sel_m(LZ4M_MASK(c), c, a, b);
        nb[0] += r != (c ? a : b);
    }
    // 2: four selects on one mask, full exec
    {
        const bool c = x < y;
        const u32x4 r = sel4_m(LZ4M_MASK(c), c, u32x4{a, b, x, y}, u32x4{y, x, b, a});
        nb[1] += (r.x != (c ? a : y)) + (r.y != (c ? b : x)) + (r.z != (c ? x : b)) + (r.w != (c ? y : a));
    }
    // 3: two selects
    {
        const bool c = (a ^ y) & 1;
        uint32_t r0, r1;
        sel2_m(LZ4M_MASK(c), c, a, b, x, y, r0, r1);
        nb[2] += (r0 != (c ? a : b)) + (r1 != (c ? x : y));
    }
    // 4: divergent: a select inside a branch taken by some lanes
    if ((x % 3) != 0) {
        const bool c = (y & 2) != 0;
        const u32x4 r = sel4_m(LZ4M_MASK(c), c, u32x4{a, b, x, y}, u32x4{y, x, b, a});
        nb[3] += (r.x != (c ? a : y)) + (r.y != (c ? b : x)) + (r.z != (c ? x : b)) + (r.w != (c ? y : a));
    }
    // 5: if / else with the same select in both parts
    uint32_t r5;
    const bool c5 = (b & 8) != 0;
    if (a & 1) {
        r5 = sel_m(LZ4M_MASK(c5), c5, x, y) + 1;
    } else {
        r5 = sel_m(LZ4M_MASK(c5), c5, x, y) + 2;
    }
    nb[4] += r5 != (c5 ? x : y) + ((a & 1) ? 1 : 2);
    // 6: chained, as dword32_tree
    {
        const uint32_t q = x & 7;
        const bool q1 = q & 1, q2 = q & 2, q4 = q & 4;
        const uint64_t m1 = LZ4M_MASK(q1), m2 = LZ4M_MASK(q2), m4 = LZ4M_MASK(q4);
        const u32x4 l = sel4_m(m1, q1, u32x4{a, b, x, y}, u32x4{b, x, y, a});
        const u32x4 h = sel4_m(m1, q1, u32x4{x, y, a, 0u}, u32x4{y, a, b, x});
        const u32x4 tt = sel4_m(m2, q2, u32x4{l.w, l.y, h.w, h.y}, u32x4{l.z, l.x, h.z, h.x});
        uint32_t lo, hi;
        sel2_m(m4, q4, tt.x, tt.y, tt.z, tt.w, lo, hi);
        const uint32_t L0 = q1 ? a : b, L1 = q1 ? b : x, L2 = q1 ? x : y, L3 = q1 ? y : a;
        const uint32_t H0 = q1 ? x : y, H1 = q1 ? y : a, H2 = q1 ? a : b, H3 = q1 ? 0u : x;
        const uint32_t elo = q4 ? (q2 ? L3 : L2) : (q2 ? L1 : L0), ehi = q4 ? (q2 ? H3 : H2) : (q2 ? H1 : H0);
        nb[5] += (lo != elo) + (hi != ehi);
    }
    for (int i = 0; i < 6; ++i) atomicAdd(&bad[i], nb[i]);
}

int main() {
    const int n = 64 * 4096;
    uint32_t* h = new uint32_t[4 * n];
    uint32_t s = 12345;
    for (int i = 0; i < 4 * n; ++i) {
        s = s * 1664525u + 1013904223u;
        h[i] = s ^ (s >> 13);
    }
    uint32_t *din, *dbad;
    hipMalloc(&din, 16 * n);
    hipMalloc(&dbad, 64);
    hipMemcpy(din, h, 16 * n, hipMemcpyHostToDevice);
    hipMemset(dbad, 0, 64);
    k<<<n / 64, 64>>>(din, dbad);
    uint32_t bad[6];
    hipMemcpy(bad, dbad, 24, hipMemcpyDeviceToHost);
    const char* names[6] = {"sel_m full exec", "sel4_m full exec", "sel2_m full exec", "sel4_m divergent",
                            "sel_m if/else", "dword32_tree chain"};
    for (int i = 0; i < 6; ++i) printf("%-20s mismatches %u\n", names[i], bad[i]);
    return 0;
}
