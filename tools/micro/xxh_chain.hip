// Microbenchmark (dev only): single-stream XXH32 accumulator chain variants
// on gfx950.  Wave j of a 4-wave workgroup runs accumulator j.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <vector>
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
constexpr uint32_t P1 = 2654435761u, P2 = 2246822519u;

__device__ __forceinline__ uint32_t vround(uint32_t acc, uint32_t in) {
    uint32_t x = acc + in * P2; x = (x << 13) | (x >> 19); return x * P1; }
__device__ __forceinline__ uint32_t s_mulp2(uint32_t x) { uint32_t r; asm("s_mul_i32 %0, %1, 0x85ebca77" : "=s"(r) : "s"(x)); return r; }
__device__ __forceinline__ uint32_t s_chain5(uint32_t acc, uint32_t px) {
    uint32_t r, t;
    asm("s_add_u32 %0, %2, %3\n\ts_lshl_b32 %1, %0, 13\n\ts_lshr_b32 %0, %0, 19\n\ts_or_b32 %0, %0, %1\n\ts_mul_i32 %0, %0, 0x9e3779b1"
        : "=&s"(r), "=&s"(t) : "s"(acc), "s"(px) : "scc");
    return r; }
__device__ __forceinline__ uint32_t s_chain64(uint32_t acc, uint32_t px) {
    uint64_t d; uint32_t r;
    asm("s_add_u32 %0, %2, %3\n\ts_add_u32 %1, %2, %3" : "=&s"(*((uint32_t*)&d)), "=&s"(*((uint32_t*)&d+1)) : "s"(acc), "s"(px) : "scc");
    asm("s_lshl_b64 %0, %1, 13" : "=s"(d) : "s"(d) : "scc");
    asm("s_mul_i32 %0, %1, 0x9e3779b1" : "=s"(r) : "s"((uint32_t)(d >> 32)));
    return r; }
__device__ __forceinline__ uint32_t v_chain(uint32_t acc, uint32_t px) {   // VALU: add, alignbit, mul_lo
    uint32_t x = acc + px; x = __builtin_amdgcn_alignbit(x, x, 19); return x * P1; }

// MODE 0: SALU chain5, VMEM 1 KiB loads 4 deep + readlane
// MODE 1: SALU chain64, same loads
// MODE 2: VALU chain (uniform), same loads, word via readlane
// MODE 3: compute only SALU chain5 (px synthetic)
// MODE 4: compute only VALU chain
template <int MODE>
__global__ __launch_bounds__(256) void k(const uint8_t* __restrict__ src, int64_t len, uint32_t* out) {
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x / 64), lane = threadIdx.x % 64;
    uint32_t v = 0x12345 + wave;
    const int64_t nk = len / 1024;
    if (MODE == 5) {
        // diagonal chain: at step t lane t holds stripe t's word; the
        // accumulator moves one lane up per step (DPP wave_ror:1)
        constexpr int D = 4;
        u32x4 buf[D];
#pragma unroll
        for (int d = 0; d < D; ++d) { buf[d] = u32x4{0,0,0,0}; if (d < nk) __builtin_memcpy(&buf[d], src + d * 1024 + 16 * lane, 16); }
        uint32_t acc = v;
        for (int64_t c = 0; c < nk; c += D) {
#pragma unroll
            for (int d = 0; d < D; ++d) {
                const uint32_t w = wave == 0 ? buf[d].x : wave == 1 ? buf[d].y : wave == 2 ? buf[d].z : buf[d].w;
                const uint32_t pw = w * P2;
                if (c + d + D < nk) __builtin_memcpy(&buf[d], src + (c + d + D) * 1024 + 16 * lane, 16);
#pragma unroll
                for (int t = 0; t < 64; ++t) {
                    uint32_t x = (uint32_t)__builtin_amdgcn_update_dpp((int)0, (int)acc, 0x13C, 0xF, 0xF, false) + pw;
                    x = __builtin_amdgcn_alignbit(x, x, 19);
                    acc = x * P1;
                }
            }
        }
        v = __builtin_amdgcn_readlane(acc, 63);
    } else if (MODE >= 3) {
        uint32_t px = wave * 7 + 1;
        for (int64_t c = 0; c < nk; ++c) {
#pragma unroll
            for (int t = 0; t < 64; ++t) {
                if (MODE == 3) v = s_chain5(v, px + t); else v = v_chain(v, px + t);
            }
        }
    } else {
        constexpr int D = 4;
        u32x4 buf[D];
#pragma unroll
        for (int d = 0; d < D; ++d) { buf[d] = u32x4{0,0,0,0}; if (d < nk) __builtin_memcpy(&buf[d], src + d * 1024 + 16 * lane, 16); }
        for (int64_t c = 0; c < nk; c += D) {
#pragma unroll
            for (int d = 0; d < D; ++d) {
                const uint32_t w = wave == 0 ? buf[d].x : wave == 1 ? buf[d].y : wave == 2 ? buf[d].z : buf[d].w;
                const uint32_t pw = w * P2;   // VALU, 64 stripes at once
                if (c + d + D < nk) __builtin_memcpy(&buf[d], src + (c + d + D) * 1024 + 16 * lane, 16);
#pragma unroll
                for (int t = 0; t < 64; ++t) {
                    const uint32_t px = __builtin_amdgcn_readlane(pw, t);
                    if (MODE == 0) v = s_chain5(v, px); else if (MODE == 1) v = s_chain64(v, px); else v = v_chain(v, px);
                }
            }
        }
    }
    if (lane == 0) out[wave] = v;
}

template <int M> float run(const uint8_t* d, int64_t len, uint32_t* o) {
    hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
    hipLaunchKernelGGL(k<M>, dim3(1), dim3(256), 0, 0, d, len, o);
    hipEventRecord(a); hipLaunchKernelGGL(k<M>, dim3(1), dim3(256), 0, 0, d, len, o); hipEventRecord(b);
    hipEventSynchronize(b); float ms; hipEventElapsedTime(&ms, a, b); return ms;
}
int main() {
    const int64_t len = 256ll << 20;
    uint8_t* d; uint32_t* o; hipMalloc(&d, len); hipMalloc(&o, 64); hipMemset(d, 7, len);
    printf("mode0 SALU5+vmem  %.3f GB/s\n", len / run<0>(d, len, o) / 1e6);
    printf("mode1 SALU64+vmem %.3f GB/s\n", len / run<1>(d, len, o) / 1e6);
    printf("mode2 VALU+vmem   %.3f GB/s\n", len / run<2>(d, len, o) / 1e6);
    printf("mode5 VALU diag   %.3f GB/s\n", len / run<5>(d, len, o) / 1e6);
    printf("mode3 SALU5 only  %.3f GB/s\n", len / run<3>(d, len, o) / 1e6);
    printf("mode4 VALU only   %.3f GB/s\n", len / run<4>(d, len, o) / 1e6);
    return 0;
}
