// lz4m_xxh32.hip -- XXH32 for MI355X (gfx950).
//
// Restates lz4libs/xxhash.c:263-416 (one-shot XXH32) and the streaming
// digest it equals over a whole buffer (xxhash.c:437-554; total length taken
// mod 2^32, xxhash.c:464).
//
// Batch kernel: one quad (4 lanes, one per accumulator) per item (block
// checksums, lz4frame.c:846/1819; config 5's root consumer).
// Long kernel: one wavefront for a single buffer (content checksum,
// lz4frame.c:1042/1171).  XXH32's four accumulators are serial recurrences
// with no associative combine: one wave per
// accumulator, the chain stepping diagonally through the lanes.
#include "lz4m_common.h"
#include "../../include/lz4m.h"
#include "lz4m_xxh32_dev.h"

namespace lz4m {

// One quad per item (xxh32_quad_acc): 16 items per 64-lane workgroup, so a
// batch of n items occupies n / 16 waves of the chip (config 5's 4 096-item
// pages: 256 waves, one per CU), each lane streaming its accumulator's words
// with 2 x kXQ loads in flight.
__global__ __launch_bounds__(64) void xxh32_batch_kernel(const uint8_t* __restrict__ src,
                                                         const int64_t* __restrict__ off,
                                                         const int64_t* __restrict__ len, uint32_t seed,
                                                         uint32_t* __restrict__ out, int64_t n) {
    const uint32_t l = threadIdx.x, a = l & 3u;
    const int64_t i = (int64_t)blockIdx.x * 16 + (l >> 2);
    const bool live = i < n;
    const int64_t L = live ? len[i] : 0;
    const uint8_t* p = src + (live ? off[i] : 0);
    const uint32_t n16 = (uint32_t)(L >> 4);
    const uint32_t steps = wave_max_u32(n16);
    // lanes with no full stripe point at an item that has one (never read past it)
    const uint64_t has = __ballot(n16 > 0);
    const uint8_t* pv = n16 > 0 ? p : (has ? (const uint8_t*)readlane64((int64_t)(uintptr_t)p, __builtin_ctzll(has)) : p);
    const uint32_t v = xxh32_quad_acc(pv, n16, steps, seed, a);
    const uint32_t h = xxh32_quad_finish(v, p, L, seed);
    if (live && a == 0) out[i] = h;
}

// Single-buffer XXH32: XXH32's four accumulators are independent serial
// recurrences (xxhash.c:492-497), so wave j of a 4-wave workgroup (one wave
// per SIMD) runs accumulator j alone: v = rotl(v + x * P2, 13) * P1 over
// words j, j + 4, j + 8, ...  The wave loads 1 KiB per instruction (lane l
// holds stripe l of the chunk, four chunks in flight) and computes x * P2 for
// all 64 stripes at once; the dependent chain then runs "diagonally": at
// step t the accumulator sits in lane t, which holds stripe t's word, and a
// DPP wave rotate (wave_ror:1, folded into the add) moves it one lane up per
// step.  Each step is three dependent VALU instructions (add, alignbit,
// mul) with no v_readlane.  16 KiB of loads stay in flight.  Measured
// 1.70 GB/s on 4 GiB (MI355X); the serial chain is the bound (a scalar-unit
// version ran at 0.47 GB/s; rotating the words to lane 0 instead of the
// accumulator, 1.44 GB/s).
__global__ __launch_bounds__(256) void xxh32_long_kernel(const uint8_t* __restrict__ src, int64_t len, uint32_t seed,
                                                         uint32_t* __restrict__ out) {
    __shared__ uint32_t accs[4];
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
    const uint32_t lane = threadIdx.x % kWave;
    const uint32_t init[4] = {seed + kP1 + kP2, seed + kP2, seed, seed - kP1};
    uint32_t acc = wave == 0 ? init[0] : wave == 1 ? init[1] : wave == 2 ? init[2] : init[3];
    constexpr int64_t kChunk = 16 * kWave;
    constexpr int kD = 16;   // 16 KiB in flight: HBM latency hides behind 1024 chain steps
    const int64_t nk = len / kChunk;
    u32x4 buf[kD];
#pragma unroll
    for (int d = 0; d < kD; ++d) {
        buf[d] = u32x4{0, 0, 0, 0};
        if (d < nk) buf[d] = ld16(src + d * kChunk + 16 * lane);
    }
    for (int64_t c = 0; c < nk; c += kD) {
#pragma unroll
        for (int d = 0; d < kD; ++d) {
            if (c + d < nk) {
                const u32x4 b = buf[d];
                const uint32_t w = wave == 0 ? b.x : wave == 1 ? b.y : wave == 2 ? b.z : b.w;
                const uint32_t pw = w * kP2;
                if (c + d + kD < nk) buf[d] = ld16(src + (c + d + kD) * kChunk + 16 * lane);
#pragma unroll
                for (int t = 0; t < kWave; ++t) {
                    uint32_t x = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)acc, 0x13C, 0xF, 0xF, false) + pw;
                    x = __builtin_amdgcn_alignbit(x, x, 19);   // rotl 13
                    acc = x * kP1;
                }
            }
        }
    }
    uint32_t v = (uint32_t)__builtin_amdgcn_readlane((int)acc, kWave - 1);
    const int64_t n16 = len / 16;
    for (int64_t s = nk * kWave; s < n16; ++s) v = xround(v, ld32(src + 16 * s + 4 * wave));
    if (lane == 0) accs[wave] = v;
    __syncthreads();
    if (threadIdx.x == 0) {
        const int64_t q = n16 * 16;
        uint32_t h = len >= 16 ? rotl32(accs[0], 1) + rotl32(accs[1], 7) + rotl32(accs[2], 12) + rotl32(accs[3], 18)
                               : seed + kP5;
        h += (uint32_t)len;
        out[0] = xfinish(h, src + q, (int)(len - q));
    }
}

}  // namespace lz4m

using namespace lz4m;

extern "C" int lz4m_xxh32_batch(const uint8_t* d_src, const int64_t* d_off, const int64_t* d_len, uint32_t seed,
                                uint32_t* d_out, int64_t n, lz4m_stream_t stream) {
    if (n < 0) return LZ4M_EINVAL;
    if (n == 0) return 0;
    hipLaunchKernelGGL(xxh32_batch_kernel, dim3((uint32_t)((n + 15) / 16)), dim3(64), 0, (hipStream_t)stream,
                       d_src, d_off, d_len, seed, d_out, n);
    return (int)hipGetLastError();
}

extern "C" int lz4m_xxh32_long(const uint8_t* d_src, int64_t len, uint32_t seed, uint32_t* d_out,
                               lz4m_stream_t stream) {
    if (len < 0) return LZ4M_EINVAL;
    hipLaunchKernelGGL(xxh32_long_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream, d_src, len, seed, d_out);
    return (int)hipGetLastError();
}
