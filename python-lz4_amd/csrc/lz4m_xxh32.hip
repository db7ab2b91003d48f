// lz4m_xxh32.hip -- XXH32 for MI355X (gfx950).
//
// Restates lz4libs/xxhash.c:263-416 (one-shot XXH32) and the streaming
// digest it equals over a whole buffer (xxhash.c:437-554; total length taken
// mod 2^32, xxhash.c:464).
//
// Batch kernel: one lane per item (block checksums, lz4frame.c:846/1819);
// each lane streams its item in 16-byte stripes.
// Long kernel: one wavefront for a single buffer (content checksum,
// lz4frame.c:1042/1171).  XXH32's four accumulators are serial recurrences
// with no associative combine, so the wave only
// parallelises the loads: all 64 lanes fetch 1 KiB per instruction, two
// batches in flight, and the four rounds per stripe run on the scalar unit
// from v_readlane'd words.
#include "lz4m_common.h"
#include "../../include/lz4m.h"
#include "lz4m_xxh32_dev.h"

namespace lz4m {

__global__ __launch_bounds__(256) void xxh32_batch_kernel(const uint8_t* __restrict__ src,
                                                          const int64_t* __restrict__ off,
                                                          const int64_t* __restrict__ len, uint32_t seed,
                                                          uint32_t* __restrict__ out, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = xxh32_lane(src + off[i], len[i], seed);
}

// Single-buffer XXH32 on one wavefront.
__global__ __launch_bounds__(64) void xxh32_long_kernel(const uint8_t* __restrict__ src, int64_t len, uint32_t seed,
                                                        uint32_t* __restrict__ out) {
    const uint32_t lane = threadIdx.x;
    uint32_t v1 = seed + kP1 + kP2, v2 = seed + kP2, v3 = seed, v4 = seed - kP1;
    constexpr int64_t kChunk = 16 * kWave;   // 1 KiB per wave load
    const int64_t nfull = len / kChunk;      // whole 1 KiB chunks
    u32x4 cur = u32x4{0, 0, 0, 0}, nxt = u32x4{0, 0, 0, 0};
    if (nfull > 0) cur = ld16(src + 16 * lane);
    for (int64_t c = 0; c < nfull; ++c) {
        if (c + 1 < nfull) nxt = ld16(src + (c + 1) * kChunk + 16 * lane);
#pragma unroll
        for (int t = 0; t < kWave; ++t) {
            v1 = xround(v1, (uint32_t)__builtin_amdgcn_readlane((int)cur.x, t));
            v2 = xround(v2, (uint32_t)__builtin_amdgcn_readlane((int)cur.y, t));
            v3 = xround(v3, (uint32_t)__builtin_amdgcn_readlane((int)cur.z, t));
            v4 = xround(v4, (uint32_t)__builtin_amdgcn_readlane((int)cur.w, t));
        }
        cur = nxt;
    }
    if (lane == 0) {
        int64_t q = nfull * kChunk;
        for (; q + 16 <= len; q += 16) {
            const u32x4 w = ld16(src + q);
            v1 = xround(v1, w.x);
            v2 = xround(v2, w.y);
            v3 = xround(v3, w.z);
            v4 = xround(v4, w.w);
        }
        uint32_t h = len >= 16 ? rotl32(v1, 1) + rotl32(v2, 7) + rotl32(v3, 12) + rotl32(v4, 18) : seed + kP5;
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
    hipLaunchKernelGGL(xxh32_batch_kernel, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                       d_src, d_off, d_len, seed, d_out, n);
    return (int)hipGetLastError();
}

extern "C" int lz4m_xxh32_long(const uint8_t* d_src, int64_t len, uint32_t seed, uint32_t* d_out,
                               lz4m_stream_t stream) {
    if (len < 0) return LZ4M_EINVAL;
    hipLaunchKernelGGL(xxh32_long_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, d_src, len, seed, d_out);
    return (int)hipGetLastError();
}
