// lz4m_xxh32_dev.h -- device XXH32 (xxhash.c:263-416), shared by kernels.
#pragma once
#include "lz4m_common.h"

namespace lz4m {

constexpr uint32_t kP1 = 2654435761u, kP2 = 2246822519u, kP3 = 3266489917u, kP4 = 668265263u,
                   kP5 = 374761393u;   // xxhash.c:263-267

__device__ __forceinline__ uint32_t rotl32(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }
__device__ __forceinline__ uint32_t xround(uint32_t acc, uint32_t in) { return rotl32(acc + in * kP2, 13) * kP1; }

// tail + avalanche (xxhash.c:278-348) over len (< 16) bytes at p
__device__ __forceinline__ uint32_t xfinish(uint32_t h, const uint8_t* p, int len) {
    while (len >= 4) {
        h = rotl32(h + ld32(p) * kP3, 17) * kP4;
        p += 4;
        len -= 4;
    }
    while (len > 0) {
        h = rotl32(h + (uint32_t)(*p++) * kP5, 11) * kP1;
        --len;
    }
    h ^= h >> 15;
    h *= kP2;
    h ^= h >> 13;
    h *= kP3;
    h ^= h >> 16;
    return h;
}

// The stripes of one item are a serial chain per accumulator; a lane keeps
// 2 x 8 stripes (256 bytes) of its item in flight so that a batch of few,
// long items (config 5's pages: 4 096 blocks of ~34 KiB) is not one memory
// round trip per 16 bytes.
__device__ __forceinline__ void xround4(uint32_t& v1, uint32_t& v2, uint32_t& v3, uint32_t& v4, u32x4 w) {
    v1 = xround(v1, w.x);
    v2 = xround(v2, w.y);
    v3 = xround(v3, w.z);
    v4 = xround(v4, w.w);
}

__device__ uint32_t xxh32_lane(const uint8_t* p, int64_t len, uint32_t seed) {
    uint32_t h;
    const int64_t n16 = len >> 4;
    if (n16 > 0) {
        uint32_t v1 = seed + kP1 + kP2, v2 = seed + kP2, v3 = seed, v4 = seed - kP1;
        constexpr int U = 8;
        int64_t s = 0;
        if (n16 >= 2 * U) {
            u32x4 cur[U];
#pragma unroll
            for (int k = 0; k < U; ++k) cur[k] = ld16(p + 16 * k);
            for (; s + 2 * U <= n16; s += U) {
                u32x4 nxt[U];
#pragma unroll
                for (int k = 0; k < U; ++k) nxt[k] = ld16(p + 16 * (s + U + k));
#pragma unroll
                for (int k = 0; k < U; ++k) xround4(v1, v2, v3, v4, cur[k]);
#pragma unroll
                for (int k = 0; k < U; ++k) cur[k] = nxt[k];
            }
#pragma unroll
            for (int k = 0; k < U; ++k) xround4(v1, v2, v3, v4, cur[k]);
            s += U;
        }
        for (; s < n16; ++s) xround4(v1, v2, v3, v4, ld16(p + 16 * s));
        h = rotl32(v1, 1) + rotl32(v2, 7) + rotl32(v3, 12) + rotl32(v4, 18);
    } else {
        h = seed + kP5;
    }
    h += (uint32_t)len;
    const int64_t q = n16 << 4;
    return xfinish(h, p + q, (int)(len - q));
}

}  // namespace lz4m
