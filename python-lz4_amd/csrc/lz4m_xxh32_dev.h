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

// ---------------------------------------------------- quad-per-item XXH32
// One QUAD (4 lanes) per item: lane a (= lane & 3) runs accumulator v[a+1]
// of XXH32_endian_align (xxhash.c:357-368) alone -- the four accumulators
// are independent serial recurrences, so an item's stripes split four ways
// and no further.  Each lane reads only its own word of every 16-byte stripe
// (a wave-instruction = one stripe of each of the wave's 16 items), and keeps
// 2 x kXQ loads in flight (two register sets, so a set is consumed only after
// the other was issued: a consumption never waits on the newest loads).  A
// batch of few long items (config 5's pages: 4 096 compressed blocks of ~34
// KiB) then has 16 384 lanes streaming, not 4 096 lanes stalled on one
// 16-byte round trip each.  Returns the lane's accumulator after the item's
// n16 full stripes; `steps` = the wave's largest n16 (uniform), p = the item
// (any valid address when n16 == 0, never read then).
constexpr int kXQ = 24;
typedef __attribute__((address_space(1))) const uint32_t gu32;
__device__ __forceinline__ uint32_t xxh32_quad_acc(const uint8_t* p, uint32_t n16, uint32_t steps, uint32_t seed,
                                                   uint32_t a) {
    uint32_t v = a == 0 ? seed + kP1 + kP2 : a == 1 ? seed + kP2 : a == 2 ? seed : seed - kP1;
    if (steps == 0) return v;
    const uint32_t last = n16 > 0 ? n16 - 1 : 0;   // loads past the item are clamped to its last stripe
    gu32* q = (gu32*)(uintptr_t)(p + 4 * a);
    uint32_t A[kXQ], B[kXQ];
#pragma unroll
    for (int k = 0; k < kXQ; ++k) A[k] = q[4 * min((uint32_t)k, last)];
    for (uint32_t s = 0; s < steps; s += 2 * kXQ) {
#pragma unroll
        for (int k = 0; k < kXQ; ++k) B[k] = q[4 * min(s + kXQ + (uint32_t)k, last)];
        __builtin_amdgcn_sched_barrier(0);   // the loads stay ahead of the consumption below
#pragma unroll
        for (int k = 0; k < kXQ; ++k) {
            const uint32_t y = xround(v, A[k]);
            v = s + (uint32_t)k < n16 ? y : v;
        }
        if (s + kXQ >= steps) break;
#pragma unroll
        for (int k = 0; k < kXQ; ++k) A[k] = q[4 * min(s + 2 * kXQ + (uint32_t)k, last)];
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int k = 0; k < kXQ; ++k) {
            const uint32_t y = xround(v, B[k]);
            v = s + kXQ + (uint32_t)k < n16 ? y : v;
        }
    }
    return v;
}

// The item's hash from its quad's four accumulators (quad lane 0 gets the
// result; xxhash.c:370-389): merge, length, tail, avalanche.
__device__ __forceinline__ uint32_t xxh32_quad_finish(uint32_t v, const uint8_t* p, int64_t len, uint32_t seed) {
    const uint32_t v1 = __builtin_amdgcn_mov_dpp(v, 0x55, 0xF, 0xF, false);   // quad_perm [1,1,1,1]
    const uint32_t v2 = __builtin_amdgcn_mov_dpp(v, 0xAA, 0xF, 0xF, false);   // [2,2,2,2]
    const uint32_t v3 = __builtin_amdgcn_mov_dpp(v, 0xFF, 0xF, 0xF, false);   // [3,3,3,3]
    const int64_t n16 = len >> 4;
    uint32_t h = n16 > 0 ? rotl32(v, 1) + rotl32(v1, 7) + rotl32(v2, 12) + rotl32(v3, 18) : seed + kP5;
    h += (uint32_t)len;
    return xfinish(h, p + 16 * n16, (int)(len - 16 * n16));
}

// the wave's largest value of x (uniform)
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t x) {
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) x = max(x, (uint32_t)__shfl_xor((int)x, d));
    return x;
}

}  // namespace lz4m
