// lz4m_common.h -- shared device helpers for the MI355X LZ4 kernels (gfx950).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace lz4m {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
// a byte in LDS (address space 3): LDS and HBM accesses stay distinct
// instructions (ds_* vs global_*), never merged into generic flat accesses,
// which the compiler must fence with vmcnt(0) + lgkmcnt(0)
typedef __attribute__((address_space(3))) uint8_t lds_u8;
__device__ __forceinline__ u32x4 lds_ld16(const lds_u8* p) {
    u32x4 v;
    __builtin_memcpy(&v, (const uint8_t*)p, 16);
    return v;
}
__device__ __forceinline__ void lds_st16(lds_u8* p, u32x4 v) { __builtin_memcpy((uint8_t*)p, &v, 16); }

constexpr int kWave = 64;

// 16-byte accesses at any byte alignment: gfx950 runs in unaligned-access
// mode, so these lower to one global_load/store_dwordx4.
__device__ __forceinline__ u32x4 ld16(const uint8_t* p) {
    u32x4 v;
    __builtin_memcpy(&v, p, 16);
    return v;
}
__device__ __forceinline__ void st16(uint8_t* p, u32x4 v) { __builtin_memcpy(p, &v, 16); }
__device__ __forceinline__ uint32_t ld32(const uint8_t* p) {
    uint32_t v;
    __builtin_memcpy(&v, p, 4);
    return v;
}
__device__ __forceinline__ uint64_t ld64(const uint8_t* p) {
    uint64_t v;
    __builtin_memcpy(&v, p, 8);
    return v;
}
__device__ __forceinline__ uint32_t ld16le(const uint8_t* p) {
    uint16_t v;
    __builtin_memcpy(&v, p, 2);
    return v;
}

// 16 bytes at p, with bytes at or beyond `avail` read as zero (never
// touches memory past p + avail).
__device__ __forceinline__ u32x4 ld16_guarded(const uint8_t* p, int64_t avail) {
    if (avail >= 16) return ld16(p);
    uint64_t lo = 0, hi = 0;
    const int n = avail <= 0 ? 0 : (int)avail;
    for (int k = 0; k < n; ++k) {
        const uint64_t b = p[k];
        if (k < 8) lo |= b << (8 * k);
        else hi |= b << (8 * (k - 8));
    }
    return u32x4{(uint32_t)lo, (uint32_t)(lo >> 32), (uint32_t)hi, (uint32_t)(hi >> 32)};
}

// The 4 bytes starting at byte k (0..15) of the 16-byte window w; bytes past
// the window read as zero.
__device__ __forceinline__ uint32_t window_dword(u32x4 w, uint32_t k) {
    const uint32_t q = k >> 2;
    const uint32_t lo = q == 0 ? w.x : q == 1 ? w.y : q == 2 ? w.z : w.w;
    const uint32_t hi = q == 0 ? w.y : q == 1 ? w.z : q == 2 ? w.w : 0u;
    return __builtin_amdgcn_alignbyte(hi, lo, k & 3);
}

// Window shifted down by one byte (byte 15 reads as zero).
__device__ __forceinline__ u32x4 window_shift1(u32x4 w) {
    return u32x4{__builtin_amdgcn_alignbyte(w.y, w.x, 1), __builtin_amdgcn_alignbyte(w.z, w.y, 1),
                 __builtin_amdgcn_alignbyte(w.w, w.z, 1), __builtin_amdgcn_alignbyte(0u, w.w, 1)};
}

__device__ __forceinline__ uint32_t byte_of(u32x4 w, int k) {
    const uint32_t d = (k >> 2) == 0 ? w.x : (k >> 2) == 1 ? w.y : (k >> 2) == 2 ? w.z : w.w;
    return (d >> ((k & 3) * 8)) & 0xFFu;
}

// Expand the first `off` (1..15) bytes of w into a 16-byte pattern with
// period `off`: E[j] = w[j % off].  Doubling keeps the valid length a
// multiple of `off`.
__device__ __forceinline__ u32x4 period_pattern(u32x4 w, uint32_t off) {
    uint64_t lo = ((uint64_t)w.y << 32) | w.x;
    uint64_t hi = ((uint64_t)w.w << 32) | w.z;
    if (off < 8) {
        lo &= (1ull << (8 * off)) - 1ull;
        hi = 0;
    } else if (off == 8) {
        hi = 0;
    } else {
        hi &= (1ull << (8 * (off - 8))) - 1ull;
    }
    for (uint32_t len = off; len < 16; len *= 2) {
        const uint32_t s = 8 * len;   // 8..120, multiple of 8
        uint64_t slo, shi;
        if (s >= 64) {
            shi = lo << (s - 64);
            slo = 0;
        } else {
            shi = (hi << s) | (lo >> (64 - s));
            slo = lo << s;
        }
        lo |= slo;
        hi |= shi;
    }
    return u32x4{(uint32_t)lo, (uint32_t)(lo >> 32), (uint32_t)hi, (uint32_t)(hi >> 32)};
}

__device__ __forceinline__ uint32_t lane_id() { return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)); }

__device__ __forceinline__ int64_t readlane64(int64_t v, int lane) {
    const uint32_t lo = __builtin_amdgcn_readlane((int)(uint32_t)v, lane);
    const uint32_t hi = __builtin_amdgcn_readlane((int)(uint32_t)((uint64_t)v >> 32), lane);
    return (int64_t)(((uint64_t)hi << 32) | lo);
}
// A lane's global-memory pointer, broadcast.  Rebuilt as a global
// (address space 1) pointer, so accesses through it stay global_* (not flat).
template <typename T>
__device__ __forceinline__ T* readlane_ptr(T* p, int lane) {
    typedef __attribute__((address_space(1))) T gT;
    gT* g = (gT*)(uintptr_t)readlane64(reinterpret_cast<int64_t>(p), lane);
    return (T*)g;
}

}  // namespace lz4m
