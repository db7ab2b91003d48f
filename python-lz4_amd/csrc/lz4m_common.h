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

// ---------------------------------------------------- aligned LDS access
// A _b64 / _b128 LDS access off its natural alignment -- and a _b32 one off
// 4 bytes -- replays at ~56 cycles per wave-instruction on gfx950
// (tools/micro/lds_align.hip; cdna_hip_programming.md Guideline 17), and the
// decoders' history buffers are read and written at arbitrary byte offsets.
// So both are made of naturally aligned dword accesses only:
// - a 16-byte read at any offset is five aligned dwords (two ds_read2_b32 and
//   one ds_read_b32) and four alignbytes;
// - an exact put of k <= 16 bytes is five ds_mskor_b32 (dst = dst & ~mask |
//   data) on the enclosing aligned dwords -- atomic per dword, so
//   neighbouring sequences that share a boundary dword can be written by one
//   instruction -- with the masks from a table by (address & 3, k) and each
//   dword's bytes placed by one v_perm with a per-lane selector (0x0C, a zero
//   byte, outside the put).
typedef __attribute__((address_space(3))) volatile uint64_t lds_vu64;
typedef __attribute__((address_space(3))) const uint32_t lds_cu32;
typedef __attribute__((address_space(3))) const uint32_t lds_cu32a __attribute__((aligned(4)));
__device__ __forceinline__ uint32_t lds_addr(const lds_u8* p) { return (uint32_t)(uintptr_t)p; }
__device__ __forceinline__ u32x4 lds_ld16a(const lds_u8* p) {
    const uint32_t a = lds_addr(p), r = a & 3u;
    const lds_cu32a* q = (const lds_cu32a*)(p - r);
    const uint32_t c0 = q[0], c1 = q[1], c2 = q[2], c3 = q[3], c4 = q[4];
    return u32x4{__builtin_amdgcn_alignbyte(c1, c0, r), __builtin_amdgcn_alignbyte(c2, c1, r),
                 __builtin_amdgcn_alignbyte(c3, c2, r), __builtin_amdgcn_alignbyte(c4, c3, r)};
}
// byte masks of an exact put of k (0..16) bytes at address & 3 == r over the
// enclosing dwords 0..3: table entry (r * 17 + k), 16 bytes (dword 4 is
// computed); built once per workgroup by lds_put_table_init
constexpr int kPutTab = 4 * 17 * 4;
__device__ __forceinline__ void lds_put_table_init(uint32_t* tab, uint32_t lane, uint32_t nlanes) {
    for (uint32_t e = lane; e < (uint32_t)kPutTab; e += nlanes) {
        const uint32_t i = e & 3u, ent = e >> 2, k = ent % 17u, r = ent / 17u;
        uint32_t m = 0;
        for (uint32_t b = 0; b < 4; ++b) {
            const uint32_t pos = 4u * i + b;   // byte of the 16..20-byte span
            if (pos >= r && pos < r + k) m |= 0xFFu << (8 * b);
        }
        tab[e] = m;
    }
}
// Exactly k bytes (k >= 16: 16) of v at LDS address p.
__device__ __forceinline__ void lds_put_al(lds_u8* p, u32x4 v, int32_t k, lds_cu32* tab) {
    const uint32_t a = lds_addr(p), r = a & 3u;
    const uint32_t kk = k >= 16 ? 16u : (uint32_t)k;
    // destination dword i, byte b holds put byte 4i + b - r: v_perm of
    // (v[i], v[i-1]) with selector byte 4 + b - r, 0x0C (zero) where the
    // mask says the byte is not the put's
    u32x4 m;
    __builtin_memcpy(&m, (const uint8_t*)(tab + 4u * (r * 17u + kk)), 16);   // 16-byte aligned
    const int32_t t4 = (int32_t)(r + kk) - 16;   // bytes in dword 4 (0..3)
    const uint32_t m4 = t4 > 0 ? (1u << (8 * t4)) - 1u : 0u;
    // r replicated into every byte by one v_perm (a v_mul_lo_u32 is quarter rate)
    const uint32_t sb = 0x07060504u - __builtin_amdgcn_perm(0u, r, 0u);
    const uint32_t b4 = a & ~3u;
    auto sel = [&](uint32_t mk) __attribute__((always_inline)) { return (mk & sb) | (~mk & 0x0C0C0C0Cu); };
    const uint32_t d0 = __builtin_amdgcn_perm(v.x, v.x, sel(m.x));
    const uint32_t d1 = __builtin_amdgcn_perm(v.y, v.x, sel(m.y));
    const uint32_t d2 = __builtin_amdgcn_perm(v.z, v.y, sel(m.z));
    const uint32_t d3 = __builtin_amdgcn_perm(v.w, v.z, sel(m.w));
    const uint32_t d4 = __builtin_amdgcn_perm(0u, v.w, sel(m4));
    asm volatile("ds_mskor_b32 %0, %1, %2 offset:0" ::"v"(b4), "v"(m.x), "v"(d0) : "memory");
    asm volatile("ds_mskor_b32 %0, %1, %2 offset:4" ::"v"(b4), "v"(m.y), "v"(d1) : "memory");
    asm volatile("ds_mskor_b32 %0, %1, %2 offset:8" ::"v"(b4), "v"(m.z), "v"(d2) : "memory");
    asm volatile("ds_mskor_b32 %0, %1, %2 offset:12" ::"v"(b4), "v"(m.w), "v"(d3) : "memory");
    asm volatile("ds_mskor_b32 %0, %1, %2 offset:16" ::"v"(b4), "v"(m4), "v"(d4) : "memory");
}

// ------------------------------------------------ period-pattern selectors
// A match with offset off < 16 repeats its first off bytes: output byte j is
// w[j % off] (LZ4_memcpy_using_offset, lz4.c:513-551).  Selector table: 8
// dwords per offset (16 x 8 = 128), entry (off, i) builds output dword i >> 1
// from bytes 0-7 (i even) or 8-15 (i odd) of w; 0x0C selects a zero byte.
__device__ __forceinline__ void period_sel_init(uint32_t* psel, uint32_t tid, uint32_t nthreads) {
    for (uint32_t e = tid; e < 16u * 8u; e += nthreads) {
        const uint32_t o = e >> 3, i = e & 7, hi = i & 1;
        uint32_t v = 0;
        for (uint32_t b = 0; b < 4; ++b) {
            const uint32_t x = o ? (4 * (i >> 1) + b) % o : 0;
            const uint32_t sb = hi ? (x >= 8 ? x - 8 : 0x0C) : (x < 8 ? x : 0x0C);
            v |= sb << (8 * b);
        }
        psel[e] = v;
    }
}
// Period-off pattern of the first off (1..15) bytes of w, E[j] = w[j % off]:
// per output dword, v_perm from bytes 0-7 and from bytes 8-15 with the
// selectors sel = psel + 8 * off.
__device__ __forceinline__ u32x4 period_perm(u32x4 w, lds_cu32* sel) {
    u32x4 r;
    r.x = __builtin_amdgcn_perm(w.y, w.x, sel[0]) | __builtin_amdgcn_perm(w.w, w.z, sel[1]);
    r.y = __builtin_amdgcn_perm(w.y, w.x, sel[2]) | __builtin_amdgcn_perm(w.w, w.z, sel[3]);
    r.z = __builtin_amdgcn_perm(w.y, w.x, sel[4]) | __builtin_amdgcn_perm(w.w, w.z, sel[5]);
    r.w = __builtin_amdgcn_perm(w.y, w.x, sel[6]) | __builtin_amdgcn_perm(w.w, w.z, sel[7]);
    return r;
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
