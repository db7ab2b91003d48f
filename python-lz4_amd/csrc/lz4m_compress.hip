// lz4m_compress.hip -- batched greedy LZ4 block compressor for MI355X (gfx950).
//
// Output is byte-identical to the reference parse
// (LZ4_compress_generic_validated, lz4libs/lz4.c:910-1302, fresh table):
//   TABLE U16_HASH4 : LZ4_compress_default on < 65547 B (byU16, 13-bit hash4)
//   TABLE U32_HASH5 : lz4.block.compress / >= 65547 B (byU32, 12-bit hash5)
//
// Mapping.  One 64-lane wavefront per block; the block's 16 KiB match table
// lives in LDS (zeroed per block, like LZ4_prepareTable).  The serial search
// loop (lz4.c:1016-1075) visits a data-independent sequence of positions
// (the skip schedule step = attempts++ >> 6 is a closed form of the attempt
// index), so the wave evaluates 64 consecutive attempts at once:
//   1. every lane hashes its attempt position and reads the table;
//   2. a lane whose hash equals an earlier lane's hash in the same step takes
//      that lane's position as its candidate (the serial loop would have
//      inserted it first);
//   3. the first lane whose candidate passes the distance check and the 4-byte
//      compare is the match the serial loop would find (ballot + ctz);
//   4. table writes of lanes up to that one are committed last-writer-wins,
//      later lanes restore what they touched.
// Backward catch-up and LZ4_count are 64-/256-byte wave compares, literal
// copies are coalesced 16-byte-per-lane copies; sequence headers are written
// by lane 0.
#include "lz4m_common.h"
#include "lz4m_worker.h"

#include <chrono>
#include <mutex>
#include <type_traits>

#include <stdio.h>
#include <stdlib.h>
#include "../../include/lz4m.h"

namespace lz4m {

int pcompress_launch(const uint8_t* d_src, const int64_t* d_src_off, const int32_t* d_src_len, uint8_t* d_dst,
                     const int64_t* d_dst_off, const int32_t* d_dst_cap, int32_t* d_out_len, int64_t n, int variant,
                     hipStream_t stream);

constexpr int kMinLength = 13;        // lz4.c:247
constexpr int kLimit64K = 65536 + 11; // lz4.c:689
constexpr int kMaxInput = 0x7E000000; // lz4.h:211

__device__ __forceinline__ int64_t bound64(int64_t n) { return n + n / 255 + 16; }

// F(m) = sum_{j=0..m} floor(j/64), m >= -1
template <typename I = int64_t>
__device__ __forceinline__ I skip_sum(I m) {
    if constexpr (std::is_signed<I>::value)
        if (m < 0) return 0;
    const I q = m >> 6, r = m & 63;
    return 32 * q * (q - 1) + q * (r + 1);
}

// offset from ip of search attempt k (lz4.c:1021-1027: step = attempts++ >> 6)
template <typename I = int64_t>
__device__ __forceinline__ I attempt_off(I k, I A, I FA) {
    return k >= 1 ? 1 + skip_sum<I>(A + k - 2) - FA : 0;
}

// Acceleration 1 (every python-lz4 default) keeps the search schedule in
// 32-bit unsigned registers (A = 64, FA = 0): a search stops at the first
// step that passes mflimit, so the largest offset it computes is below
// n + 2^20 < 2^32 for any n <= LZ4_MAX_INPUT_SIZE.

typedef __attribute__((address_space(3))) uint16_t lds_t16;   // hash-table entries in LDS
typedef __attribute__((address_space(3))) uint32_t lds_t32;

template <int V>
struct Table;

template <>
struct Table<LZ4M_TABLE_U16_HASH4> {   // 8192 x u16 (lz4.c:756-762, 839-843)
    static constexpr int kEntries = 8192;
    __device__ static __forceinline__ uint32_t hash(const uint8_t* p) {
        return (ld32(p) * 2654435761u) >> (32 - 13);
    }
    __device__ static __forceinline__ uint32_t hash_v(u32x4 v) { return (v.x * 2654435761u) >> (32 - 13); }
    __device__ static __forceinline__ uint32_t get(const uint16_t* t, uint32_t h) { return ((const lds_t16*)t)[h]; }
    __device__ static __forceinline__ void put(uint16_t* t, uint32_t h, uint32_t v) { ((lds_t16*)t)[h] = (uint16_t)v; }
    // volatile: kept in program order, never forwarded (the probe reads back
    // what OTHER lanes wrote).  The table is in LDS: the accesses are cast to
    // the LDS address space, else a volatile access through the generic
    // pointer is a FLAT instruction that waits for every outstanding load.
    __device__ static __forceinline__ uint32_t get_v(uint16_t* t, uint32_t h) { return ((volatile lds_t16*)t)[h]; }
    __device__ static __forceinline__ void put_v(uint16_t* t, uint32_t h, uint32_t v) {
        ((volatile lds_t16*)t)[h] = (uint16_t)v;
    }
    static constexpr bool kDistCheck = false;   // lz4.c:1064, LZ4_DISTANCE_MAX == 65535
    // store v, return the entry before it: a masked OR with return on the
    // enclosing dword (no 16-bit exchange exists)
    __device__ static __forceinline__ uint32_t xchg(uint16_t* t, uint32_t h, uint32_t v) {
        const uint32_t a = (uint32_t)(uintptr_t)((lds_t16*)t + h) & ~3u, sh = (h & 1u) * 16u;
        uint32_t old;
        // (the wait inside: the compiler does not count an asm's LDS return)
        asm volatile("ds_mskor_rtn_b32 %0, %1, %2, %3\n\ts_waitcnt lgkmcnt(0)"
                     : "=v"(old) : "v"(a), "v"(0xFFFFu << sh), "v"((v & 0xFFFFu) << sh) : "memory");
        return (old >> sh) & 0xFFFFu;
    }
};

template <>
struct Table<LZ4M_TABLE_U32_HASH5> {   // 4096 x u32 (lz4.c:764-774, 834-838)
    static constexpr int kEntries = 4096;
    __device__ static __forceinline__ uint32_t hash(const uint8_t* p) {
        return (uint32_t)(((ld64(p) << 24) * 889523592379ull) >> (64 - 12));
    }
    __device__ static __forceinline__ uint32_t hash_v(u32x4 v) {
        const uint64_t x = ((uint64_t)v.y << 32) | v.x;
        return (uint32_t)(((x << 24) * 889523592379ull) >> (64 - 12));
    }
    __device__ static __forceinline__ uint32_t get(const uint16_t* t, uint32_t h) { return ((const lds_t32*)t)[h]; }
    __device__ static __forceinline__ void put(uint16_t* t, uint32_t h, uint32_t v) { ((lds_t32*)t)[h] = v; }
    __device__ static __forceinline__ uint32_t get_v(uint16_t* t, uint32_t h) { return ((volatile lds_t32*)t)[h]; }
    __device__ static __forceinline__ void put_v(uint16_t* t, uint32_t h, uint32_t v) { ((volatile lds_t32*)t)[h] = v; }
    static constexpr bool kDistCheck = true;
    __device__ static __forceinline__ uint32_t xchg(uint16_t* t, uint32_t h, uint32_t v) {
        return __hip_atomic_exchange((lds_t32*)t + h, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
};

// The byU32 / hash5 table (same hash, same semantics) for indexes below 2^17
// -- the speculative linked passes, where an index is a byte of 64 KiB of
// history + a block of <= 64 KiB: the low 16 bits of entry h are a u16 at
// t[h] and bit 16 is bit h of a 4096-bit map behind them (8.5 KiB instead
// of 16: 16 workgroups per CU instead of 9).  A store writes both parts; an
// exchange swaps both, each with a masked OR on its enclosing dword (lanes on
// one dword are applied in lane order, as Table<U32>::xchg's exchange).
constexpr int kTableU17 = 0x117;
constexpr int kU17Halves = 4096 + 256;   // table size in u16
template <>
struct Table<kTableU17> {
    static constexpr int kEntries = 4096;
    __device__ static __forceinline__ uint32_t hash(const uint8_t* p) { return Table<LZ4M_TABLE_U32_HASH5>::hash(p); }
    __device__ static __forceinline__ uint32_t hash_v(u32x4 v) { return Table<LZ4M_TABLE_U32_HASH5>::hash_v(v); }
    __device__ static __forceinline__ uint32_t get_v(uint16_t* t, uint32_t h) {
        const uint32_t lo = ((volatile lds_t16*)t)[h];
        const uint32_t m = ((volatile lds_t32*)(t + 4096))[h >> 5];
        return lo | (((m >> (h & 31u)) & 1u) << 16);
    }
    __device__ static __forceinline__ uint32_t get(const uint16_t* t, uint32_t h) { return get_v((uint16_t*)t, h); }
    __device__ static __forceinline__ void put_v(uint16_t* t, uint32_t h, uint32_t v) {
        ((volatile lds_t16*)t)[h] = (uint16_t)v;
        const uint32_t a = (uint32_t)(uintptr_t)((lds_t32*)(t + 4096) + (h >> 5)), b = 1u << (h & 31u);
        asm volatile("ds_mskor_b32 %0, %1, %2" : : "v"(a), "v"(b), "v"(((v >> 16) & 1u) << (h & 31u)) : "memory");
    }
    __device__ static __forceinline__ void put(uint16_t* t, uint32_t h, uint32_t v) { put_v(t, h, v); }
    static constexpr bool kDistCheck = true;
    __device__ static __forceinline__ uint32_t xchg(uint16_t* t, uint32_t h, uint32_t v) {
        const uint32_t a = (uint32_t)(uintptr_t)((lds_t16*)t + h) & ~3u, sh = (h & 1u) * 16u;
        const uint32_t am = (uint32_t)(uintptr_t)((lds_t32*)(t + 4096) + (h >> 5)), bit = h & 31u;
        uint32_t lo, hi;
        asm volatile("ds_mskor_rtn_b32 %0, %2, %3, %4\n\tds_mskor_rtn_b32 %1, %5, %6, %7\n\ts_waitcnt lgkmcnt(0)"
                     : "=&v"(lo), "=&v"(hi)
                     : "v"(a), "v"(0xFFFFu << sh), "v"((v & 0xFFFFu) << sh), "v"(am), "v"(1u << bit),
                       "v"(((v >> 16) & 1u) << bit)
                     : "memory");
        return ((lo >> sh) & 0xFFFFu) | (((hi >> bit) & 1u) << 16);
    }
};

// The search step inserts its 64 positions with one LDS
// exchange per lane; lanes of a wave that hit the same bucket are applied in
// lane order (gfx950: every one of 33.5 M instructions of random collision
// patterns, tools/micro/lds_xchg_order.hip, r05l), so each lane reads back
// exactly the entry the serial loop (lz4.c:1016-1075) would read: the table's
// for the first lane of a bucket, the previous lane's position for the others.
// After the step's first hit f, the first lane after f in each bucket writes
// back what it read (positions increase with the lane, so that lane is the one
// whose read value is below lane f+1's position).  Replaces a read, a probe
// write, a read back and a loop over the colliding groups.

__device__ __forceinline__ uint32_t uni(uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); }
__device__ __forceinline__ int64_t uni64(int64_t v) {
    const uint32_t lo = uni((uint32_t)v), hi = uni((uint32_t)((uint64_t)v >> 32));
    return (int64_t)(((uint64_t)hi << 32) | lo);
}

// Coalesced copy of len bytes (wave-cooperative); never writes past d+d_room
// or reads past s+s_room.
// The source and destination never overlap: each lane requests four 16-byte
// pieces before storing any (one memory round trip per 4 KiB, not per 1 KiB).
__device__ __forceinline__ void wave_copy(uint8_t* d, const uint8_t* s, int64_t len, int64_t d_room,
                                          int64_t s_room, uint32_t lane) {
    constexpr int kU = 4;
    for (int64_t base = 0; base < len; base += 16 * kWave * kU) {
        u32x4 v[kU];
#pragma unroll
        for (int u = 0; u < kU; ++u) {
            const int64_t pos = base + 16 * kWave * u + 16 * (int64_t)lane;
            const bool whole = pos < len && (len - pos >= 16 || s_room - pos >= 16);
            v[u] = whole ? ld16(s + pos) : u32x4{0, 0, 0, 0};
        }
#pragma unroll
        for (int u = 0; u < kU; ++u) {
            const int64_t pos = base + 16 * kWave * u + 16 * (int64_t)lane;
            if (pos < len) {
                if (len - pos >= 16 || (d_room - pos >= 16 && s_room - pos >= 16)) {
                    st16(d + pos, v[u]);
                } else {
                    for (int64_t k = pos; k < len; ++k) d[k] = s[k];
                }
            }
        }
    }
}

// Exactly k bytes (k >= 16: 16) of v at global address p
__device__ __forceinline__ void gbl_put_c(uint8_t* p, u32x4 v, int32_t k) {
    if (k >= 16) {
        st16(p, v);
        return;
    }
    for (int32_t j = 0; j < k; ++j) p[j] = (uint8_t)byte_of(v, j);
}

// kTnMerge: at acceleration 1 the test of the next position after a
// match (lz4.c:1207-1258) may be lane 0 of the next search step instead of a
// step of its own.  Exact: it is the search attempt at ip with anchor == ip
// (no catch-up, no literals), after the insert of ip - 2; the step's other
// lanes are the first 63 attempts of the search from ip + 1 that follows a
// failed test (the output-limit check of a zero-length literal run is implied
// by the match's, lz4.c:1085-1089 vs 1184-1190).  A 64-lane step costs more
// than the lone test, so this pays only where the test mostly fails: the
// parse keeps a running hit rate of the test (1/256 units, weight 1/8) and
// merges while it is below kTnMerge (0: never; 257: always).  r05h:
// always merging cost silesia-like / text blocks 10 / 30 % and saved 13 % on
// binary records; r05i, against never: threshold 64 -5.5 % silesia-like,
// +2.4 % text, -12 % records (96: -5.0 / +3.4 / -12; 128: -3.5 / +8.5 / -12).
constexpr int32_t kTnMerge = 64;

// length bytes after a token nibble of 15 (lz4.c:1094-1099, 1184-1194);
// returns the new output position.  Written by lane 0.
__device__ __forceinline__ int64_t put_len(uint8_t* dst, int64_t op, int64_t len, uint32_t lane) {
    const int64_t n255 = len / 255;
    for (int64_t k = lane; k < n255; k += kWave) dst[op + k] = 255;
    if (lane == 0) dst[op + n255] = (uint8_t)(len - 255 * n255);
    return op + n255 + 1;
}

// ---- source window ---------------------------------------------------------
// The bytes around the parse position live in a 1 KiB LDS ring, refilled
// 512 B at a time (8 B per lane) ahead of the parse, so the hash inputs, the
// literal copies and the source side of catch-up / match counting are LDS
// reads; only the candidate side (anywhere in the last 64 KiB) is read from
// HBM / L2, 20 bytes per candidate, which settles the 4-byte check, a short
// catch-up and a short match in one round trip.
constexpr int kRing = 1024;
constexpr int kChunk = 512;   // refill unit: 8 bytes per lane
constexpr int kLaneB = kChunk / kWave;
static_assert(kLaneB == 16 || kLaneB == 8, "ring refill granularity");
static_assert(kChunk <= kRing / 2, "ring too small for its refill unit");
constexpr int kRingBytes = kRing + 32;   // + a mirror of the first 32 bytes
typedef __attribute__((address_space(3))) uint32_t lds_u32;
#define RING_DECL                                                               \
    __shared__ __attribute__((aligned(16))) uint8_t ring_mem[kRingBytes];         \
    lds_u8* ring = (lds_u8*)ring_mem;

struct Win {
    lds_u8* r;
    int32_t base;   // window position at ring offset 0 (the block start)
    int32_t whi;    // resident: [max(base, whi - kRing), whi)
    int32_t iend;
    __device__ __forceinline__ bool has(int32_t p, int32_t len) const {
        return p >= base && p >= whi - kRing && p + len <= whi;
    }
};

// bytes [p-4, p) -> pm and [p, p+16) -> v from the ring (p resident per has(p-4, 20))
__device__ __forceinline__ void ring_fetch(const Win& W, int32_t p, uint32_t& pm, u32x4& v) {
    const uint32_t i = (uint32_t)(p - W.base) & (kRing - 1);
    const uint32_t sh = i & 3, j = i >> 2;
    const lds_u32* R = (const lds_u32*)W.r;
    const uint32_t a = R[(j - 1) & (kRing / 4 - 1)];
    const uint32_t b = R[j], c = R[j + 1], d = R[j + 2], e = R[j + 3], f = R[j + 4];
    pm = __builtin_amdgcn_alignbyte(b, a, sh);
    v = u32x4{__builtin_amdgcn_alignbyte(c, b, sh), __builtin_amdgcn_alignbyte(d, c, sh),
              __builtin_amdgcn_alignbyte(e, d, sh), __builtin_amdgcn_alignbyte(f, e, sh)};
}

__device__ __forceinline__ u32x4 ring_fetch16(const Win& W, int32_t p) {
    const uint32_t i = (uint32_t)(p - W.base) & (kRing - 1);
    const uint32_t sh = i & 3, j = i >> 2;
    const lds_u32* R = (const lds_u32*)W.r;
    const uint32_t b = R[j], c = R[j + 1], d = R[j + 2], e = R[j + 3], f = R[j + 4];
    return u32x4{__builtin_amdgcn_alignbyte(c, b, sh), __builtin_amdgcn_alignbyte(d, c, sh),
                 __builtin_amdgcn_alignbyte(e, d, sh), __builtin_amdgcn_alignbyte(f, e, sh)};
}

// a refill may overwrite ring bytes that are before `keep` (or before the block)
__device__ __forceinline__ bool can_fill(const Win& W, int32_t keep) {
    return W.whi < W.iend && W.whi - kRing + kChunk <= (keep > W.base ? keep : W.base);
}
// bytes [p, p+16) of the window for 0 <= p < iend; bytes at or past iend are
// unspecified.  One unconditional load whose address is clamped into the
// window (the caller's buffer may end at iend), realigned in registers --
// loads in branches make the compiler wait for them at the join.
__device__ __forceinline__ u32x4 shr_bytes(u32x4 r, uint32_t d) {
    const uint32_t q = d >> 2, s = d & 3;
    const uint32_t a0 = q == 0 ? r.x : q == 1 ? r.y : q == 2 ? r.z : r.w;
    const uint32_t a1 = q == 0 ? r.y : q == 1 ? r.z : q == 2 ? r.w : 0u;
    const uint32_t a2 = q == 0 ? r.z : q == 1 ? r.w : 0u;
    const uint32_t a3 = q == 0 ? r.w : 0u;
    return u32x4{__builtin_amdgcn_alignbyte(a1, a0, s), __builtin_amdgcn_alignbyte(a2, a1, s),
                 __builtin_amdgcn_alignbyte(a3, a2, s), __builtin_amdgcn_alignbyte(0u, a3, s)};
}
__device__ __forceinline__ u32x4 ld16_win(const uint8_t* w, int32_t p, int32_t iend) {
    if (iend < 16) return ld16_guarded(w + p, iend - p);   // tiny window (uniform)
    const int32_t q = p < iend - 16 ? p : iend - 16;
    return shr_bytes(ld16(w + q), (uint32_t)(p - q));
}
// the 4 bytes before window position p (bytes before the window start read
// as 0); the window holds >= 4 bytes
__device__ __forceinline__ uint32_t ld_before(const uint8_t* w, int32_t p) {
    const uint32_t x = ld32(w + (p >= 4 ? p - 4 : 0));
    return p >= 4 ? x : p <= 0 ? 0u : x << (8 * (4 - (uint32_t)p));
}

__device__ __forceinline__ u32x4 fill_load(const Win& W, const uint8_t* w, uint32_t lane) {
    const int32_t p = W.whi + kLaneB * (int32_t)lane;
    return ld16_win(w, p < W.iend ? p : W.iend - 1, W.iend);
}
__device__ __forceinline__ void fill_commit(Win& W, u32x4 v, uint32_t lane) {
    const uint32_t o = (uint32_t)(W.whi - W.base + kLaneB * (int32_t)lane) & (kRing - 1);
    if (kLaneB == 16) {
        lds_st16(W.r + o, v);
        if (o < 32) lds_st16(W.r + kRing + o, v);
    } else {
        const uint64_t x = ((uint64_t)v.y << 32) | v.x;
        __builtin_memcpy((uint8_t*)(W.r + o), &x, 8);
        if (o < 32) __builtin_memcpy((uint8_t*)(W.r + kRing + o), &x, 8);
    }
    W.whi += kChunk;
}
// synchronous top-up until `need` is resident (or nothing more may be evicted)
__device__ __forceinline__ void top_up(Win& W, const uint8_t* w, int32_t need, int32_t keep, uint32_t lane) {
    while (W.whi < need && can_fill(W, keep)) fill_commit(W, fill_load(W, w, lane), lane);
}

// bytes [p-4, p) and [p, p+16) of the window: from the ring, or (some lane
// outside it) from memory
__device__ __forceinline__ void src_fetch(const Win& W, const uint8_t* w, int32_t p, uint32_t& pm, u32x4& v) {
    const bool in = W.has(p - 4, 20);
    ring_fetch(W, p, pm, v);
    if (__any(!in)) {
        const u32x4 gv = ld16_win(w, p, W.iend);
        const uint32_t gm = ld_before(w, p);
        if (!in) {
            v = gv;
            pm = gm;
        }
    }
}

// LW (the whole window staged in LDS: the lone-block kernels, the LDS-staged
// linked passes): window reads are single LDS reads at any alignment -- no
// ring, no refills, no clamped realignment -- [p, p+16) by three aligned
// 8-byte reads and a funnel, [p-4, p) by two aligned dwords.  The staging
// zero-fills 64 bytes past the window, so reads past iend stay inside it.
__device__ __forceinline__ u32x4 lw_ld16(const uint8_t* w, int32_t p) { return lds_ld16a((const lds_u8*)(w + p)); }
__device__ __forceinline__ uint32_t lw_ld4(const uint8_t* w, int32_t p) {
    const lds_u8* q = (const lds_u8*)(w + p);
    const uint32_t a = lds_addr(q);
    const lds_cu32* d = (const lds_cu32*)(q - (a & 3u));
    return __builtin_amdgcn_alignbyte(d[1], d[0], a & 3u);
}
__device__ __forceinline__ uint32_t lw_before(const uint8_t* w, int32_t p) {   // as ld_before
    const uint32_t x = lw_ld4(w, p >= 4 ? p - 4 : 0);
    return p >= 4 ? x : p <= 0 ? 0u : x << (8 * (4 - (uint32_t)p));
}

// LW with `stage` (the lone-block kernel): the window is still being staged
// by the other waves, kStageChunk bytes at a time, and stage[c] != 0 once
// chunk c is in LDS.  lw_need(x) waits until bytes [0, x) are; `have` (wave
// uniform) is what the parse already knows to be staged.
constexpr int32_t kStageChunk = 4096;
// stage[kStageFail] != 0: a wait gave up (the staged bytes never came); the
// parse then runs on to its end without waiting and the lone-block kernel
// reports kSoloStageFail instead of the bytes it made (no
// silently wrong block)
constexpr int32_t kStageFail = 17;
constexpr int32_t kSoloStageFail = LZ4M_SOLO_STAGE_FAIL;   // internal result: redo the call another way (lz4m_host.hip)
typedef __attribute__((address_space(3))) volatile int32_t lds_vi32;
__device__ __forceinline__ void lw_need(const int32_t* stage, int32_t& have, int32_t x) {
    if (stage == nullptr) return;
    while (have < x) {
        const lds_vi32* f = (const lds_vi32*)stage;
        const int32_t c = have / kStageChunk;
        uint32_t spins = 0;
        for (; f[c] == 0 && spins < (1u << 22); ++spins) __builtin_amdgcn_s_sleep(1);
        if (spins == (1u << 22)) {   // (~0.1 s): give up, flag it, wait no more
            *(lds_vi32*)(const_cast<int32_t*>(stage) + kStageFail) = 1;
            have = INT32_MAX;
            return;
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        have += kStageChunk;
    }
}

// number of equal leading bytes of a ^ b over 12 bytes (the dwords y, z, w)
__device__ __forceinline__ int eq12(u32x4 a, u32x4 b) {
    const uint32_t x1 = a.y ^ b.y, x2 = a.z ^ b.z, x3 = a.w ^ b.w;
    if (x1) return (int)(__builtin_ctz(x1) >> 3);
    if (x2) return 4 + (int)(__builtin_ctz(x2) >> 3);
    if (x3) return 8 + (int)(__builtin_ctz(x3) >> 3);
    return 12;
}

__device__ __forceinline__ u32x4 readlane_x4(u32x4 v, int l) {
    return u32x4{(uint32_t)__builtin_amdgcn_readlane((int)v.x, l), (uint32_t)__builtin_amdgcn_readlane((int)v.y, l),
                 (uint32_t)__builtin_amdgcn_readlane((int)v.z, l), (uint32_t)__builtin_amdgcn_readlane((int)v.w, l)};
}

// Window form.  The block is w[hist .. hist+n); w[0 .. hist) is history the
// parse may match into (a dictionary or the previous blocks of a linked
// frame).  Table entries are indexes: window byte p has index ibase + p, so
// the block starts at index ibase + hist (the stream's currentOffset,
// lz4.c:925-926).  A candidate below low_idx is outside the valid area
// (dictSmall, lz4.c:1061/1247) and one more than 65535 back is too far
// (lz4.c:1062-1065, byU32 only).  Backward catch-up stops at window byte
// low_src for matches inside the block and low_dict for matches in the
// history (lowLimit, lz4.c:966, 1036-1053).  The caller prepares the table
// (zeroed for a fresh stream, lz4.c:1513 / LZ4_prepareTable; loaded from a
// dictionary; or carried over from the previous block).
// oracle: orc_compress_window (oracle/lz4_oracle.c).
// LW: the window w is staged in LDS (see lw_ld16); the ring is not used.
// last_lit (nullptr, or LDS): the last literals are NOT copied; lane 0 stores
// {their output offset, their window offset} there for the caller to copy
// (the lone-block kernel copies them straight from the staged block to the
// host with all four waves: one wave copying 64 KiB inside LDS was 25 % of a
// random block's call).
template <int V, bool ACC1 = false, bool LW = false>
__device__ __forceinline__ int32_t compress_block_w(const uint8_t* __restrict__ w, int32_t hist, int32_t n, uint8_t* dst,
                                    int32_t cap, int accel, uint16_t* tab, lds_u8* ring, uint32_t lane,
                                    uint32_t ibase, uint32_t low_idx, int32_t low_src, int32_t low_dict,
                                    int32_t* last_lit = nullptr, const int32_t* stage = nullptr) {
    using T = Table<V>;
    if (n > kMaxInput) return 0;                               // lz4.c:1324
    const bool limited = cap < bound64(n);
    if (n == 0) {                                              // lz4.c:1325-1336
        if (limited && cap <= 0) return 0;
        if (lane == 0) dst[0] = 0;
        return 1;
    }
    if (V == LZ4M_TABLE_U16_HASH4 && n >= kLimit64K) return 0;   // lz4.c:963

    const int32_t iend = hist + n;
    const int32_t mflimit1 = iend - 12 + 1;                     // lz4.c:942
    const int32_t matchlimit = iend - 5;
    using SI = typename std::conditional<ACC1, uint32_t, int64_t>::type;   // search-schedule integers
    const SI A = ACC1 ? (SI)64 : (SI)((int64_t)accel << 6);   // searchMatchNb start
    const SI FA = ACC1 ? (SI)0 : skip_sum<SI>(A - 1);
    int32_t anchor = hist, ip = hist, op = 0;
    Win W{ring, hist, hist, iend};
    // the match being encoded: ip side P = [pbase, pbase+16), candidate side
    // G = [gbase, gbase+16), back = bytes the catch-up moved before them
    u32x4 P, G;
    int32_t pbase = 0, gbase = 0, back = 0;

    int32_t staged = 0;   // LW with `stage`: bytes known to be in LDS (wave uniform)
    int32_t tnb = 0;      // 1: the next search step starts with the test of position ip (kTnMerge)
    int32_t tnh = 128;    // running hit rate of the test of the next position, 1/256 units
    if (n < kMinLength) goto last_literals;                    // lz4.c:981

    if constexpr (!LW) top_up(W, w, hist + kRing, hist, lane);
    if constexpr (LW) lw_need(stage, staged, hist + 8);
    if (lane == 0) T::put_v(tab, T::hash(w + hist), ibase + (uint32_t)hist);   // lz4.c:984
    ip = hist + 1;

    for (;;) {
        int32_t match;
        uint32_t PM, GM;
        {   // ---- search (lz4.c:1016-1075), 64 attempts per wave step ----
            SI k0 = 0;
            // the search origin (lz4.c:1017 forwardIp): ip, or ip + 1 after the
            // test of ip in lane 0 (tnb); attempt k of lane l: k = k0 + l - tnb
            const int32_t ipo = ip + tnb;
            for (;;) {
                const SI k = k0 + (SI)lane - (SI)tnb;
                // attempts 0..63 of acceleration 1 are consecutive positions
                // (with tnb, lane 0's "attempt -1" is the tested position ip)
                const bool unit = A == 64 && k0 == 0;
                const SI pos64 = ipo + (unit ? k : attempt_off<SI>(k, A, FA));
                const SI nxt = unit ? pos64 + 1 : ipo + 1 + skip_sum<SI>(A + k - 1) - FA;   // attempt k+1
                const bool valid = nxt <= (SI)mflimit1;
                const int32_t pos = valid ? (int32_t)pos64 : ip;
                const uint64_t vmask = __ballot(valid);
                const int nvalid = __builtin_popcountll(vmask);   // valid lanes are a prefix
                uint32_t pm = 0;
                u32x4 pv = u32x4{0, 0, 0, 0};
                if constexpr (LW) {
                    if (stage != nullptr && nvalid > 0)
                        lw_need(stage, staged, __builtin_amdgcn_readlane(pos, nvalid - 1) + 24);
                    pv = lw_ld16(w, pos);
                    pm = lw_before(w, pos);
                } else {
                    if (nvalid > 0) {
                        const int32_t pmax = __builtin_amdgcn_readlane(pos, nvalid - 1);
                        if (pmax + 16 > W.whi) top_up(W, w, pmax + 16 + kChunk, anchor - 8, lane);
                    }
                    src_fetch(W, w, pos, pm, pv);
                }
                const uint32_t cur = ibase + (uint32_t)pos;
                // each lane exchanges its position into its bucket (one LDS
                // round trip; the lanes of a bucket in lane order, below)
                uint32_t h = 0, old = 0;
                if (tnb && k0 == 0 && lane == 0) {   // lz4.c:1207-1208: ip - 2 first
                    const u32x4 pv2 = u32x4{__builtin_amdgcn_alignbyte(pv.x, pm, 2),
                                            __builtin_amdgcn_alignbyte(pv.y, pv.x, 2), 0u, 0u};
                    T::put_v(tab, T::hash_v(pv2), cur - 2u);
                }
                if (valid) {
                    h = T::hash_v(pv);
                    old = T::xchg(tab, h, cur);
                }
                // the exchange returns to each lane what the serial insert
                // order reads: the previous lane's position of its bucket, or
                // the table's entry for the bucket's first lane
                const uint32_t cand = old;
                int32_t cpos = pos;
                bool ok = false;
                u32x4 gv = u32x4{0, 0, 0, 0};
                uint32_t gm = 0;
                ok = valid && !((T::kDistCheck && cand + 65535u < cur) || cand < low_idx);
                if (ok) cpos = (int32_t)cand - (int32_t)ibase;
                // refill the ring ahead of the parse under the same wait
                const bool pf = !LW && W.whi < ip + (kRing - kChunk) && can_fill(W, anchor - 8);
                u32x4 fv = u32x4{0, 0, 0, 0};
                if (pf) fv = fill_load(W, w, lane);
                if constexpr (LW) {
                    gv = lw_ld16(w, cpos);
                    gm = lw_before(w, cpos);
                } else {
                    gv = ld16_win(w, cpos, iend);   // unconditional (cpos = pos when not ok)
                    gm = ld_before(w, cpos);
                }
                const bool hit = ok && gv.x == pv.x;
                const uint64_t hmask = __ballot(hit);
                const int f = hmask ? __builtin_ctzll(hmask) : nvalid;   // last lane processed: f (or all valid)
                if (tnb && k0 == 0) tnh += ((int32_t)(hmask & 1u) * 256 - tnh) >> 3;
                // undo the lanes after f: the first of each bucket restores
                if (f < nvalid) {
                    const uint32_t cf1 = (uint32_t)__builtin_amdgcn_readlane((int)cur, f < 63 ? f + 1 : 63);
                    if (valid && (int)lane > f && old < cf1) T::put_v(tab, h, old);
                }
                if (pf) fill_commit(W, fv, lane);
                if (hmask) {
                    ip = __builtin_amdgcn_readlane(pos, f);
                    match = __builtin_amdgcn_readlane(cpos, f);
                    P = readlane_x4(pv, f);
                    G = readlane_x4(gv, f);
                    PM = (uint32_t)__builtin_amdgcn_readlane((int)pm, f);
                    GM = (uint32_t)__builtin_amdgcn_readlane((int)gm, f);
                    break;
                }
                if (nvalid < kWave) goto last_literals;        // forwardIp > mflimitPlusOne
                k0 += kWave;
            }
            pbase = ip;
            gbase = match;
        }

        {   // ---- backward catch-up (lz4.c:1080) ----
            const int32_t low = match < hist ? low_dict : low_src;
            const int32_t lim = (ip - anchor) < (match - low) ? (ip - anchor) : (match - low);
            const uint32_t x = PM ^ GM;   // byte 3: ip[-1] vs match[-1]
            int32_t r = x == 0 ? 4 : (int32_t)(__builtin_clz(x) >> 3);
            if (r > lim) r = lim;
            ip -= r;
            match -= r;
            if (r == 4 && lim > 4) {
                for (;;) {
                    const int32_t a = ip - 1 - lane, b = match - 1 - lane;
                    const bool okc = a >= anchor && b >= low && w[a < 0 ? 0 : a] == w[b < 0 ? 0 : b];
                    const uint64_t m = __ballot(okc);
                    const int run = ~m == 0 ? kWave : (int)__builtin_ctzll(~m);   // leading lanes that extend
                    ip -= run;
                    match -= run;
                    if (run < kWave) break;
                }
            }
            back = pbase - ip;
        }

    next_match:   // (the separate test of the next position: anchor == ip, no literals)
        {   // ---- match length, then the sequence's bytes (lz4.c:1083-1197) ----
            // LZ4_count(ip+4, match+4, matchlimit) first (it reads the source
            // only), so that the sequence's size is known before any byte of it
            // is written: bytes 4..15 of P/G, then 4 bytes per lane from HBM; a
            // match in the history runs on into the block (lz4.c:1141-1153) --
            // the window is contiguous
            const int32_t lit = ip - anchor;
            const uint32_t off = (uint32_t)(ip - match);
            const int32_t avail = matchlimit - (pbase + 4);
            int32_t c = eq12(P, G);
            if (c > avail) c = avail;
            int32_t mcode = back + c;
            if (c == 12 && avail > 12) {
                int32_t more = 0;
                const int32_t p = pbase + 16, q = gbase + 16;
                for (;;) {
                    if constexpr (LW) {   // the compares read no further than matchlimit
                        const int32_t x = p + more + 4 * kWave + 8;
                        lw_need(stage, staged, x < iend ? x : iend);
                    }
                    const int32_t av = matchlimit - (p + more);
                    const int32_t at = more + 4 * (int32_t)lane;
                    const int32_t rem = av - 4 * (int32_t)lane;   // bytes this lane may compare
                    uint32_t x = 0xFFFFFFFFu;   // nonzero = mismatch within range
                    int lim = 0;
                    if (rem >= 4) {
                        x = ld32(w + p + at) ^ ld32(w + q + at);
                        lim = 4;
                    } else if (rem > 0) {
                        uint32_t xa = 0, xb = 0;
                        for (int j = 0; j < (int)rem; ++j) {
                            xa |= (uint32_t)w[p + at + j] << (8 * j);
                            xb |= (uint32_t)w[q + at + j] << (8 * j);
                        }
                        x = xa ^ xb;
                        lim = (int)rem;
                    }
                    int eq = lim;
                    if (x != 0) {
                        const int cz = (int)(__builtin_ctz(x) >> 3);
                        eq = cz < lim ? cz : lim;
                    }
                    const uint64_t stop = __ballot(eq < 4);
                    if (stop == 0) {
                        more += 4 * kWave;
                        continue;
                    }
                    const int fl = __builtin_ctzll(stop);
                    more += 4 * (int32_t)fl + __builtin_amdgcn_readlane(eq, fl);
                    break;
                }
                mcode += more;
            }
            mcode = (int32_t)uni((uint32_t)mcode);
            // the output checks, in the reference's order (lz4.c:1085-1089, 1184-1190;
            // for the test of the next position the first is implied by the second)
            if (limited && op + 1 + lit + (2 + 1 + 5) + lit / 255 > cap) return 0;
            const int32_t llb = lit >= 15 ? (lit - 15) / 255 + 1 : 0;   // literal-length bytes
            const int32_t mlb = mcode >= 15 ? (mcode - 15) / 255 + 1 : 0;   // match-length bytes
            if (limited && op + 1 + llb + lit + 2 + (1 + 5) + (mcode + 240) / 255 > cap) return 0;
            const uint32_t tok = ((uint32_t)(lit < 15 ? lit : 15) << 4) | (uint32_t)(mcode < 15 ? mcode : 15);
            {
                const int32_t tok_pos = op;
                op += 1;
                if (llb) op = put_len(dst, op, lit - 15, lane);
                uint8_t* d = dst + op;
                const int32_t d_room = cap - op;
                for (int32_t b0 = 0; b0 < lit; b0 += 16 * kWave) {
                    const int32_t q = b0 + 16 * (int32_t)lane;
                    if (q < lit) {
                        const int32_t p = anchor + q;
                        u32x4 v;
                        if constexpr (LW) {
                            v = lw_ld16(w, p);
                        } else {
                            const bool in = W.has(p, 16);
                            v = ring_fetch16(W, p);
                            if (__any(!in)) {
                                const u32x4 gv = ld16_win(w, p, iend);
                                if (!in) v = gv;
                            }
                        }
                        if (lit - q >= 16 || d_room - q >= 16) {
                            st16(d + q, v);
                        } else {
                            for (int32_t j = 0; j < lit - q; ++j) d[q + j] = (uint8_t)byte_of(v, (int)j);
                        }
                    }
                }
                op += lit;
                if (lane == 0) {
                    dst[op] = (uint8_t)off;
                    dst[op + 1] = (uint8_t)(off >> 8);
                }
                op += 2;
                if (mlb) op = put_len(dst, op, mcode - 15, lane);
                if (lane == 0) dst[tok_pos] = (uint8_t)tok;
            }
            ip += mcode + 4;
        }
        anchor = ip;
        if (ip >= mflimit1) break;                             // lz4.c:1204
        tnb = A == 64 && tnh < kTnMerge;
        if (tnb) continue;   // the test of ip: lane 0 of the next search step

        {   // ---- fill table, test next position (lz4.c:1207-1258) ----
            uint32_t pm;
            u32x4 pv;
            if constexpr (LW) {
                lw_need(stage, staged, ip + 24);
                pv = lw_ld16(w, ip);
                pm = lw_before(w, ip);
            } else {
                if (ip + 16 > W.whi) top_up(W, w, ip + 16 + kChunk, ip - 8, lane);
                src_fetch(W, w, ip, pm, pv);
            }
            // bytes [ip-2, ip+6)
            const u32x4 pv2 = u32x4{__builtin_amdgcn_alignbyte(pv.x, pm, 2), __builtin_amdgcn_alignbyte(pv.y, pv.x, 2),
                                    0u, 0u};
            const uint32_t h2 = T::hash_v(pv2);
            const uint32_t h = T::hash_v(pv);
            const uint32_t cur = ibase + (uint32_t)ip;
            if (lane == 0) T::put_v(tab, h2, cur - 2u);
            const uint32_t cand = uni(T::get_v(tab, h));
            if (lane == 0) T::put_v(tab, h, cur);
            const bool ok = cand >= low_idx && (!T::kDistCheck || cand + 65535u >= cur);
            {
                const int32_t cpos = ok ? (int32_t)cand - (int32_t)ibase : ip;
                // (a candidate inside the ring read from there instead: -0.5 %, r04aa)
                const u32x4 gv = LW ? lw_ld16(w, cpos) : ld16_win(w, cpos, iend);
                const bool thit = ok && gv.x == pv.x;
                tnh += ((int32_t)thit * 256 - tnh) >> 3;
                if (thit) {
                    match = cpos;
                    P = pv;
                    G = gv;
                    pbase = ip;
                    gbase = cpos;
                    back = 0;
                    goto next_match;
                }
            }
        }
        ++ip;
    }

last_literals:
    {   // lz4.c:1266-1293
        const int32_t run = iend - anchor;
        if (limited && op + run + 1 + (run + 255 - 15) / 255 > cap) return 0;
        const int32_t tpos = op;
        op += 1;
        if (run >= 15) {
            if (lane == 0) dst[tpos] = 15 << 4;
            op = put_len(dst, op, run - 15, lane);
        } else if (lane == 0) {
            dst[tpos] = (uint8_t)(run << 4);
        }
        if (last_lit != nullptr) {
            if (lane == 0) {
                last_lit[0] = op;
                last_lit[1] = anchor;
            }
        } else {
            wave_copy(dst + op, w + anchor, run, cap - op, iend - anchor, lane);
        }
        op += run;
    }
    return op;
}

// zero the 16 KiB table (a fresh stream: lz4.c:1513, 1522 / LZ4_prepareTable)
__device__ __forceinline__ void zero_table(uint16_t* tab, uint32_t lane) {
    u32x4* t4 = reinterpret_cast<u32x4*>(tab);
    for (int k = lane; k < 16384 / 16; k += kWave) t4[k] = u32x4{0, 0, 0, 0};
    __builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0)
}

// One block with a fresh table (LZ4_compress_generic_validated, noDict).
template <int V, bool ACC1, bool LW = false>
__device__ __forceinline__ int64_t compress_block(const uint8_t* __restrict__ src, int64_t n, uint8_t* dst,
                                                  int64_t cap, int accel, uint16_t* tab, lds_u8* ring,
                                                  uint32_t lane, int32_t* last_lit = nullptr,
                                                  const int32_t* stage = nullptr) {
    if (n > kMaxInput) return 0;
    zero_table(tab, lane);
    return compress_block_w<V, ACC1, LW>(src, 0, n, dst, cap, accel, tab, ring, lane, 0u, 0u, 0, 0, last_lit,
                                         stage);
}

// `only`: -1 every block; 0 only blocks < 65547 B; 1 only blocks >= 65547 B.
// LZ4M_TABLE_AUTO launches the U16 kernel with 0 and the U32 kernel with 1
// (lz4.c:1352-1357): one kernel holding both parses would need 196 VGPRs.
// ACC1: acceleration 1, the 32-bit search schedule (compress_block_w).
template <int V, bool ACC1>
__global__ __launch_bounds__(64) void compress_kernel(const uint8_t* __restrict__ src,
                                                      const int64_t* __restrict__ src_off,
                                                      const int32_t* __restrict__ src_len, uint8_t* dst,
                                                      const int64_t* __restrict__ dst_off,
                                                      const int32_t* __restrict__ dst_cap,
                                                      int32_t* __restrict__ out_len, int64_t n, int accel, int only) {
    __shared__ __attribute__((aligned(16))) uint16_t tab[8192];
    RING_DECL
    const uint32_t lane = threadIdx.x;
    for (int64_t b = blockIdx.x; b < n; b += gridDim.x) {
        const int64_t len = src_len[b];
        if (only >= 0 && (len >= kLimit64K) != (only == 1)) continue;
        const int64_t r = compress_block<V, ACC1>(src + src_off[b], len, dst + dst_off[b], dst_cap[b], accel, tab, ring,
                                                  lane);
        if (lane == 0) out_len[b] = (int32_t)r;
    }
}

// One lone block of < 65547 bytes (the single-call API, lz4m_host.hip): the
// workgroup's four waves stage the whole block in LDS, then wave 0 runs the
// same parse with every source read -- hash inputs, candidates, catch-up,
// match extension, literals -- from LDS instead of L2/HBM, and writes the
// compressed block into LDS too, so no memory operation of the parse waits
// for a store to reach L2.  A lone block is latency-bound (the skip-ahead
// search waits one round trip per 64 attempts); occupancy does not matter for
// a batch of one, so ~150 KiB of LDS per workgroup is free here.  Output
// bytes are the batched kernel's.
constexpr int kSoloMax = kLimit64K - 1;                  // the U16 table's range (lz4.c:1352)
constexpr int kSoloBuf = ((kSoloMax + 64) + 15) & ~15;   // + zero padding past the block
constexpr int kSoloBound = kSoloMax + kSoloMax / 255 + 16;          // LZ4_compressBound(kSoloMax)
constexpr int kSoloOut = ((kSoloBound + 15) & ~15) + 64;            // + room for 16-byte wild stores
constexpr int kSoloU = 4;   // 16-byte pieces in flight per lane when staging (16 x 64 lanes x 4 = one 4 KiB chunk)
static_assert(16 * 64 * kSoloU == kStageChunk, "a staging round is one chunk");
template <int V, bool ACC1>
__device__ __forceinline__ void compress_solo_body(const uint8_t* __restrict__ src, int32_t len, uint8_t* dst,
                                                   int32_t cap, int32_t* __restrict__ out_len, int accel,
                                                   uint8_t* h_out, int32_t* h_done, uint8_t* blk, uint8_t* obuf,
                                                   uint16_t* tab, lds_u8* ring, int32_t& solo_r, int32_t* last_lit,
                                                   int32_t* stage) {
    const uint32_t t = threadIdx.x;
    constexpr int kStep = 16 * 256;
    const int32_t lim = len + 64 < kSoloBuf ? len + 64 : kSoloBuf;   // the block and 64 zero bytes
    uint32_t* ts = h_done ? reinterpret_cast<uint32_t*>(h_done + 1) : nullptr;   // CallMeta::work (LZ4M_WORKER_TS)
    (void)ts;
    LZ4M_WTS(ts, 0);
    // Waves 1-3 stage the block in 4 KiB chunks (chunk c by wave 1 + c % 3,
    // four 16-byte pieces per lane in flight), each flagged in `stage` once in
    // LDS; wave 0 zeroes the table and parses meanwhile, waiting for a chunk
    // only when it reaches it (lw_need): the PCIe staging overlaps the parse.
    constexpr int kStages = (kSoloBuf + kStageChunk - 1) / kStageChunk;
    static_assert(kStages == kStageFail, "the failure flag follows the chunk flags");
    if (t <= kStages) stage[t] = 0;   // the chunk flags and stage[kStageFail]
    if (t == 0) last_lit[0] = -1;
    __syncthreads();
    const uint32_t wv = t >> 6, ln = t & 63;
    if (wv >= 1) {
        for (int32_t c = (int32_t)wv - 1; c * kStageChunk < lim; c += 3) {
            u32x4 v[kSoloU];
#pragma unroll
            for (int u = 0; u < kSoloU; ++u) {
                const int32_t p = c * kStageChunk + u * 16 * kWave + 16 * (int32_t)ln;
                v[u] = p + 16 <= len ? ld16(src + p) : ld16_guarded(src + p, len - p);
            }
#pragma unroll
            for (int u = 0; u < kSoloU; ++u) {
                const int32_t p = c * kStageChunk + u * 16 * kWave + 16 * (int32_t)ln;
                if (p < lim) lds_st16((lds_u8*)blk + p, v[u]);
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            if (ln == 0) *(lds_vi32*)(stage + c) = 1;
        }
    } else {
        LZ4M_WTS(ts, 1);
        // a capacity at or above the bound parses as "not limited" whatever its
        // size (lz4.c:1330-1343), so the bound is the LDS output's size
        const int32_t bound = len + len / 255 + 16;
        const int64_t r = compress_block<V, ACC1, true>((const uint8_t*)blk, len, obuf, cap < bound ? cap : bound,
                                                        accel, tab, ring, t, last_lit, stage);
        if (t == 0) {
            *out_len = (int32_t)r;
            solo_r = (int32_t)r;
        }
    }
    __syncthreads();
    LZ4M_WTS(ts, 2);
    // the compressed bytes from LDS to the caller's mapped host buffer (or to
    // dst), all four waves: LDS reads and stores only, nothing waits on a
    // store.  The last literals come straight from the staged block.  A
    // staging wait that gave up: no bytes, kSoloStageFail.
    const bool sfail = *(const lds_vi32*)(stage + kStageFail) != 0;
    if (sfail && t == 0) *out_len = kSoloStageFail;
    const int32_t r = sfail ? 0 : solo_r;
    uint8_t* out = h_out != nullptr ? h_out : dst;
    const int32_t split = r > 0 && last_lit[0] >= 0 ? last_lit[0] : r;   // [0, split) in obuf
    for (int32_t p = 16 * (int32_t)t; p < split; p += kStep) {
        const u32x4 v = lds_ld16((const lds_u8*)obuf + p);
        if (p + 16 <= split) {
            st16(out + p, v);
        } else {
            for (int32_t k = p; k < split; ++k) out[k] = obuf[k];
        }
    }
    if (split < r) {
        const lds_u8* lit = (const lds_u8*)blk + last_lit[1];
        uint8_t* o = out + split;
        const int32_t m = r - split;
        for (int32_t p = 16 * (int32_t)t; p < m; p += kStep) {
            const u32x4 v = lds_ld16a(lit + p);
            if (p + 16 <= m) {
                st16(o + p, v);
            } else {
                for (int32_t j = 0; j < m - p; ++j) o[p + j] = (uint8_t)byte_of(v, (int)j);
            }
        }
    }
    if (h_done != nullptr) {   // all of the above visible to the host, then the flag it polls
        // every storing thread releases its own h_out stores at system scope
        // (a workgroup barrier alone does not wait for other waves' stores to
        // reach memory: ADVICE r03); then one thread stores the flag
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
        __syncthreads();
        LZ4M_WTS(ts, 3);
        if (t == 0) __hip_atomic_store(h_done, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// ---------------------------------------------------------------------------
// Blocks with history: lz4.block.compress(dict=) and linked frames.
// ---------------------------------------------------------------------------

using TabU32 = Table<LZ4M_TABLE_U32_HASH5>;
constexpr uint32_t kWin = 65536;   // LZ4 window / LZ4_loadDict's index origin

// lz4.block.compress(source, dict=D) (_block.c:93-107): LZ4_resetStream,
// LZ4_loadDict (lz4.c:1541-1581), LZ4_compress_fast_continue (lz4.c:1684-1701,
// usingExtDict).  dict_len[b] < 0: no dictionary (a reset stream, as
// lz4.block.compress without dict=).  Otherwise the last min(D, 64 KiB) bytes
// of the dictionary sit immediately before the source in `src`.
__global__ __launch_bounds__(64) void compress_dict_kernel(const uint8_t* __restrict__ src,
                                                           const int64_t* __restrict__ src_off,
                                                           const int32_t* __restrict__ src_len,
                                                           const int32_t* __restrict__ dict_len, uint8_t* dst,
                                                           const int64_t* __restrict__ dst_off,
                                                           const int32_t* __restrict__ dst_cap,
                                                           int32_t* __restrict__ out_len, int64_t n, int accel,
                                                           int prefix) {
    __shared__ __attribute__((aligned(16))) uint16_t tab[8192];
    RING_DECL
    uint32_t* t32 = reinterpret_cast<uint32_t*>(tab);
    const uint32_t lane = threadIdx.x;
    for (int64_t b = blockIdx.x; b < n; b += gridDim.x) {
        const int64_t len = src_len[b];
        const int64_t dl = dict_len[b];
        const uint8_t* s = src + src_off[b];
        zero_table(tab, lane);
        // one call site: the three modes differ only in window and index parameters
        const uint8_t* w = s;
        int32_t hist = 0;
        uint32_t ibase = 0, low_idx = 0;
        if (dl >= 0 && dl < 8) {   // no dictionary kept (lz4.c:1564-1566): prefix mode, dictSmall, offset 64 KiB
            ibase = low_idx = kWin;
        } else if (dl >= 8) {
            hist = (int32_t)(dl < (int64_t)kWin ? dl : (int64_t)kWin);
            w = s - hist;
            ibase = low_idx = kWin - (uint32_t)hist;
            // every third position, later positions win (lz4.c:1575-1578)
            for (int32_t p = 3 * (int32_t)lane; p <= hist - 8; p += 3 * kWave)
                atomicMax(&t32[TabU32::hash(w + p)], ibase + (uint32_t)p);
            __builtin_amdgcn_s_waitcnt(0xc07f);
        }
        // catch-up floor of matches inside the block: the block start
        // (usingExtDict, lz4.c:1052-1053) or, in prefix mode, the dictionary
        // start like every other match (lz4.c:967)
        const int32_t low_src = prefix ? 0 : hist;
        const int32_t r = compress_block_w<LZ4M_TABLE_U32_HASH5>(w, hist, (int32_t)len, dst + dst_off[b], dst_cap[b],
                                                                 accel, tab, ring, lane, ibase, low_idx, low_src, 0);
        if (lane == 0) out_len[b] = (int32_t)r;
    }
}

// Linked blocks, serially: one wave per stream (a block with link[b] == 0 and
// the blocks after it with link == 1), the table carried in LDS from block to
// block exactly as LZ4_compress_fast_continue carries it (prefix mode over
// the contiguous source, lz4.c:1665-1675; LZ4F_compressBlock_continue,
// lz4frame.c:865-871).  The 2 GB renormalisation (LZ4_renormDictT,
// lz4.c:1612-1630) is applied as a window shift.
__global__ __launch_bounds__(64) void compress_chain_kernel(const uint8_t* __restrict__ src,
                                                            const int64_t* __restrict__ src_off,
                                                            const int32_t* __restrict__ src_len,
                                                            const int32_t* __restrict__ link, uint8_t* dst,
                                                            const int64_t* __restrict__ dst_off,
                                                            const int32_t* __restrict__ dst_cap,
                                                            int32_t* __restrict__ out_len, int64_t n, int accel) {
    __shared__ __attribute__((aligned(16))) uint16_t tab[8192];
    RING_DECL
    uint32_t* t32 = reinterpret_cast<uint32_t*>(tab);
    const uint32_t lane = threadIdx.x;
    for (int64_t b0 = blockIdx.x; b0 < n; b0 += gridDim.x) {
        if (b0 > 0 && link[b0]) continue;
        zero_table(tab, lane);
        const uint8_t* w = src + src_off[b0];
        uint32_t start = 0;
        for (int64_t b = b0; b < n && (b == b0 || link[b]); ++b) {
            const int64_t len = src_len[b];
            // renormalise well before the reference does (2 GB): the shift
            // never changes a parse, and keeps window positions in int32
            if ((uint64_t)start + (uint64_t)len > 0x40000000ull) {
                const uint32_t delta = start - kWin;
                for (int i = lane; i < 4096; i += kWave) {
                    const uint32_t v = t32[i];
                    t32[i] = v < delta ? 0u : v - delta;
                }
                __builtin_amdgcn_s_waitcnt(0xc07f);
                w += delta;
                start = kWin;
            }
            const int32_t hist = (int32_t)((src + src_off[b]) - w);
            const int32_t r = compress_block_w<LZ4M_TABLE_U32_HASH5>(w, hist, (int32_t)len, dst + dst_off[b], dst_cap[b],
                                                                     accel, tab, ring, lane, 0u, 0u, 0, 0);
            if (lane == 0) out_len[b] = (int32_t)r;
            start += (uint32_t)len;
        }
    }
}

// Linked blocks, speculatively in parallel: one wave per block, passes until
// nothing changes.  A block of a linked stream depends on the stream only
// through the table its predecessor leaves behind, and only through the
// entries of the predecessor itself: every older position is more than 65535
// bytes back when blocks are >= 64 KiB (lz4.c:1062-1065).  Each block runs in
// its own index space -- its window starts 64 KiB before it, its first byte
// has index 65536 -- so every table entry older than its predecessor reads as
// "too far" and a table is handed on by shifting it into the successor's
// index space (entries that become too far are cleared).
//   pass 0: every block compresses from an empty table (speculation);
//   pass j: a block whose predecessor's table changed in pass j-1 compresses
//           again from that table; the others keep their result.
// When a pass changes no table, every block's last run used the table its
// predecessor really leaves, and by induction from the stream's first block
// (a fresh table) every output equals the serial chain's.
// Entries 4k .. 4k+3 of a table in LDS as u32 (V = kTableU17: from the
// split form; lanes 8j .. 8j+7 read one dword of the bit map)
template <int V>
__device__ __forceinline__ u32x4 tab_get4(const uint16_t* tab, int k) {
    if constexpr (V == kTableU17) {
        const uint64_t lo = *(const lds_vu64*)((const lds_u8*)tab + 8 * k);
        const uint32_t m = *(const lds_t32*)(tab + 4096 + 2 * (k >> 3)) >> ((k & 7) * 4);
        return u32x4{(uint32_t)(lo & 0xFFFFu) | ((m & 1u) << 16), (uint32_t)((lo >> 16) & 0xFFFFu) | ((m & 2u) << 15),
                     (uint32_t)((lo >> 32) & 0xFFFFu) | ((m & 4u) << 14), (uint32_t)(lo >> 48) | ((m & 8u) << 13)};
    } else {
        return reinterpret_cast<const u32x4*>(tab)[k];
    }
}

// Store entries 4k .. 4k+3 (values < 2^17 for kTableU17); the whole wave
// calls it with k = lane + 64 i
template <int V>
__device__ __forceinline__ void tab_set4(uint16_t* tab, int k, u32x4 v, uint32_t lane) {
    if constexpr (V == kTableU17) {
        *(lds_vu64*)((lds_u8*)tab + 8 * k) = (uint64_t)((v.x & 0xFFFFu) | (v.y << 16)) |
                                             ((uint64_t)((v.z & 0xFFFFu) | (v.w << 16)) << 32);
        uint32_t m = (((v.x >> 16) & 1u) | ((v.y >> 15) & 2u) | ((v.z >> 14) & 4u) | ((v.w >> 13) & 8u))
                     << ((k & 7) * 4);
        m |= (uint32_t)__shfl_xor((int)m, 1);
        m |= (uint32_t)__shfl_xor((int)m, 2);
        m |= (uint32_t)__shfl_xor((int)m, 4);
        if ((lane & 7u) == 0) *(lds_t32*)(tab + 4096 + 2 * (k >> 3)) = m;
    } else {
        reinterpret_cast<u32x4*>(tab)[k] = v;
    }
}

// V: LZ4M_TABLE_U32_HASH5, or kTableU17 when every block is <= 64 KiB (a
// larger one sets bit 2 of counters[1] and the host runs the U32 kernel)
template <int V>
__global__ __launch_bounds__(64) void compress_spec_kernel(
    const uint8_t* __restrict__ src, const int64_t* __restrict__ src_off, const int32_t* __restrict__ src_len,
    const int32_t* __restrict__ link, uint8_t* dst, const int64_t* __restrict__ dst_off,
    const int32_t* __restrict__ dst_cap, int32_t* __restrict__ out_len, int64_t n, int accel,
    const uint32_t* __restrict__ t_prev, uint32_t* __restrict__ t_cur, const uint8_t* __restrict__ chg_prev,
    uint8_t* __restrict__ chg_cur, int32_t* counters, int pass) {
    constexpr bool U17 = V == kTableU17;
    __shared__ __attribute__((aligned(16))) uint16_t tab[U17 ? kU17Halves : 8192];
    RING_DECL
    u32x4* t4 = reinterpret_cast<u32x4*>(tab);
    const uint32_t lane = threadIdx.x;
    for (int64_t b = blockIdx.x; b < n; b += gridDim.x) {
        const bool linked = b > 0 && link[b] != 0;
        const bool feeds = b + 1 < n && link[b + 1] != 0;   // someone reads this block's table
        const u32x4* mine_prev = reinterpret_cast<const u32x4*>(t_prev + (size_t)b * 4096);
        u32x4* mine_cur = reinterpret_cast<u32x4*>(t_cur + (size_t)b * 4096);
        const bool redo = pass == 0 || (linked && chg_prev[b - 1] != 0);
        if (!redo) {   // input unchanged: keep output and table
            if (feeds)
                for (int k = lane; k < 1024; k += kWave) mine_cur[k] = mine_prev[k];
            if (lane == 0) chg_cur[b] = 0;
            continue;
        }
        const int64_t len = src_len[b];
        int64_t hist = 0;
        if (linked) {
            if (src_len[b - 1] < (int32_t)kWin) {   // speculation needs >= 64 KiB predecessors
                if (lane == 0) {
                    atomicOr(&counters[1], 1);
                    out_len[b] = 0;
                    chg_cur[b] = 0;
                }
                continue;
            }
            hist = kWin;
        }
        if (U17 && hist + len > 2 * (int64_t)kWin) {   // indexes past 2^17: the U32 kernel's job
            if (lane == 0) atomicOr(&counters[1], 2);
            continue;
        }
        if (pass == 0 || !linked) {
            if (U17) {
                for (int k = lane; k < kU17Halves / 8; k += kWave) t4[k] = u32x4{0, 0, 0, 0};
                __builtin_amdgcn_s_waitcnt(0xc07f);
            } else {
                zero_table(tab, lane);
            }
        } else {
            const u32x4* pred = reinterpret_cast<const u32x4*>(t_prev + (size_t)(b - 1) * 4096);
            for (int k = lane; k < 1024; k += kWave) tab_set4<V>(tab, k, pred[k], lane);
            __builtin_amdgcn_s_waitcnt(0xc07f);
        }
        const uint8_t* w = src + src_off[b] - hist;
        const int64_t r = compress_block_w<V>(w, hist, len, dst + dst_off[b], dst_cap[b],
                                              accel, tab, ring, lane, 0u, 0u, 0, 0);
        if (lane == 0) out_len[b] = (int32_t)r;
        if (!feeds) {
            if (lane == 0) chg_cur[b] = 0;
            continue;
        }
        // hand the table on in the successor's index space: index i here is
        // index i - shift there; entries the successor can never use become 0
        const uint32_t shift = (uint32_t)(len + hist) - kWin;
        bool diff = false;
        __builtin_amdgcn_s_waitcnt(0xc07f);
        for (int k = lane; k < 1024; k += kWave) {
            u32x4 v = tab_get4<V>(tab, k);
            v.x = v.x > shift ? v.x - shift : 0u;
            v.y = v.y > shift ? v.y - shift : 0u;
            v.z = v.z > shift ? v.z - shift : 0u;
            v.w = v.w > shift ? v.w - shift : 0u;
            mine_cur[k] = v;
            if (pass != 0) {
                const u32x4 o = mine_prev[k];
                diff |= (o.x != v.x) | (o.y != v.y) | (o.z != v.z) | (o.w != v.w);
            }
        }
        const bool changed = pass == 0 || __ballot(diff) != 0;
        if (lane == 0) {
            chg_cur[b] = changed ? 1 : 0;
            if (changed) atomicAdd(&counters[0], 1);
        }
    }
}

// Late passes of the speculative linked compressor, when few blocks are left
// to redo (pass j >= 1 redoes block b only if b-1's table changed in pass
// j-1; on 4 096 silesia-like blocks 4 095, 1 051, 216, 14 in passes 1-4).
// Such a pass is bound by ONE block's latency: 16.3 ms for a wave that reads
// its candidates and history from L2/HBM.  Here one workgroup per redo block
// stages the block and its 64 KiB of history in LDS (148 KiB with the table
// and ring: one workgroup per CU), and wave 0 runs the same parse with every
// source read from LDS: 13.6 ms.  The serial parse itself (~5 000 cycles per
// sequence, ~6 300 sequences) is what remains.
//   compress_spec_list_kernel: blocks kept as they are hand their table on
//     and the redo blocks are listed (counters[2]);
//   compress_spec_lds_kernel: workgroup i redoes list[i] (grid = the number
//     of tables the previous pass changed, which the host read).
// Outputs, tables and change flags are exactly the batched pass's.
constexpr int32_t kSpecLdsWin = 2 * (int32_t)kWin;   // history + a block of <= 64 KiB

__global__ __launch_bounds__(256) void compress_spec_list_kernel(const int32_t* __restrict__ link, int64_t n,
                                                                 const uint32_t* __restrict__ t_prev,
                                                                 uint32_t* __restrict__ t_cur,
                                                                 const uint8_t* __restrict__ chg_prev,
                                                                 uint8_t* __restrict__ chg_cur, int32_t* counters,
                                                                 int32_t* __restrict__ list) {
    const uint32_t lane = threadIdx.x & 63;
    for (int64_t b = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); b < n; b += (int64_t)gridDim.x * 4) {
        const bool linked = b > 0 && link[b] != 0;
        if (linked && chg_prev[b - 1] != 0) {   // redo: listed for the LDS kernel
            if (lane == 0) list[atomicAdd(&counters[2], 1)] = (int32_t)b;
            continue;
        }
        const bool feeds = b + 1 < n && link[b + 1] != 0;
        const u32x4* mine_prev = reinterpret_cast<const u32x4*>(t_prev + (size_t)b * 4096);
        u32x4* mine_cur = reinterpret_cast<u32x4*>(t_cur + (size_t)b * 4096);
        if (feeds)
            for (int k = lane; k < 1024; k += kWave) mine_cur[k] = mine_prev[k];
        if (lane == 0) chg_cur[b] = 0;
    }
}

__global__ __launch_bounds__(256) void compress_spec_lds_kernel(
    const uint8_t* __restrict__ src, const int64_t* __restrict__ src_off, const int32_t* __restrict__ src_len,
    const int32_t* __restrict__ link, uint8_t* dst, const int64_t* __restrict__ dst_off,
    const int32_t* __restrict__ dst_cap, int32_t* __restrict__ out_len, int64_t n, int accel,
    const uint32_t* __restrict__ t_prev, uint32_t* __restrict__ t_cur, uint8_t* __restrict__ chg_cur,
    int32_t* counters, const int32_t* __restrict__ list) {
    __shared__ __attribute__((aligned(16))) uint8_t win[kSpecLdsWin + 64];
    __shared__ __attribute__((aligned(16))) uint16_t tab[8192];
    __shared__ int32_t diff_any;
    RING_DECL
    u32x4* t4 = reinterpret_cast<u32x4*>(tab);
    const uint32_t t = threadIdx.x, lane = t & 63;
    const int64_t b = list[blockIdx.x];   // linked, b >= 1, its predecessor's table changed
    if (b < 1 || b >= n) return;           // (the host sized the grid from the same count; never taken)
    const bool feeds = b + 1 < n && link[b + 1] != 0;
    const int32_t len = src_len[b];
    if (src_len[b - 1] < (int32_t)kWin) {   // speculation needs >= 64 KiB predecessors (as compress_spec_kernel)
        if (t == 0) {
            atomicOr(&counters[1], 1);
            out_len[b] = 0;
            chg_cur[b] = 0;
        }
        return;
    }
    const int32_t hist = (int32_t)kWin;
    const uint8_t* wg = src + src_off[b] - hist;
    const bool staged = hist + len <= kSpecLdsWin;   // larger blocks parse from memory, as the batched pass
    if (staged) {
        constexpr int kU = 4, kStep = 16 * 256;
        const int32_t lim = hist + len + 64;
        for (int32_t base = 0; base < lim; base += kU * kStep) {
            u32x4 v[kU];
#pragma unroll
            for (int u = 0; u < kU; ++u) {
                const int32_t p = base + u * kStep + 16 * (int32_t)t;
                v[u] = p + 16 <= hist + len ? ld16(wg + p) : ld16_guarded(wg + p, hist + len - p);
            }
#pragma unroll
            for (int u = 0; u < kU; ++u) {
                const int32_t p = base + u * kStep + 16 * (int32_t)t;
                if (p < lim) lds_st16((lds_u8*)win + p, v[u]);
            }
        }
    }
    const u32x4* pred = reinterpret_cast<const u32x4*>(t_prev + (size_t)(b - 1) * 4096);
    for (int k = t; k < 1024; k += 256) t4[k] = pred[k];
    if (t == 0) diff_any = 0;
    __syncthreads();
    if (t < kWave) {
        // two call sites, so that the staged one compiles to LDS instructions
        // (a pointer that may be either is a flat one: every flat load also
        // waits for the wave's stores in flight)
        int64_t r;
        if (staged)
            r = compress_block_w<LZ4M_TABLE_U32_HASH5, false, true>((const uint8_t*)win, hist, len, dst + dst_off[b],
                                                                    dst_cap[b], accel, tab, ring, lane, 0u, 0u, 0, 0);
        else
            r = compress_block_w<LZ4M_TABLE_U32_HASH5>(wg, hist, len, dst + dst_off[b], dst_cap[b], accel, tab, ring,
                                                       lane, 0u, 0u, 0, 0);
        if (lane == 0) out_len[b] = (int32_t)r;
    }
    __syncthreads();
    if (!feeds) {
        if (t == 0) chg_cur[b] = 0;
        return;
    }
    // hand the table on in the successor's index space (as compress_spec_kernel)
    const uint32_t shift = (uint32_t)(len + hist) - kWin;
    const u32x4* mine_prev = reinterpret_cast<const u32x4*>(t_prev + (size_t)b * 4096);
    u32x4* mine_cur = reinterpret_cast<u32x4*>(t_cur + (size_t)b * 4096);
    bool diff = false;
    for (int k = t; k < 1024; k += 256) {
        u32x4 v = t4[k];
        v.x = v.x > shift ? v.x - shift : 0u;
        v.y = v.y > shift ? v.y - shift : 0u;
        v.z = v.z > shift ? v.z - shift : 0u;
        v.w = v.w > shift ? v.w - shift : 0u;
        mine_cur[k] = v;
        const u32x4 o = mine_prev[k];
        diff |= (o.x != v.x) | (o.y != v.y) | (o.z != v.z) | (o.w != v.w);
    }
    if (__ballot(diff) != 0 && lane == 0) diff_any = 1;
    __syncthreads();
    if (t == 0) {
        chg_cur[b] = diff_any ? 1 : 0;
        if (diff_any) atomicAdd(&counters[0], 1);
    }
}


// (the LDS buffers are the caller's: one set for the launch-per-call kernel,
// one set shared by every table variant of the persistent worker)
template <int V, bool ACC1>
__global__ __launch_bounds__(256) void compress_solo_kernel(const uint8_t* __restrict__ src, int32_t len,
                                                            uint8_t* dst, int32_t cap, int32_t* __restrict__ out_len,
                                                            int accel, uint8_t* h_out, int32_t* h_done) {
    __shared__ int32_t solo_r, last_lit[2], stage[kStageFail + 1];
    __shared__ __attribute__((aligned(16))) uint8_t blk[kSoloBuf];
    __shared__ __attribute__((aligned(16))) uint8_t obuf[kSoloOut];
    __shared__ __attribute__((aligned(16))) uint16_t tab[8192];
    RING_DECL
    compress_solo_body<V, ACC1>(src, len, dst, cap, out_len, accel, h_out, h_done, blk, obuf, tab, ring, solo_r,
                                last_lit, stage);
}

// The single-call compress worker (lz4m_worker.h): one persistent workgroup
// serving lone-block compress requests from its mailbox with the solo body;
// the LDS buffers are declared once here and shared by every table variant.
__global__ __launch_bounds__(256) void compress_worker(Mailbox* mb, uint8_t* hd, uint8_t* dbuf, uint64_t idle,
                                                      uint64_t life) {
    __shared__ uint32_t cmd[8];
    __shared__ int32_t solo_r, last_lit[2], stage[kStageFail + 1];
    __shared__ __attribute__((aligned(16))) uint8_t blk[kSoloBuf];
    __shared__ __attribute__((aligned(16))) uint8_t obuf[kSoloOut];
    __shared__ __attribute__((aligned(16))) uint16_t tab[8192];
    RING_DECL
    uint64_t birth = 0;
    uint32_t last = worker_init(mb, cmd, birth);
    for (;;) {
        if (worker_next(mb, last, idle, birth, life, cmd) == 0) break;
        const int32_t rec_off = (int32_t)cmd[1], len = (int32_t)cmd[2], cap = (int32_t)cmd[3];
        const int table = (int)cmd[4];
        int accel = (int)cmd[5];
        if (accel < 1) accel = 1;   // lz4.c:1350-1351
        if (accel > 65537) accel = 65537;
        CallMeta* rec = reinterpret_cast<CallMeta*>(hd + rec_off);
        uint8_t* hout = hd + rec_off + kCallMeta;
        if (table == LZ4M_TABLE_U32_HASH5) {
            if (accel == 1)
                compress_solo_body<LZ4M_TABLE_U32_HASH5, true>(hd, len, dbuf, cap, &rec->result, accel, hout, &rec->done,
                                                              blk, obuf, tab, ring, solo_r, last_lit, stage);
            else
                compress_solo_body<LZ4M_TABLE_U32_HASH5, false>(hd, len, dbuf, cap, &rec->result, accel, hout,
                                                               &rec->done, blk, obuf, tab, ring, solo_r, last_lit, stage);
        } else {   // AUTO / U16: below 65547 bytes the byU16 parse (lz4.c:1352-1357)
            if (accel == 1)
                compress_solo_body<LZ4M_TABLE_U16_HASH4, true>(hd, len, dbuf, cap, &rec->result, accel, hout, &rec->done,
                                                              blk, obuf, tab, ring, solo_r, last_lit, stage);
            else
                compress_solo_body<LZ4M_TABLE_U16_HASH4, false>(hd, len, dbuf, cap, &rec->result, accel, hout,
                                                               &rec->done, blk, obuf, tab, ring, solo_r, last_lit, stage);
        }
    }
}

// ---- the lane-order self-test (the search step's exchange rests on it) ----
// Every wave runs 64 instructions of each exchange form the compressors use
// (ds_wrxchg_rtn_b32 on 32-bit entries, ds_mskor_rtn_b32 on 16-bit halves)
// with pseudo-random bucket collisions, and counts the instructions whose
// lanes did not each read back the nearest lower lane of their bucket.
__global__ __launch_bounds__(256) void lds_order_kernel(uint32_t seed, uint32_t* bad) {
    __shared__ uint32_t tab[4][64];
    const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
    uint32_t nbad = 0;
    for (int it = 0; it < 128; ++it) {
        tab[w][lane] = 0;
        __builtin_amdgcn_s_waitcnt(0xc07f);
        uint32_t x = (seed + 7919u * (uint32_t)it + 104729u * (blockIdx.x * 4u + w)) * 2654435761u ^ (lane * 40503u);
        x ^= x >> 13;
        x *= 0x5bd1e995u;
        x ^= x >> 15;
        const uint32_t nb = 1u << (it & 6);   // 1 .. 64 buckets
        const uint32_t h = x & (nb - 1u);
        uint32_t prev;
        if (it & 1) {
            const uint32_t a = (uint32_t)(uintptr_t)((lds_t16*)&tab[w][0] + h) & ~3u, sh = (h & 1u) * 16u;
            uint32_t old;
            asm volatile("ds_mskor_rtn_b32 %0, %1, %2, %3\n\ts_waitcnt lgkmcnt(0)"
                         : "=v"(old) : "v"(a), "v"(0xFFFFu << sh), "v"((lane + 1u) << sh) : "memory");
            prev = (old >> sh) & 0xFFFFu;
        } else {
            prev = __hip_atomic_exchange((lds_t32*)&tab[w][h], lane + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        uint32_t exp = 0;
        for (int l = 0; l < 64; ++l) {
            const uint32_t hl = (uint32_t)__shfl((int)h, l);
            if (l < (int)lane && hl == h) exp = (uint32_t)l + 1u;
        }
        if (__ballot(prev != exp)) ++nbad;
    }
    if (lane == 0 && nbad) atomicAdd(bad, nbad);
}

}  // namespace lz4m

using namespace lz4m;

extern "C" int lz4m_selftest_lds_order(void) {
    uint32_t* d = nullptr;
    hipStream_t s = nullptr;
    uint32_t h = 0;
    int rc = (int)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    if (rc == 0) rc = (int)hipMalloc(&d, sizeof(uint32_t));
    if (rc == 0) rc = (int)hipMemsetAsync(d, 0, sizeof(uint32_t), s);
    if (rc == 0) {
        hipLaunchKernelGGL(lds_order_kernel, dim3(256), dim3(256), 0, s, 0x9E3779B9u, d);
        rc = (int)hipGetLastError();
    }
    if (rc == 0) rc = (int)hipMemcpyAsync(&h, d, sizeof(uint32_t), hipMemcpyDeviceToHost, s);
    if (rc == 0) rc = (int)hipStreamSynchronize(s);
    if (d) (void)hipFree(d);
    if (s) (void)hipStreamDestroy(s);
    return rc ? -rc : (int)h;
}

// 0 once the current device passed the lane-order self-test; LZ4M_EDEVICE
// once it failed it (the exact compressor would not reproduce the
// reference's bytes).  Run at a device's first compression.  Only a verdict
// is kept (per device ordinal): a HIP error while running the test (no
// memory, a stream capture in progress) is returned as it is, and the next
// call tries again.
static int lds_order_check() {
    constexpr int kMaxDev = 64;
    static std::mutex mu;
    static int verdict[kMaxDev] = {0};   // 0 untested, 1 passed, 2 failed
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDev) dev = 0;
    std::lock_guard<std::mutex> lock(mu);
    if (verdict[dev] == 0) {
        const int r = lz4m_selftest_lds_order();
        if (r < 0) return -r;   // the test did not run: a HIP error, not a verdict
        verdict[dev] = r == 0 ? 1 : 2;
        if (r != 0) fprintf(stderr, "lz4m: LDS lane-order self-test failed on device %d (%d): compression disabled\n", dev, r);
    }
    return verdict[dev] == 1 ? 0 : LZ4M_EDEVICE;
}

extern "C" int lz4m_compress_worker_launch(Mailbox* mb, uint8_t* hd, uint8_t* dbuf, uint64_t idle_ticks,
                                           uint64_t life_ticks, hipStream_t stream) {
    if (const int e = lds_order_check()) return e;
    hipLaunchKernelGGL(compress_worker, dim3(1), dim3(256), 0, stream, mb, hd, dbuf, idle_ticks, life_ticks);
    return (int)hipGetLastError();
}

extern "C" int lz4m_compress_bound(int input_size) {
    if ((unsigned)input_size > (unsigned)kMaxInput) return 0;
    return input_size + input_size / 255 + 16;
}

extern "C" int lz4m_compress_solo(const uint8_t* d_src, int32_t len, uint8_t* d_dst, int32_t cap,
                                  int32_t* d_out_len, int table, int acceleration, uint8_t* h_out,
                                  int32_t* h_done, lz4m_stream_t stream) {
    if (len < 0 || len > kSoloMax || cap < 0) return LZ4M_EINVAL;
    if (const int e = lds_order_check()) return e;
    if (acceleration < 1) acceleration = 1;        // lz4.c:1350-1351
    if (acceleration > 65537) acceleration = 65537;
    hipStream_t s = (hipStream_t)stream;
    auto go = [&](auto v_tag) {
        constexpr int V = decltype(v_tag)::value;
        if (acceleration == 1)
            hipLaunchKernelGGL((compress_solo_kernel<V, true>), dim3(1), dim3(256), 0, s, d_src, len, d_dst, cap,
                               d_out_len, acceleration, h_out, h_done);
        else
            hipLaunchKernelGGL((compress_solo_kernel<V, false>), dim3(1), dim3(256), 0, s, d_src, len, d_dst, cap,
                               d_out_len, acceleration, h_out, h_done);
    };
    switch (table) {
        case LZ4M_TABLE_AUTO:       // len < 65547: the byU16 parse (lz4.c:1352-1357)
        case LZ4M_TABLE_U16_HASH4:
            go(std::integral_constant<int, LZ4M_TABLE_U16_HASH4>{});
            break;
        case LZ4M_TABLE_U32_HASH5:
            go(std::integral_constant<int, LZ4M_TABLE_U32_HASH5>{});
            break;
        default:
            return LZ4M_EINVAL;
    }
    return (int)hipGetLastError();
}

extern "C" int lz4m_compress_batch(const uint8_t* d_src, const int64_t* d_src_off, const int32_t* d_src_len,
                                   uint8_t* d_dst, const int64_t* d_dst_off, const int32_t* d_dst_cap,
                                   int32_t* d_out_len, int64_t n, int table, int acceleration,
                                   lz4m_stream_t stream) {
    if (n < 0) return LZ4M_EINVAL;
    if (n == 0) return 0;
    if (const int e = lds_order_check()) return e;
    if (acceleration < 1) acceleration = 1;        // lz4.c:1350-1351
    if (acceleration > 65537) acceleration = 65537;
    const uint32_t grid = (uint32_t)(n < (1ll << 30) ? n : (1ll << 30));
    hipStream_t s = (hipStream_t)stream;
    // acceleration 1 (the python-lz4 default) runs the 32-bit-schedule instance
    auto exact = [&](auto v_tag, int only) {
        constexpr int V = decltype(v_tag)::value;
        if (acceleration == 1)
            hipLaunchKernelGGL((compress_kernel<V, true>), dim3(grid), dim3(64), 0, s, d_src, d_src_off, d_src_len, d_dst,
                               d_dst_off, d_dst_cap, d_out_len, n, acceleration, only);
        else
            hipLaunchKernelGGL((compress_kernel<V, false>), dim3(grid), dim3(64), 0, s, d_src, d_src_off, d_src_len,
                               d_dst, d_dst_off, d_dst_cap, d_out_len, n, acceleration, only);
    };
    using U16 = std::integral_constant<int, LZ4M_TABLE_U16_HASH4>;
    using U32 = std::integral_constant<int, LZ4M_TABLE_U32_HASH5>;
    switch (table) {
        case LZ4M_TABLE_U16_HASH4:
            exact(U16{}, -1);
            break;
        case LZ4M_TABLE_U32_HASH5:
            exact(U32{}, -1);
            break;
        case LZ4M_PARSE_PARALLEL:
            return pcompress_launch(d_src, d_src_off, d_src_len, d_dst, d_dst_off, d_dst_cap, d_out_len, n, 0, s);
        case LZ4M_PARSE_PARALLEL_HQ:
            return pcompress_launch(d_src, d_src_off, d_src_len, d_dst, d_dst_off, d_dst_cap, d_out_len, n, 1, s);
        case LZ4M_PARSE_PARALLEL_LARGE:
            return pcompress_launch(d_src, d_src_off, d_src_len, d_dst, d_dst_off, d_dst_cap, d_out_len, n, 2, s);
        case LZ4M_TABLE_AUTO:
            exact(U16{}, 0);
            exact(U32{}, 1);
            break;
        default:
            return LZ4M_EINVAL;
    }
    return (int)hipGetLastError();
}

static int compress_dict_launch(const uint8_t* d_src, const int64_t* d_src_off, const int32_t* d_src_len,
                                const int32_t* d_dict_len, uint8_t* d_dst, const int64_t* d_dst_off,
                                const int32_t* d_dst_cap, int32_t* d_out_len, int64_t n, int acceleration,
                                int prefix, lz4m_stream_t stream) {
    if (n < 0) return LZ4M_EINVAL;
    if (n == 0) return 0;
    if (const int e = lds_order_check()) return e;
    if (acceleration < 1) acceleration = 1;
    if (acceleration > 65537) acceleration = 65537;
    const uint32_t grid = (uint32_t)(n < (1ll << 30) ? n : (1ll << 30));
    hipLaunchKernelGGL(compress_dict_kernel, dim3(grid), dim3(64), 0, (hipStream_t)stream, d_src, d_src_off,
                       d_src_len, d_dict_len, d_dst, d_dst_off, d_dst_cap, d_out_len, n, acceleration, prefix);
    return (int)hipGetLastError();
}

extern "C" int lz4m_compress_dict_batch(const uint8_t* d_src, const int64_t* d_src_off, const int32_t* d_src_len,
                                        const int32_t* d_dict_len, uint8_t* d_dst, const int64_t* d_dst_off,
                                        const int32_t* d_dst_cap, int32_t* d_out_len, int64_t n, int acceleration,
                                        lz4m_stream_t stream) {
    return compress_dict_launch(d_src, d_src_off, d_src_len, d_dict_len, d_dst, d_dst_off, d_dst_cap, d_out_len, n,
                                acceleration, 0, stream);
}

extern "C" int lz4m_compress_prefix_batch(const uint8_t* d_src, const int64_t* d_src_off, const int32_t* d_src_len,
                                          const int32_t* d_dict_len, uint8_t* d_dst, const int64_t* d_dst_off,
                                          const int32_t* d_dst_cap, int32_t* d_out_len, int64_t n, int acceleration,
                                          lz4m_stream_t stream) {
    return compress_dict_launch(d_src, d_src_off, d_src_len, d_dict_len, d_dst, d_dst_off, d_dst_cap, d_out_len, n,
                                acceleration, 1, stream);
}

extern "C" int lz4m_compress_prof(unsigned long long* out, int reset) {
    (void)out;
    (void)reset;
    return -1;
}

static thread_local int g_linked_passes = 0;
extern "C" int lz4m_compress_linked_passes(void) { return g_linked_passes; }

extern "C" size_t lz4m_compress_linked_workspace_size(int64_t n) {
    if (n <= 0) return 64;
    return 64 + (size_t)n * 2 * 16384 + (((size_t)n * 2 + 63) & ~(size_t)63) + (size_t)n * 4;
}

// LZ4M_SPEC_LDS: redo counts up to which a pass >= 1 runs the LDS-staged
// kernels (0 = always the batched pass).  Default 256, one workgroup per CU:
// a lone 64 KiB silesia-like block takes 13.6 ms staged against 16.3 ms in
// the batched kernel, but a pass of 1 051 staged blocks (5 rounds of 256 CUs)
// took 46 ms against 20.5 (profiles/r04/r04r_time_linked_*.log)
static int64_t spec_lds_max() {
    const char* e = getenv("LZ4M_SPEC_LDS");   // read per call (tests switch it)
    return e ? (int64_t)atoll(e) : (int64_t)256;
}

extern "C" int lz4m_compress_linked_batch(const uint8_t* d_src, const int64_t* d_src_off, const int32_t* d_src_len,
                                          const int32_t* d_link, uint8_t* d_dst, const int64_t* d_dst_off,
                                          const int32_t* d_dst_cap, int32_t* d_out_len, int64_t n, int acceleration,
                                          int mode, void* d_work, size_t work_bytes, lz4m_stream_t stream) {
    if (n < 0 || (mode != LZ4M_LINKED_SERIAL && mode != LZ4M_LINKED_SPECULATIVE)) return LZ4M_EINVAL;
    if (n == 0) return 0;
    if (mode == LZ4M_LINKED_SPECULATIVE && (d_work == nullptr || work_bytes < lz4m_compress_linked_workspace_size(n)))
        return LZ4M_EINVAL;
    if (const int e = lds_order_check()) return e;
    if (acceleration < 1) acceleration = 1;
    if (acceleration > 65537) acceleration = 65537;
    hipStream_t s = (hipStream_t)stream;
    const uint32_t grid = (uint32_t)(n < (1ll << 30) ? n : (1ll << 30));
    if (mode == LZ4M_LINKED_SERIAL) {
        hipLaunchKernelGGL(compress_chain_kernel, dim3(grid), dim3(64), 0, s, d_src, d_src_off, d_src_len, d_link,
                           d_dst, d_dst_off, d_dst_cap, d_out_len, n, acceleration);
        return (int)hipGetLastError();
    }
    if (d_work == nullptr || work_bytes < lz4m_compress_linked_workspace_size(n)) return LZ4M_EINVAL;
    uint8_t* base = (uint8_t*)d_work;
    int32_t* counters = (int32_t*)base;
    uint32_t* tb[2] = {(uint32_t*)(base + 64), (uint32_t*)(base + 64 + (size_t)n * 16384)};
    uint8_t* cb[2] = {base + 64 + (size_t)n * 32768, base + 64 + (size_t)n * 32768 + (size_t)n};
    int32_t* list = (int32_t*)(base + 64 + (size_t)n * 32768 + (((size_t)n * 2 + 63) & ~(size_t)63));
    int32_t h_counters[3] = {0, 0, 0};
    g_linked_passes = 0;
    const int64_t lds_max = spec_lds_max();
    const bool verbose = getenv("LZ4M_SPEC_VERBOSE") != nullptr;
    // LZ4M_SPEC_U17=0 (A/B): the batched passes keep the 16 KiB u32 table
    bool u17 = [] {
        const char* e = getenv("LZ4M_SPEC_U17");
        return e == nullptr || atoi(e) != 0;
    }();
    // blocks the u32 kernel runs at once (9 workgroups per CU x the CUs)
    static const int64_t u32_fit = [] {
        int dev = 0, cus = 0, per = 0;
        (void)hipGetDevice(&dev);
        (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
        (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(
            &per, reinterpret_cast<const void*>(compress_spec_kernel<LZ4M_TABLE_U32_HASH5>), 64, 0);
        return (int64_t)cus * per;
    }();
    auto t_prev = std::chrono::steady_clock::now();
    for (int64_t pass = 0; pass <= n; ++pass) {
        g_linked_passes = (int)pass + 1;
        hipError_t e = hipMemsetAsync(counters, 0, 12, s);
        if (e != hipSuccess) return (int)e;
        const int cur = (int)(pass & 1), prev = cur ^ 1;
        const int64_t redo = h_counters[0];   // the previous pass's changed tables = this pass's redo blocks
        if (pass > 0 && redo <= lds_max) {
            const uint32_t lgrid = (uint32_t)((n + 3) / 4 < 65536 ? (n + 3) / 4 : 65536);
            hipLaunchKernelGGL(compress_spec_list_kernel, dim3(lgrid), dim3(256), 0, s, d_link, n, tb[prev], tb[cur],
                               cb[prev], cb[cur], counters, list);
            if (redo > 0)
                hipLaunchKernelGGL(compress_spec_lds_kernel, dim3((uint32_t)redo), dim3(256), 0, s, d_src, d_src_off,
                                   d_src_len, d_link, d_dst, d_dst_off, d_dst_cap, d_out_len, n, acceleration,
                                   tb[prev], tb[cur], cb[cur], counters, list);
        } else {
            // the split table pays when the u32 kernel's workgroups do not all fit at once
            // (r05bd: 4 096 blocks 24.2 -> 18.7 ms; 1 180 blocks 14.5 -> 16.6 ms, so not there)
            if (u17 && (pass == 0 || redo > u32_fit))
                hipLaunchKernelGGL(compress_spec_kernel<kTableU17>, dim3(grid), dim3(64), 0, s, d_src, d_src_off,
                                   d_src_len, d_link, d_dst, d_dst_off, d_dst_cap, d_out_len, n, acceleration, tb[prev],
                                   tb[cur], cb[prev], cb[cur], counters, (int)pass);
            else
                hipLaunchKernelGGL(compress_spec_kernel<LZ4M_TABLE_U32_HASH5>, dim3(grid), dim3(64), 0, s, d_src,
                                   d_src_off, d_src_len, d_link, d_dst, d_dst_off, d_dst_cap, d_out_len, n,
                                   acceleration, tb[prev], tb[cur], cb[prev], cb[cur], counters, (int)pass);
        }
        e = hipGetLastError();
        if (e != hipSuccess) return (int)e;
        e = hipMemcpyAsync(h_counters, counters, 12, hipMemcpyDeviceToHost, s);
        if (e == hipSuccess) e = hipStreamSynchronize(s);
        if (e != hipSuccess) return (int)e;
        if (h_counters[1] & 1) return LZ4M_EINVAL;
        if (h_counters[1] & 2) {   // a block over 64 KiB: start again with the U32 table
            u17 = false;
            pass = -1;
            h_counters[0] = 0;
            continue;
        }
        if (verbose) {   // (the host waits for every pass: its wall time is the pass's)
            const auto t_now = std::chrono::steady_clock::now();
            fprintf(stderr, "[lz4m] linked pass %d: %lld redone%s, %d tables changed, %.2f ms\n", (int)pass,
                    (long long)(pass == 0 ? n : redo), pass > 0 && redo <= lds_max ? " (LDS-staged)" : "",
                    h_counters[0], std::chrono::duration<double, std::milli>(t_now - t_prev).count());
            t_prev = t_now;
        }
        if (h_counters[0] == 0) return 0;
    }
    return 0;
}
