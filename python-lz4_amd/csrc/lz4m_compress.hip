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
__device__ __forceinline__ int64_t skip_sum(int64_t m) {
    if (m < 0) return 0;
    const int64_t q = m >> 6, r = m & 63;
    return 32 * q * (q - 1) + q * (r + 1);
}

template <int V>
struct Table;

template <>
struct Table<LZ4M_TABLE_U16_HASH4> {   // 8192 x u16 (lz4.c:756-762, 839-843)
    static constexpr int kEntries = 8192;
    __device__ static __forceinline__ uint32_t hash(const uint8_t* p) {
        return (ld32(p) * 2654435761u) >> (32 - 13);
    }
    __device__ static __forceinline__ uint32_t get(const uint16_t* t, uint32_t h) { return t[h]; }
    __device__ static __forceinline__ void put(uint16_t* t, uint32_t h, uint32_t v) { t[h] = (uint16_t)v; }
    static constexpr bool kDistCheck = false;   // lz4.c:1064, LZ4_DISTANCE_MAX == 65535
};

template <>
struct Table<LZ4M_TABLE_U32_HASH5> {   // 4096 x u32 (lz4.c:764-774, 834-838)
    static constexpr int kEntries = 4096;
    __device__ static __forceinline__ uint32_t hash(const uint8_t* p) {
        return (uint32_t)(((ld64(p) << 24) * 889523592379ull) >> (64 - 12));
    }
    __device__ static __forceinline__ uint32_t get(const uint16_t* t, uint32_t h) {
        return reinterpret_cast<const uint32_t*>(t)[h];
    }
    __device__ static __forceinline__ void put(uint16_t* t, uint32_t h, uint32_t v) {
        reinterpret_cast<uint32_t*>(t)[h] = v;
    }
    static constexpr bool kDistCheck = true;
};

__device__ __forceinline__ uint32_t uni(uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); }
__device__ __forceinline__ int64_t uni64(int64_t v) {
    const uint32_t lo = uni((uint32_t)v), hi = uni((uint32_t)((uint64_t)v >> 32));
    return (int64_t)(((uint64_t)hi << 32) | lo);
}

// Coalesced copy of len bytes (wave-cooperative); never writes past d+d_room
// or reads past s+s_room.
__device__ __forceinline__ void wave_copy(uint8_t* d, const uint8_t* s, int64_t len, int64_t d_room,
                                          int64_t s_room, uint32_t lane) {
    for (int64_t base = 0; base < len; base += 16 * kWave) {
        const int64_t pos = base + 16 * (int64_t)lane;
        if (pos < len) {
            if (len - pos >= 16 || (d_room - pos >= 16 && s_room - pos >= 16)) {
                st16(d + pos, ld16(s + pos));
            } else {
                for (int64_t k = pos; k < len; ++k) d[k] = s[k];
            }
        }
    }
}

// length bytes after a token nibble of 15 (lz4.c:1094-1099, 1184-1194);
// returns the new output position.  Written by lane 0.
__device__ __forceinline__ int64_t put_len(uint8_t* dst, int64_t op, int64_t len, uint32_t lane) {
    const int64_t n255 = len / 255;
    for (int64_t k = lane; k < n255; k += kWave) dst[op + k] = 255;
    if (lane == 0) dst[op + n255] = (uint8_t)(len - 255 * n255);
    return op + n255 + 1;
}

template <int V>
__device__ int64_t compress_block(const uint8_t* __restrict__ src, int64_t n, uint8_t* dst, int64_t cap,
                                  int accel, uint16_t* tab, uint32_t lane) {
    using T = Table<V>;
    if (n > kMaxInput) return 0;                               // lz4.c:1324
    const bool limited = cap < bound64(n);
    if (n == 0) {                                              // lz4.c:1325-1336
        if (limited && cap <= 0) return 0;
        if (lane == 0) dst[0] = 0;
        return 1;
    }
    if (V == LZ4M_TABLE_U16_HASH4 && n >= kLimit64K) return 0;   // lz4.c:963

    const int64_t mflimit1 = n - 12 + 1;                        // lz4.c:942
    const int64_t matchlimit = n - 5;
    const int64_t A = (int64_t)accel << 6;                      // searchMatchNb start
    const int64_t FA = skip_sum(A - 1);
    int64_t anchor = 0, ip = 0, op = 0;

    // fresh table (lz4.c:1513, 1522 / LZ4_prepareTable)
    {
        u32x4* t4 = reinterpret_cast<u32x4*>(tab);
        for (int k = lane; k < 16384 / 16; k += kWave) t4[k] = u32x4{0, 0, 0, 0};
        __builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0)
    }
    if (n < kMinLength) goto last_literals;                    // lz4.c:981

    if (lane == 0) T::put(tab, T::hash(src), 0);               // lz4.c:984
    ip = 1;

    for (;;) {
        int64_t match;
        int64_t tok_pos;
        {   // ---- search (lz4.c:1016-1075), 64 attempts per wave step ----
            int64_t k0 = 0;
            for (;;) {
                const int64_t k = k0 + lane;
                const int64_t pos = ip + (k >= 1 ? 1 + skip_sum(A + k - 2) - FA : 0);
                const int64_t nxt = ip + 1 + skip_sum(A + k - 1) - FA;   // position of attempt k+1
                const bool valid = nxt <= mflimit1;
                const uint64_t vmask = __ballot(valid);
                const int nvalid = __builtin_popcountll(vmask);   // valid lanes are a prefix
                uint32_t h = 0, old = 0;
                if (valid) {
                    h = T::hash(src + pos);
                    old = T::get(tab, h);
                    T::put(tab, h, lane);                      // collision probe
                }
                __builtin_amdgcn_s_waitcnt(0xc07f);
                bool dup = false;
                if (valid) dup = T::get(tab, h) != lane;
                int pred = -1;      // nearest earlier lane with the same hash
                int succ = 1 << 20; // nearest later valid lane with the same hash (none: +inf)
                if (__ballot(dup) != 0) {
                    for (int d = 1; d < nvalid; ++d) {
                        const uint32_t hu = __shfl_up(h, d);
                        const uint32_t hd = __shfl_down(h, d);
                        if (valid && (int)lane >= d && pred < 0 && hu == h) pred = (int)lane - d;
                        if (valid && (int)lane + d < nvalid && succ == (1 << 20) && hd == h) succ = (int)lane + d;
                    }
                }
                const int64_t pred_pos = __shfl(pos, pred < 0 ? (int)lane : pred);
                const int64_t cand = pred >= 0 ? pred_pos : (int64_t)old;
                bool hit = false;
                if (valid) {
                    const bool far = T::kDistCheck && cand + 65535 < pos;
                    hit = !far && ld32(src + cand) == ld32(src + pos);
                }
                const uint64_t hmask = __ballot(hit);
                const int f = hmask ? __builtin_ctzll(hmask) : nvalid;   // last lane processed: f (or all valid)
                // restore lanes after f, then commit lanes <= f (last writer wins)
                if (valid && (int)lane > f) T::put(tab, h, old);
                __builtin_amdgcn_s_waitcnt(0xc07f);
                if (valid && (int)lane <= f && (succ > f)) T::put(tab, h, (uint32_t)pos);
                __builtin_amdgcn_s_waitcnt(0xc07f);
                if (hmask) {
                    ip = __shfl(pos, f);
                    match = __shfl(cand, f);
                    break;
                }
                if (nvalid < kWave) goto last_literals;        // forwardIp > mflimitPlusOne
                k0 += kWave;
            }
            ip = uni64(ip);
            match = uni64(match);
        }

        {   // ---- backward catch-up (lz4.c:1080) ----
            for (;;) {
                const int64_t a = ip - 1 - lane, b = match - 1 - lane;
                const bool ok = a >= anchor && b >= 0 && src[a < 0 ? 0 : a] == src[b < 0 ? 0 : b];
                const uint64_t m = __ballot(ok);
                const int run = ~m == 0 ? kWave : (int)__builtin_ctzll(~m);   // leading lanes that extend
                ip -= run;
                match -= run;
                if (run < kWave) break;
            }
        }

        {   // ---- literal run (lz4.c:1083-1107) ----
            const int64_t lit = ip - anchor;
            tok_pos = op;
            op += 1;
            if (limited && op + lit + (2 + 1 + 5) + lit / 255 > cap) return 0;
            if (lit >= 15) {
                if (lane == 0) dst[tok_pos] = 15 << 4;
                op = put_len(dst, op, lit - 15, lane);
            } else if (lane == 0) {
                dst[tok_pos] = (uint8_t)(lit << 4);
            }
            wave_copy(dst + op, src + anchor, lit, cap - op, n - anchor, lane);
            op += lit;
        }

    next_match:
        {   // ---- offset + match length (lz4.c:1125-1197) ----
            const uint32_t off = (uint32_t)(ip - match);
            if (lane == 0) {
                dst[op] = (uint8_t)off;
                dst[op + 1] = (uint8_t)(off >> 8);
            }
            op += 2;
            // LZ4_count(ip+4, match+4, matchlimit), 4 bytes per lane
            int64_t mcode = 0;
            const int64_t p = ip + 4, q = match + 4;
            for (;;) {
                const int64_t avail = matchlimit - (p + mcode);
                const int64_t at = mcode + 4 * (int64_t)lane;
                const int64_t rem = avail - 4 * (int64_t)lane;   // bytes this lane may compare
                uint32_t x = 0xFFFFFFFFu;   // nonzero = mismatch within range
                int lim = 0;
                if (rem >= 4) {
                    x = ld32(src + p + at) ^ ld32(src + q + at);
                    lim = 4;
                } else if (rem > 0) {
                    uint32_t xa = 0, xb = 0;
                    for (int j = 0; j < (int)rem; ++j) {
                        xa |= (uint32_t)src[p + at + j] << (8 * j);
                        xb |= (uint32_t)src[q + at + j] << (8 * j);
                    }
                    x = xa ^ xb;
                    lim = (int)rem;
                }
                // lane's count of equal leading bytes (0..4), limited by range
                int eq = lim;
                if (x != 0) {
                    const int cz = (int)(__builtin_ctz(x) >> 3);
                    eq = cz < lim ? cz : lim;
                }
                const uint64_t stop = __ballot(eq < 4);
                if (stop == 0) {
                    mcode += 4 * kWave;
                    continue;
                }
                const int fl = __builtin_ctzll(stop);
                mcode += 4 * (int64_t)fl + __shfl(eq, fl);
                break;
            }
            mcode = uni64(mcode);
            ip += mcode + 4;
            if (limited && op + (1 + 5) + (mcode + 240) / 255 > cap) return 0;
            uint32_t tok_lo;
            if (mcode >= 15) {
                tok_lo = 15;
                op = put_len(dst, op, mcode - 15, lane);
            } else {
                tok_lo = (uint32_t)mcode;
            }
            if (lane == 0) dst[tok_pos] = (uint8_t)(dst[tok_pos] + tok_lo);
        }
        anchor = ip;
        if (ip >= mflimit1) break;                             // lz4.c:1204

        {   // ---- fill table, test next position (lz4.c:1207-1258) ----
            if (lane == 0) T::put(tab, T::hash(src + ip - 2), (uint32_t)(ip - 2));
            __builtin_amdgcn_s_waitcnt(0xc07f);
            const uint32_t h = T::hash(src + ip);
            const uint32_t cand = uni(T::get(tab, h));
            __builtin_amdgcn_s_waitcnt(0xc07f);
            if (lane == 0) T::put(tab, h, (uint32_t)ip);
            __builtin_amdgcn_s_waitcnt(0xc07f);
            const bool ok_dist = !T::kDistCheck || (int64_t)cand + 65535 >= ip;
            if (ok_dist && ld32(src + cand) == ld32(src + ip)) {
                match = cand;
                tok_pos = op;
                if (lane == 0) dst[tok_pos] = 0;
                op += 1;
                goto next_match;
            }
        }
        ++ip;
    }

last_literals:
    {   // lz4.c:1266-1293
        const int64_t run = n - anchor;
        if (limited && op + run + 1 + (run + 255 - 15) / 255 > cap) return 0;
        const int64_t tpos = op;
        op += 1;
        if (run >= 15) {
            if (lane == 0) dst[tpos] = 15 << 4;
            op = put_len(dst, op, run - 15, lane);
        } else if (lane == 0) {
            dst[tpos] = (uint8_t)(run << 4);
        }
        wave_copy(dst + op, src + anchor, run, cap - op, n - anchor, lane);
        op += run;
    }
    return op;
}

template <int V>
__global__ __launch_bounds__(64) void compress_kernel(const uint8_t* __restrict__ src,
                                                      const int64_t* __restrict__ src_off,
                                                      const int32_t* __restrict__ src_len, uint8_t* dst,
                                                      const int64_t* __restrict__ dst_off,
                                                      const int32_t* __restrict__ dst_cap,
                                                      int32_t* __restrict__ out_len, int64_t n, int accel) {
    __shared__ __attribute__((aligned(16))) uint16_t tab[8192];
    const uint32_t lane = threadIdx.x;
    for (int64_t b = blockIdx.x; b < n; b += gridDim.x) {
        const int64_t len = src_len[b];
        const int64_t r = compress_block<V>(src + src_off[b], len, dst + dst_off[b], dst_cap[b], accel, tab, lane);
        if (lane == 0) out_len[b] = (int32_t)r;
    }
}

// AUTO: U16 for blocks < 65547 B, U32 otherwise (lz4.c:1352-1357)
__global__ __launch_bounds__(64) void compress_kernel_auto(const uint8_t* __restrict__ src,
                                                           const int64_t* __restrict__ src_off,
                                                           const int32_t* __restrict__ src_len, uint8_t* dst,
                                                           const int64_t* __restrict__ dst_off,
                                                           const int32_t* __restrict__ dst_cap,
                                                           int32_t* __restrict__ out_len, int64_t n, int accel) {
    __shared__ __attribute__((aligned(16))) uint16_t tab[8192];
    const uint32_t lane = threadIdx.x;
    for (int64_t b = blockIdx.x; b < n; b += gridDim.x) {
        const int64_t len = src_len[b];
        int64_t r;
        if (len < kLimit64K)
            r = compress_block<LZ4M_TABLE_U16_HASH4>(src + src_off[b], len, dst + dst_off[b], dst_cap[b], accel,
                                                     tab, lane);
        else
            r = compress_block<LZ4M_TABLE_U32_HASH5>(src + src_off[b], len, dst + dst_off[b], dst_cap[b], accel,
                                                     tab, lane);
        if (lane == 0) out_len[b] = (int32_t)r;
    }
}

}  // namespace lz4m

using namespace lz4m;

extern "C" int lz4m_compress_bound(int input_size) {
    if ((unsigned)input_size > (unsigned)kMaxInput) return 0;
    return input_size + input_size / 255 + 16;
}

extern "C" int lz4m_compress_batch(const uint8_t* d_src, const int64_t* d_src_off, const int32_t* d_src_len,
                                   uint8_t* d_dst, const int64_t* d_dst_off, const int32_t* d_dst_cap,
                                   int32_t* d_out_len, int64_t n, int table, int acceleration,
                                   lz4m_stream_t stream) {
    if (n < 0) return LZ4M_EINVAL;
    if (n == 0) return 0;
    if (acceleration < 1) acceleration = 1;        // lz4.c:1350-1351
    if (acceleration > 65537) acceleration = 65537;
    const uint32_t grid = (uint32_t)(n < (1ll << 30) ? n : (1ll << 30));
    hipStream_t s = (hipStream_t)stream;
    switch (table) {
        case LZ4M_TABLE_U16_HASH4:
            hipLaunchKernelGGL(compress_kernel<LZ4M_TABLE_U16_HASH4>, dim3(grid), dim3(64), 0, s, d_src, d_src_off,
                               d_src_len, d_dst, d_dst_off, d_dst_cap, d_out_len, n, acceleration);
            break;
        case LZ4M_TABLE_U32_HASH5:
            hipLaunchKernelGGL(compress_kernel<LZ4M_TABLE_U32_HASH5>, dim3(grid), dim3(64), 0, s, d_src, d_src_off,
                               d_src_len, d_dst, d_dst_off, d_dst_cap, d_out_len, n, acceleration);
            break;
        case LZ4M_PARSE_PARALLEL:
            return pcompress_launch(d_src, d_src_off, d_src_len, d_dst, d_dst_off, d_dst_cap, d_out_len, n, 0, s);
        case LZ4M_PARSE_PARALLEL_HQ:
            return pcompress_launch(d_src, d_src_off, d_src_len, d_dst, d_dst_off, d_dst_cap, d_out_len, n, 1, s);
        case LZ4M_PARSE_PARALLEL_LARGE:
            return pcompress_launch(d_src, d_src_off, d_src_len, d_dst, d_dst_off, d_dst_cap, d_out_len, n, 2, s);
        case LZ4M_TABLE_AUTO:
            hipLaunchKernelGGL(compress_kernel_auto, dim3(grid), dim3(64), 0, s, d_src, d_src_off, d_src_len, d_dst,
                               d_dst_off, d_dst_cap, d_out_len, n, acceleration);
            break;
        default:
            return LZ4M_EINVAL;
    }
    return (int)hipGetLastError();
}
