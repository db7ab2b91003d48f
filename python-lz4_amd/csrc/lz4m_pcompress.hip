// lz4m_pcompress.hip -- parallel-parse LZ4 block compressor for MI355X (gfx950).
//
// A valid LZ4 block for every input (any lz4libs decoder reads it), at the
// ratio of LZ4_compress_default (measured: -0.02 % size on the synthetic
// corpus; tests bound it at 5 %), but NOT byte-identical to it: the drop-in
// lz4.block / lz4.frame paths keep the exact kernel (lz4m_compress.hip); this
// one serves bulk compression (BASELINE config 3).
//
// Parse = greedy with full insertion: every position p enters a 13-bit hash4
// table (lz4.c:756-762) and its match candidate is the most recent earlier
// position with the same hash; at the parse position the candidate is taken
// if its 4 bytes match (lz4.c:1064-1066), extended forward up to
// matchlimit = n - 5 (LASTLITERALS, lz4.c:943) and backward over pending
// literals (catch-up, lz4.c:1080); matches start at or before n - 12
// (MFLIMIT, lz4.c:942).
//
// Mapping: one wavefront per block (<= 64 KiB, u16 positions in a 16 KiB LDS
// table), 64 consecutive positions per step:
//   1. each lane hashes its position; a 64-key bitonic sort of (hash, lane)
//      gives the nearest earlier lane with the same hash and whether a later
//      lane shares it -- so candidates are exactly "most recent previous
//      occurrence" and the table is updated by one writer per hash;
//   2. every lane verifies its candidate and measures forward (<= 20 B) and
//      backward (<= 4 B) match bytes in parallel: one memory round trip per
//      step, not per sequence;
//   3. the greedy parse walks the ballot mask of verified lanes (scalar);
//   4. the step's sequences are encoded byte-parallel: sizes, a wave prefix
//      sum, then lane t computes output byte t (token, length bytes, literal,
//      offset) -- one coalesced 64-byte store per round.
#include "lz4m_common.h"
#include "../../include/lz4m.h"

namespace lz4m {

constexpr uint32_t kEmpty = 0xFFFFu;

__device__ __forceinline__ uint32_t phash(uint32_t v) { return (v * 2654435761u) >> 19; }

// equal leading bytes of two 16-byte windows (0..16)
__device__ __forceinline__ uint32_t eq_prefix16(u32x4 a, u32x4 b) {
    const uint32_t x0 = a.x ^ b.x, x1 = a.y ^ b.y, x2 = a.z ^ b.z, x3 = a.w ^ b.w;
    if (x0) return __builtin_ctz(x0) >> 3;
    if (x1) return 4 + (__builtin_ctz(x1) >> 3);
    if (x2) return 8 + (__builtin_ctz(x2) >> 3);
    if (x3) return 12 + (__builtin_ctz(x3) >> 3);
    return 16;
}

__device__ __forceinline__ int32_t rdl(int32_t v, int l) { return __builtin_amdgcn_readlane(v, l); }

__device__ __forceinline__ int32_t ext_len(int32_t x) { return x >= 15 ? 1 + (x - 15) / 255 : 0; }

// Wave-cooperative forward match length of s[a..] vs s[c..] (c < a), at most
// `lim` bytes; a + lim <= n - 5, so every 4-byte read stays in the block.
__device__ __forceinline__ int32_t wave_count(const uint8_t* s, int32_t a, int32_t c, int32_t lim, uint32_t lane) {
    for (int32_t done = 0; done < lim; done += 256) {
        const int32_t k = done + 4 * (int32_t)lane;
        int32_t e = 0;   // equal bytes in this lane's dword (4 = all)
        if (k < lim) {
            const uint32_t x = ld32(s + a + k) ^ ld32(s + c + k);
            e = x ? (int32_t)(__builtin_ctz(x) >> 3) : 4;
            const int32_t nb = lim - k < 4 ? lim - k : 4;
            if (e > nb) e = nb;
            if (nb < 4 && e == nb) e = nb;   // reached the limit inside this dword
        }
        const bool full = k + 4 <= lim && e == 4;
        const uint64_t stop = __ballot(!full);
        if (stop == 0) continue;
        const int l = __builtin_ctzll(stop);
        return done + 4 * l + rdl(e, l);
    }
    return lim;
}

// Encode `ns` sequences (lane s < ns holds lstart/lit/off/ml of sequence s;
// ml == 0 marks the final literals-only sequence) at d + op, byte-parallel.
// Returns the bytes written, or -1 if they do not fit before cap.
__device__ __forceinline__ int32_t emit_seqs(const uint8_t* s, uint8_t* d, int32_t op, int32_t cap, int ns,
                                             int32_t lstart, int32_t lit, int32_t off, int32_t ml, uint32_t lane) {
    const bool v = (int)lane < ns;
    const int32_t el = v ? ext_len(lit) : 0;
    const int32_t em = v && ml ? ext_len(ml - 4) : 0;
    const int32_t size = v ? 1 + el + lit + (ml ? 2 + em : 0) : 0;
    // inclusive wave prefix sum
    int32_t inc = size;
#pragma unroll
    for (int k = 1; k < 64; k <<= 1) {
        const int32_t y = __shfl_up(inc, k);
        if ((int)lane >= k) inc += y;
    }
    const int32_t base = inc - size;
    const int32_t total = rdl(inc, ns - 1);
    if (op + total > cap) return -1;
    for (int32_t t0 = 0; t0 < total; t0 += 64) {
        const int32_t t = t0 + (int32_t)lane;
        int sq = 0;
        for (int k = 1; k < ns; ++k)
            if (t >= rdl(base, k)) sq = k;
        const int32_t b = __shfl(base, sq), L = __shfl(lit, sq), O = __shfl(off, sq), M = __shfl(ml, sq),
                      S = __shfl(lstart, sq);
        if (t < total) {
            const int32_t r = t - b;
            const int32_t EL = ext_len(L);
            uint32_t byte;
            if (r == 0) {
                const int32_t ln = L < 15 ? L : 15;
                const int32_t mn = M ? (M - 4 < 15 ? M - 4 : 15) : 0;
                byte = (uint32_t)((ln << 4) | mn);
            } else if (r <= EL) {
                byte = r < EL ? 255u : (uint32_t)((L - 15) % 255);
            } else if (r <= EL + L) {
                byte = s[S + (r - 1 - EL)];
            } else if (r == EL + L + 1) {
                byte = (uint32_t)(O & 0xFF);
            } else if (r == EL + L + 2) {
                byte = (uint32_t)(O >> 8);
            } else {
                const int32_t EM = ext_len(M - 4);
                const int32_t k = r - (EL + L + 3);
                byte = k < EM - 1 ? 255u : (uint32_t)((M - 4 - 15) % 255);
            }
            d[op + t] = (uint8_t)byte;
        }
    }
    return total;
}

__global__ __launch_bounds__(64) void pcompress_kernel(const uint8_t* __restrict__ src,
                                                       const int64_t* __restrict__ src_off,
                                                       const int32_t* __restrict__ src_len, uint8_t* __restrict__ dst,
                                                       const int64_t* __restrict__ dst_off,
                                                       const int32_t* __restrict__ dst_cap,
                                                       int32_t* __restrict__ out_len, int64_t n) {
    __shared__ __attribute__((aligned(16))) uint16_t table[8192];
    const uint32_t lane = threadIdx.x;
    for (int64_t b = blockIdx.x; b < n; b += gridDim.x) {
        const int32_t N = src_len[b];
        const int32_t cap = dst_cap[b];
        const uint8_t* s = src + src_off[b];
        uint8_t* d = dst + dst_off[b];
        if (N < 0 || N > 65536) {   // this kernel handles blocks up to 64 KiB
            if (lane == 0) out_len[b] = 0;
            continue;
        }
        for (int k = (int)lane; k < 8192 / 8; k += 64)
            reinterpret_cast<u32x4*>(table)[k] = u32x4{0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu};
        int32_t anchor = 0, cur = 0, op = 0;
        bool fail = false;
        const int32_t mlast = N - 12;      // last match start (MFLIMIT)
        const int32_t matchlimit = N - 5;  // match end bound (LASTLITERALS)
        for (int32_t p0 = 0; p0 + 4 <= N; p0 += 64) {
            const int32_t p = p0 + (int32_t)lane;
            const bool act = p + 4 <= N;
            const uint32_t v = act ? ld32(s + p) : 0u;
            const uint32_t h = act ? phash(v) : 8192u;
            // ---- nearest earlier / later lane with the same hash: bitonic sort
            uint32_t key = (h << 6) | lane;
#pragma unroll
            for (int k = 2; k <= 64; k <<= 1) {
#pragma unroll
                for (int j = k >> 1; j > 0; j >>= 1) {
                    const uint32_t other = (uint32_t)__shfl_xor((int)key, j);
                    const bool up = (lane & k) == 0;
                    const bool lower = (lane & j) == 0;
                    key = (lower == up) ? (key < other ? key : other) : (key > other ? key : other);
                }
            }
            const uint32_t kprev = (uint32_t)__shfl_up((int)key, 1);
            const uint32_t knext = (uint32_t)__shfl_down((int)key, 1);
            const bool sprev = lane > 0 && (kprev >> 6) == (key >> 6);
            const bool snext = lane < 63 && (knext >> 6) == (key >> 6);
            const uint32_t info = (sprev ? (0x40u | (kprev & 63)) : 0u) | (snext ? 0x80u : 0u);
            // deliver to the original lane (key & 63)
            const uint32_t mine = (uint32_t)__builtin_amdgcn_ds_permute((int)((key & 63) << 2), (int)info);
            // ---- table
            const uint32_t old = act ? table[h] : kEmpty;
            int32_t cand = (mine & 0x40u) ? p0 + (int32_t)(mine & 63) : (old == kEmpty ? -1 : (int32_t)old);
            if (act && !(mine & 0x80u)) table[h] = (uint16_t)p;
            // ---- verify + forward / backward lengths
            bool ok = act && cand >= 0 && p <= mlast;
            int32_t L = 0, back = 0;
            if (ok) ok = ld32(s + cand) == v;
            if (ok) {
                const int32_t lim = matchlimit - p;   // max match length here
                if (lim < 4) {
                    ok = false;
                } else {
                    const u32x4 a = ld16_guarded(s + p + 4, N - p - 4);
                    const u32x4 c = ld16_guarded(s + cand + 4, N - cand - 4);
                    L = 4 + (int32_t)eq_prefix16(a, c);
                    if (L > lim) L = lim;
                    if (cand >= 4) {
                        const uint32_t x = ld32(s + p - 4) ^ ld32(s + cand - 4);
                        back = x ? (int32_t)(__builtin_clz(x) >> 3) : 4;
                    }
                }
            }
            const uint64_t mask = __ballot(ok);
            // ---- greedy parse of this step's positions
            int ns = 0;
            int32_t q_ls = 0, q_lit = 0, q_off = 0, q_ml = 0;   // sequence ns lives in lane ns
            while (cur < p0 + 64 && cur <= mlast) {
                const int32_t rel = cur - p0;
                const uint64_t m = rel <= 0 ? mask : (rel >= 64 ? 0ull : (mask >> rel) << rel);
                if (m == 0) break;
                const int j = __builtin_ctzll(m);
                int32_t st = p0 + j;
                int32_t c = rdl(cand, j);
                int32_t len = rdl(L, j);
                int32_t bk = rdl(back, j);
                const int32_t lim = matchlimit - st;
                if (len == 20 && len < lim) len = 20 + wave_count(s, st + 20, c + 20, lim - 20, lane);
                // catch-up over pending literals (lz4.c:1080)
                if (bk > st - anchor) bk = st - anchor;
                if (bk == 4) {
                    while (st - bk > anchor && c - bk > 0 && s[st - bk - 1] == s[c - bk - 1]) ++bk;
                }
                st -= bk;
                c -= bk;
                len += bk;
                if ((int)lane == ns) {
                    q_ls = anchor;
                    q_lit = st - anchor;
                    q_off = st - c;
                    q_ml = len;
                }
                ++ns;
                cur = st + len;
                anchor = cur;
                if (ns == 64) break;
            }
            if (ns > 0) {
                const int32_t w = emit_seqs(s, d, op, cap, ns, q_ls, q_lit, q_off, q_ml, lane);
                if (w < 0) {
                    fail = true;
                    break;
                }
                op += w;
            }
        }
        if (!fail) {   // last literals (lz4.c:1266-1293)
            const int32_t w = emit_seqs(s, d, op, cap, 1, anchor, N - anchor, 0, 0, lane);
            if (w < 0) {
                fail = true;
            } else {
                op += w;
            }
        }
        if (lane == 0) out_len[b] = fail ? 0 : op;
    }
}

int pcompress_launch(const uint8_t* d_src, const int64_t* d_src_off, const int32_t* d_src_len, uint8_t* d_dst,
                     const int64_t* d_dst_off, const int32_t* d_dst_cap, int32_t* d_out_len, int64_t n,
                     hipStream_t stream) {
    const uint32_t grid = (uint32_t)(n < (1ll << 30) ? n : (1ll << 30));
    hipLaunchKernelGGL(pcompress_kernel, dim3(grid), dim3(64), 0, stream, d_src, d_src_off, d_src_len, d_dst,
                       d_dst_off, d_dst_cap, d_out_len, n);
    return (int)hipGetLastError();
}

}  // namespace lz4m
