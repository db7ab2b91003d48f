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
//   1. each lane hashes its position; one wave ballot per hash bit gives the
//      mask of lanes sharing its hash, hence the nearest earlier lane with
//      the same hash and whether a later lane shares it -- so candidates are
//      exactly "most recent previous occurrence" and the table is updated by
//      one writer per hash;
//   2. every lane verifies its candidate and measures forward (<= 20 B) and
//      backward (<= 4 B) match bytes in parallel: one memory round trip per
//      step, not per sequence;
//   3. the greedy walk over the ballot mask of verified lanes (scalar) only
//      picks the sequence starts; anchors, catch-up, sizes, prefix sums and
//      the compaction of sequence k into lane k run across the wave;
//   4. the step's sequences are encoded byte-parallel: lane t computes output
//      byte t (token, length bytes, literal, offset) -- one coalesced 64-byte
//      store per round.
// The kernel is bound by instruction issue (VALU ~0.75 per CU-cycle, PMC):
// every step above is written to keep both the VALU and the per-CU scalar
// unit short.
#include "lz4m_common.h"

#include <stdlib.h>
#include "../../include/lz4m.h"

namespace lz4m {

constexpr uint32_t kEmpty = 0xFFFFu;

// hash of 4 bytes into HB bits (LZ4_hash4, lz4.c:756-762: 13 bits for the
// byU16 table).  The table is the kernel's whole LDS, and the kernel is
// latency bound: a 12-bit table (8 KB) fits 20 waves per CU instead of 10
// and compresses 1.7x faster for +1.5 % size on the silesia-like mix
// (LZ4M_PARSE_PARALLEL); 13 bits (LZ4M_PARSE_PARALLEL_HQ) keeps the
// reference's table size and ratio (-0.02 %).
template <int HB>
__device__ __forceinline__ uint32_t phash(uint32_t v) { return (v * 2654435761u) >> (32 - HB); }

// equal leading bytes of two 16-byte windows (0..16), branch-free: v_ffbl
// gives ~0u for a zero word, so OR-ing the word's bit base (32 / 64 / 96)
// keeps "no difference" the largest value and one unsigned min over the four
// words finds the first differing bit (the divergent if-chain ran every
// level for the lanes without a candidate, which compare equal windows)
__device__ __forceinline__ uint32_t ffbl(uint32_t x) {
    uint32_t r;
    asm("v_ffbl_b32 %0, %1" : "=v"(r) : "v"(x));   // ~0u for x == 0 (the compiler re-tests zero otherwise)
    return r;
}

__device__ __forceinline__ uint32_t eq_prefix16(u32x4 a, u32x4 b) {
    const uint32_t f0 = ffbl(a.x ^ b.x);
    const uint32_t f1 = ffbl(a.y ^ b.y) | 32u;
    const uint32_t f2 = ffbl(a.z ^ b.z) | 64u;
    const uint32_t f3 = ffbl(a.w ^ b.w) | 96u;
    const uint32_t m = __builtin_elementwise_min(__builtin_elementwise_min(f0, f1), __builtin_elementwise_min(f2, f3));
    return m >= 128u ? 16u : m >> 3;
}

__device__ __forceinline__ int32_t rdl(int32_t v, int l) { return __builtin_amdgcn_readlane(v, l); }

// Mask of the lanes whose HB-bit hash equals this lane's (active lanes only):
// AND over the hash bits of "same bit" masks, each from one wave ballot.
template <int HB>
__device__ __forceinline__ uint64_t same_hash_mask(uint32_t h, bool act) {
    const uint64_t a = __ballot(act);
    uint32_t lo = (uint32_t)a, hi = (uint32_t)(a >> 32);
#pragma unroll
    for (int b = 0; b < HB; ++b) {
        // bit b, replicated, from one v_bfe_i32 that the ballot's compare
        // also reads (written as plain C the compiler turns the compare into
        // a shift + sign test: one VALU more per hash bit; measured +1.6 %)
        uint32_t rep;
        asm("v_bfe_i32 %0, %1, %2, 1" : "=v"(rep) : "v"(h), "i"(b));
        const uint64_t B = __ballot(rep != 0u);
        // mask &= ~(B ^ rep) as one v_bitop3 per half: f(S0, S1, S2) =
        // S1 & (S0 xnor S2), truth table 0x84 (symmetric in S0 / S2)
        lo = __builtin_amdgcn_bitop3_b32((uint32_t)B, lo, rep, 0x84);
        hi = __builtin_amdgcn_bitop3_b32((uint32_t)(B >> 32), hi, rep, 0x84);
    }
    return ((uint64_t)hi << 32) | lo;
}

// y / 255 for y >= 0.  Blocks <= 64 KiB: (z + z/256) / 256 with z = y + 1,
// exact for y < 65 790 (checked exhaustively), two shifts and two adds where
// the division is a quarter-rate v_mul_hi_u32
template <bool BIG>
__device__ __forceinline__ int32_t div255(int32_t y) {
    if (BIG) return y / 255;
    const int32_t z = y + 1;
    return (z + (z >> 8)) >> 8;
}

// length bytes after the token for a length field x (0 below 15)
template <bool BIG>
__device__ __forceinline__ int32_t ext_len(int32_t x) { return x >= 15 ? 1 + div255<BIG>(x - 15) : 0; }

// inclusive prefix sum across the wave: row_shr 1/2/4/8 inside 16-lane rows,
// then row_bcast:15 / row_bcast:31 carry the row totals (VALU only)
__device__ __forceinline__ int32_t wave_incl_sum(int32_t v) {
    v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xF, 0xF, false);   // row_shr:1
    v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xF, 0xF, false);   // row_shr:2
    v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xF, 0xF, false);   // row_shr:4
    v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xF, 0xF, false);   // row_shr:8
    v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xA, 0xF, false);   // row_bcast:15 -> rows 1, 3
    v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xC, 0xF, false);   // row_bcast:31 -> rows 2, 3
    return v;
}

// inclusive prefix max across the wave (v >= 0), as wave_incl_sum
__device__ __forceinline__ int32_t wave_incl_max(int32_t v) {
    v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x111, 0xF, 0xF, false));   // row_shr:1
    v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x112, 0xF, 0xF, false));   // row_shr:2
    v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x114, 0xF, 0xF, false));   // row_shr:4
    v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x118, 0xF, 0xF, false));   // row_shr:8
    v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x142, 0xA, 0xF, false));   // row_bcast:15 -> rows 1, 3
    v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x143, 0xC, 0xF, false));   // row_bcast:31 -> rows 2, 3
    return v;
}

// OR of v over the wave (uniform): inclusive prefix OR as wave_incl_sum, read at lane 63
__device__ __forceinline__ uint32_t wave_or(uint32_t v) {
    v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, false);   // row_shr:1
    v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xF, 0xF, false);   // row_shr:2
    v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xF, 0xF, false);   // row_shr:4
    v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xF, 0xF, false);   // row_shr:8
    v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xA, 0xF, false);   // row_bcast:15 -> rows 1, 3
    v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xC, 0xF, false);   // row_bcast:31 -> rows 2, 3
    return (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
}


// set bits of m in lanes below this one
__device__ __forceinline__ int32_t count_below(uint64_t m) {
    return (int32_t)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// Wave-cooperative forward match length of s[a..] vs s[c..] (c < a), at most
// `lim` bytes; a + lim <= n - 5, so every 4-byte read stays in the block.
__device__ __forceinline__ int32_t wave_count(const uint8_t* s, int32_t a, int32_t c, int32_t lim, uint32_t lane) {
    int32_t done = 0;
    {   // the first 256 bytes: 4 per lane (most long matches end here)
        const int32_t k = 4 * (int32_t)lane;
        int32_t e = 0;   // equal bytes in this lane's dword (4 = all)
        if (k < lim) {
            const uint32_t x = ld32(s + a + k) ^ ld32(s + c + k);
            e = x ? (int32_t)(__builtin_ctz(x) >> 3) : 4;
            const int32_t nb = lim - k < 4 ? lim - k : 4;
            if (e > nb) e = nb;
        }
        const bool full = k + 4 <= lim && e == 4;
        const uint64_t stop = __ballot(!full);
        if (stop != 0) {
            const int l = __builtin_ctzll(stop);
            return 4 * l + rdl(e, l);
        }
        done = 256;
    }
    // past 256 bytes (byte runs, repeated records): 16 bytes per lane, 1 KiB
    // per round trip (r06u: +0.5 % silesia / text, +3 % runs, same output;
    // 16 bytes per lane from the first byte on lost 4 %, r06r)
    for (; done < lim; done += 1024) {
        const int32_t k = done + 16 * (int32_t)lane;
        int32_t e = 0;   // equal bytes in this lane's 16 (16 = all)
        if (k < lim) {
            const int32_t nb = lim - k < 16 ? lim - k : 16;
            const u32x4 x = nb == 16 ? ld16(s + a + k) : ld16_guarded(s + a + k, nb);
            const u32x4 y = nb == 16 ? ld16(s + c + k) : ld16_guarded(s + c + k, nb);
            e = (int32_t)eq_prefix16(x, y);
            if (e > nb) e = nb;
        }
        const bool full = k + 16 <= lim && e == 16;
        const uint64_t stop = __ballot(!full);
        if (stop == 0) continue;
        const int l = __builtin_ctzll(stop);
        return done + 16 * l + rdl(e, l);
    }
    return lim;
}

// Encode `ns` sequences (lane s < ns holds lstart/lit/off/ml of sequence s;
// ml == 0 marks the final literals-only sequence) at d + op, byte-parallel.
// Returns the bytes written, or -1 if they do not fit before cap.
template <bool BIG>
__device__ __forceinline__ int32_t seq_size(int32_t lit, int32_t ml) {
    return 1 + ext_len<BIG>(lit) + lit + (ml ? 2 + ext_len<BIG>(ml - 4) : 0);
}

constexpr int32_t kLongLit = 64;   // literals at least this long are copied 16 B per lane

// Encode the ns sequences held in lanes 0..ns-1 (ml == 0 marks the final
// literals-only sequence) at d + op.  obase = output offset of the sequence;
// pbase = its first index in the "byte-parallel" space, which holds every
// output byte except the literals of long-literal sequences (those are
// copied by the whole wave, 16 bytes per lane).  Short-literal bytes come
// from the registers of the current / previous 64-position chunk (v0 / vprev,
// byte 0 of lane q - p0 is s[q]) when in reach, else from memory.
template <bool BIG>
__device__ __forceinline__ int32_t emit_seqs(const uint8_t* s, uint8_t* d, int32_t op, int32_t cap, int ns,
                                             int32_t lstart, int32_t lit, int32_t off, int32_t ml, int32_t obase,
                                             int32_t pbase, int32_t total, int32_t ptotal, int32_t p0, uint32_t v0,
                                             uint32_t vprev, uint32_t lane) {
    if (op + total > cap) return -1;
    for (int32_t t0 = 0; t0 < ptotal; t0 += 64) {
        const int32_t t = t0 + (int32_t)lane;
        // last sequence k < ns with pbase_k <= t (pbase ascends with k), in
        // ds_bpermute byte-address units (4 k): the sequence k0 covering t0 (pbase_0 = 0), then every sequence that
        // starts inside (t0, t0 + 64) marks its first byte's lane (one forward
        // permute; lanes with no mark send 0 to lane 0, which k0 covers) and a
        // prefix max carries the marks up the wave (one LDS round trip where
        // a 6-step bpermute binary search took six: +0.7-1 %, r06r)
        const bool sin = (int)lane < ns;
        const int k0 = (int)__popcll(__ballot(sin && pbase <= t0)) - 1;
        const int32_t prel = pbase - t0;
        const bool mk = sin && prel > 0 && prel < 64;
        const int32_t got = __builtin_amdgcn_ds_permute((mk ? prel : 0) << 2, mk ? (int)lane + 1 : 0);
        const int sq4 = wave_incl_max(got - 1 > k0 ? got - 1 : k0) << 2;
        const int32_t pb = __builtin_amdgcn_ds_bpermute(sq4, pbase), ob = __builtin_amdgcn_ds_bpermute(sq4, obase),
                      L = __builtin_amdgcn_ds_bpermute(sq4, lit), O = __builtin_amdgcn_ds_bpermute(sq4, off),
                      M = __builtin_amdgcn_ds_bpermute(sq4, ml), S = __builtin_amdgcn_ds_bpermute(sq4, lstart);
        const int32_t EL = ext_len<BIG>(L);
        const bool longlit = L >= kLongLit;
        int32_t r = t - pb;                 // index within the sequence's byte-parallel part
        if (longlit && r > EL) r += L;      // skip the wave-copied literals
        // literal byte source (register window or memory)
        const int32_t q = S + (r - 1 - EL);
        const int32_t rel = q - p0;
        const uint32_t w0 = (uint32_t)__builtin_amdgcn_ds_bpermute((rel & 63) << 2, (int)v0);
        const uint32_t w1 = (uint32_t)__builtin_amdgcn_ds_bpermute((rel & 63) << 2, (int)vprev);
        if (t < ptotal) {
            // every candidate byte, then one select chain (branch-free but for
            // literals outside the two register windows)
            const int32_t ln = L < 15 ? L : 15;
            const int32_t mn = M ? (M - 4 < 15 ? M - 4 : 15) : 0;
            const uint32_t tokb = (uint32_t)((ln << 4) | mn);
            // the last length byte: what the 255s before it leave (no modulo)
            const uint32_t lext = r < EL ? 255u : (uint32_t)(L - 15 - 255 * (EL - 1));
            const int32_t EM = ext_len<BIG>(M - 4);
            const uint32_t mext = r - (EL + L + 3) < EM - 1 ? 255u : (uint32_t)(M - 4 - 15 - 255 * (EM - 1));
            const bool win0 = (uint32_t)rel < 64u, win1 = (uint32_t)(rel + 64) < 64u;
            uint32_t litb = (win0 ? w0 : w1) & 0xFFu;
            if (r > EL && r <= EL + L && !win0 && !win1) litb = s[(uint32_t)q];
            const uint32_t byte = r == 0 ? tokb
                                  : r <= EL ? lext
                                  : r <= EL + L ? litb
                                  : r == EL + L + 1 ? (uint32_t)(O & 0xFF)
                                  : r == EL + L + 2 ? (uint32_t)((O >> 8) & 0xFF)
                                  : mext;
            d[(uint32_t)(op + ob + r)] = (uint8_t)byte;
        }
    }
    // long literals: coalesced 16-byte-per-lane copies
    for (uint64_t lm = __ballot((int)lane < ns && lit >= kLongLit); lm; lm &= lm - 1) {
        const int k = __builtin_ctzll(lm);
        const int32_t L = rdl(lit, k);
        const int32_t S = rdl(lstart, k);
        uint8_t* o = d + op + rdl(obase, k) + 1 + ext_len<BIG>(L);
        for (int32_t x = 16 * (int32_t)lane; x < L; x += 16 * 64) {
            if (x + 16 <= L) {
                st16(o + x, ld16(s + S + x));
            } else {
                for (int32_t y = x; y < L; ++y) o[y] = s[S + y];
            }
        }
    }
    return total;
}

// Bytes [p, p + 4) as a little-endian word, zero past n.
__device__ __forceinline__ uint32_t load_word(const uint8_t* s, int32_t p, int32_t n) {
    if (p + 4 <= n) return ld32(s + (uint32_t)p);
    uint32_t x = 0;
    for (int k = 0; k < 3; ++k)
        if (p + k < n) x |= (uint32_t)s[p + k] << (8 * k);
    return x;
}

// Candidates of one 64-position chunk; the verify loads are issued here and
// consumed by chunk_finish, so their latency overlaps the previous chunk's
// parse and encode.
struct Chunk {
    uint32_t v;       // bytes [p, p + 4) of this lane's position
    int32_t cand;     // candidate position or -1
    bool okc;         // candidate worth verifying
    uint32_t xc;      // bytes at cand
    u32x4 fa, fc;     // 16 bytes after p / after cand
    uint32_t bp, bc;  // 4 bytes before p / before cand
};

// (Measured and not kept, r05n: each lane exchanging its position into its
// bucket -- the lanes of one LDS instruction applied in lane order, as the
// exact compressor's search step does -- in place of the per-hash-bit
// ballots: 0.8 % slower, the 16-bit form's return needing an explicit wait.)

// WIN (blocks > 64 KiB): the table holds the low 16 bits of each position
// (u16, as for blocks <= 64 KiB) instead of whole u32 positions, and a
// candidate is the most recent earlier position with those bits -- inside
// the 64 KiB an offset can reach (lz4.c:1064).  An entry older than that
// aliases to a position in the window; the 4-byte verify takes it only if its
// bytes match, and then it is a valid match like any other.  Half the LDS of
// the u32 table, so twice the waves per CU.
template <bool BIG, int HB, bool WIN = false>
__device__ __forceinline__ void chunk_issue(Chunk& C, const uint8_t* s, uint32_t* table32, int32_t p0, uint32_t v,
                                            int32_t N, int32_t mlast, uint32_t lane) {
    constexpr bool U32 = BIG && !WIN;   // whole positions in a u32 table
    const int32_t p = p0 + (int32_t)lane;
    const bool act = p + 4 <= N;
    const uint32_t h = act ? phash<HB>(v) : (1u << HB);
    // lanes with the same hash (one ballot per hash bit), hence the nearest
    // earlier one (the candidate) and whether a later one exists (then this
    // lane does not write the table)
    const uint64_t eq = same_hash_mask<HB>(h, act);
    const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
    const uint64_t earlier = eq & lt;
    const bool later = (eq >> lane) > 1u;
    uint16_t* table16 = reinterpret_cast<uint16_t*>(table32);
    const uint32_t empty = U32 ? 0xFFFFFFFFu : kEmpty;
    const uint32_t old = act ? (U32 ? table32[h] : (uint32_t)table16[h]) : empty;
    int32_t cand;
    if (earlier) {
        cand = p0 + 63 - (int32_t)__builtin_clzll(earlier);
    } else if (old == empty) {
        cand = -1;
    } else if (WIN) {   // the most recent earlier position with these low 16 bits (none at distance 0)
        const int32_t dd = (p - (int32_t)old) & 0xFFFF;
        cand = dd ? p - dd : -1;
    } else {
        cand = (int32_t)old;
    }
    if (act && !later) {
        if (U32) {
            table32[h] = (uint32_t)p;
        } else {
            table16[h] = (uint16_t)p;
        }
    }
    C.v = v;
    C.cand = cand;
    // LZ4_DISTANCE_MAX (lz4.c:1064): only checkable past 64 KiB
    C.okc = act && cand >= 0 && p <= mlast && (!U32 || p - cand <= 65535);
    // every address stays inside the block (N >= 4 here; p <= mlast when okc)
    const int32_t cs = C.okc ? cand : 0;
    const int32_t ps = C.okc ? p : 0;
    // (unsigned 32-bit offsets: the loads take the block base from SGPRs
    // and skip the per-lane 64-bit address arithmetic)
    C.xc = ld32(s + (uint32_t)cs);
    if (p0 + 84 <= N) {   // every lane's 16 bytes in the block (cand < p): no guard
        C.fa = ld16(s + (uint32_t)(ps + 4));
        C.fc = ld16(s + (uint32_t)(cs + 4));
    } else {
        C.fa = ld16_guarded(s + ps + 4, N - ps - 4);
        C.fc = ld16_guarded(s + cs + 4, N - cs - 4);
    }
    const bool bk = C.okc && cand >= 4;
    C.bp = bk ? ld32(s + (uint32_t)(p - 4)) : 0u;
    C.bc = bk ? ld32(s + (uint32_t)(cand - 4)) : 1u;
}

__device__ __forceinline__ uint64_t chunk_finish(const Chunk& C, int32_t p0, int32_t matchlimit, int32_t& L,
                                                 int32_t& back, uint32_t lane) {
    const int32_t p = p0 + (int32_t)lane;
    const int32_t lim = matchlimit - p;
    const bool ok = C.okc && C.xc == C.v && lim >= 4;
    L = 4 + (int32_t)eq_prefix16(C.fa, C.fc);
    if (L > lim) L = lim;
    const uint32_t x = C.bp ^ C.bc;
    back = C.cand >= 4 ? (x ? (int32_t)(__builtin_clz(x) >> 3) : 4) : 0;
    return __ballot(ok);
}

// SEG (blocks > 64 KiB, lz4m_pcompress_large_batch): a block is parsed as
// up to kSegs segments of >= 256 KiB, one wavefront each, so that a batch of
// few large blocks (config 4: 2 048 x 4 MiB) still fills the chip.  Segment k
// parses [lo, hi) with a fresh table and its own anchor at lo: its matches
// start at or before hi - 4 and end at or before hi (and within the block's
// MFLIMIT / LASTLITERALS, lz4.c:942-943), and a segment other than the last writes no
// last-literals sequence.  Its sequences go to a scratch slot with, in
// seg_meta: bytes written, end anchor, the first sequence's literal length
// (-1: none) and match length.  pcompress_stitch_kernel then joins the slots
// into the block: the literals a segment leaves pending are merged into the
// next first sequence's literal run (its token and length bytes rewritten),
// which is the only place two segments' sequences meet.
constexpr int kSegs = 16;
constexpr int32_t kSegMin = 256 << 10;

__host__ __device__ inline int32_t seg_len(int32_t n) {
    const int32_t q = (int32_t)((((int64_t)n + kSegs - 1) / kSegs + 63) & ~(int64_t)63);
    return q > kSegMin ? q : kSegMin;
}
// scratch bytes of one segment slot (>= LZ4_compressBound of the segment)
__host__ __device__ inline int64_t seg_slot(int32_t seg) { return (((int64_t)seg + seg / 255 + 80) + 15) & ~(int64_t)15; }
// segments of an n-byte block (1..kSegs; non-decreasing in n, so a batch's
// longest block bounds every block's count)
__host__ __device__ inline int32_t seg_count(int32_t n) {
    if (n <= 0) return 1;
    const int32_t seg = seg_len(n);
    return (int32_t)(((int64_t)n + seg - 1) / seg);
}

template <bool BIG, int HB, bool WIN = false, bool SEG = false>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu((BIG && !WIN) || HB > 12 ? 1 : 5))) void pcompress_kernel(const uint8_t* __restrict__ src,
                                                       const int64_t* __restrict__ src_off,
                                                       const int32_t* __restrict__ src_len, uint8_t* __restrict__ dst,
                                                       const int64_t* __restrict__ dst_off,
                                                       const int32_t* __restrict__ dst_cap,
                                                       int32_t* __restrict__ out_len, int64_t n,
                                                       int32_t* __restrict__ seg_meta = nullptr, int64_t seg_cap = 0,
                                                       int32_t segs = 1) {
    static_assert(!SEG || (BIG && WIN), "segments are parsed with the windowed table");
    // 8192 hash4 entries: u16 positions (blocks <= 64 KiB) or u32 (BIG)
    constexpr int kWords = (BIG && !WIN) ? (1 << HB) : (1 << HB) / 2;   // table size in u32 words
    __shared__ __attribute__((aligned(16))) uint32_t table[kWords];
    const uint32_t lane = threadIdx.x;
    const int64_t items = SEG ? n * segs : n;
    for (int64_t b = blockIdx.x; b < items; b += gridDim.x) {
        int32_t N, cap, lo = 0, mlast, matchlimit;
        bool fin = true;
        const uint8_t* s;
        uint8_t* d;
        if (SEG) {
            // block blk's segments take slots blk * segs .. + segs - 1 (segs:
            // the batch's longest block's count)
            const int64_t blk = b / segs;
            const int32_t k = (int32_t)(b % segs), NB = src_len[blk];
            const int32_t seg = NB > 0 ? seg_len(NB) : kSegMin;
            const int64_t lo64 = (int64_t)k * seg;
            const bool badb = NB < 0 || seg_slot(seg) > seg_cap || seg_count(NB) > segs;
            if (badb || (k > 0 && lo64 >= NB)) {   // no such segment / bad block
                if (lane == 0) reinterpret_cast<int4*>(seg_meta)[b] = make_int4(badb ? -1 : 0, 0, -1, 0);
                continue;
            }
            lo = (int32_t)lo64;
            const int32_t hi = NB - lo > seg ? lo + seg : NB;
            fin = hi == NB;
            N = fin || NB - hi < 3 ? NB : hi + 3;   // positions < hi have their 4 hash bytes (inside the block)
            // the block's MFLIMIT / LASTLITERALS bind every segment (a short last segment)
            mlast = fin || hi - 4 > NB - 12 ? NB - 12 : hi - 4;
            matchlimit = fin || hi > NB - 5 ? NB - 5 : hi;
            s = src + src_off[blk];
            d = dst + b * seg_cap;
            cap = (int32_t)seg_cap;
        } else {
            N = src_len[b];
            cap = dst_cap[b];
            s = src + src_off[b];
            d = dst + dst_off[b];
            if (N < 0 || (!BIG && N > 65536)) {   // the u16 table covers blocks up to 64 KiB
                if (lane == 0) out_len[b] = 0;
                continue;
            }
            mlast = N - 12;      // last match start (MFLIMIT)
            matchlimit = N - 5;  // match end bound (LASTLITERALS)
        }
        for (int k = (int)lane; k < kWords / 4; k += 64)
            reinterpret_cast<u32x4*>(table)[k] = u32x4{0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu};
        int32_t anchor = lo, cur = lo, op = 0;
        int32_t f_lit = -1, f_ml = 0;   // SEG: the first sequence's literal and match lengths
        bool fail = false;
        uint32_t vprev = 0;
        Chunk A;
        int32_t L = 0, back = 0;
        uint64_t mask = 0;
        uint32_t wnext = 0;   // the hash word of the chunk after next, loaded a chunk ahead
        if (N - lo >= 4) {
            chunk_issue<BIG, HB, WIN>(A, s, table, lo, load_word(s, lo + (int32_t)lane, N), N, mlast, lane);
            mask = chunk_finish(A, lo, matchlimit, L, back, lane);
            if (lo + 68 <= N) wnext = load_word(s, lo + 64 + (int32_t)lane, N);
        }
        // Per chunk: issue B's loads (and the word of the chunk after B),
        // walk A, finish B, then encode A.  No store sits between a load and
        // its use, so every wait is for loads only (gfx9 counts stores in
        // vmcnt, and a wait behind a variable number of stores is vmcnt(0)).
        for (int32_t p0 = lo; p0 + 4 <= N; p0 += 64) {
            const bool has_next = p0 + 68 <= N;
            Chunk B;
            uint32_t wafter = 0;
            // B's loads are issued after A's walk, whose
            // long-match counts and catch-up loads wait at once (gfx9 counts
            // loads in order: such a wait would also wait for B's)
            auto issue_b = [&]() __attribute__((always_inline)) {
                if (has_next) {
                    chunk_issue<BIG, HB, WIN>(B, s, table, p0 + 64, wnext, N, mlast, lane);
                    if (p0 + 132 <= N) wafter = load_word(s, p0 + 128 + (int32_t)lane, N);
                }
            };
            // ---- greedy parse of chunk p0.  The serial walk only picks the
            // sequence starts: the first verified lane at or after the previous
            // match's end (catch-up moves a start back but not the end).
            // (verified lanes all start at or before mlast, so `rem` -- the
            // verified lanes at or after the walk position -- running empty
            // ends the walk)
            uint64_t chosen = 0;
            int32_t Lx = L;   // match length, extended past 20 for the picked lanes
            const int32_t rel0 = cur - p0;
            uint64_t rem = rel0 <= 0 ? mask : rel0 >= 64 ? 0ull : mask & (~0ull << rel0);
            while (rem) {
                const int j = __builtin_ctzll(rem);
                int32_t len = rdl(L, j);
                if (len == 20 && len < matchlimit - (p0 + j)) {
                    len = 20 + wave_count(s, p0 + j + 20, rdl(A.cand, j) + 20, matchlimit - (p0 + j) - 20, lane);
                    if ((int)lane == j) Lx = len;
                }
                chosen |= 1ull << j;
                const int32_t e = j + len;   // match end, relative to p0
                cur = p0 + e;
                rem = e >= 64 ? 0ull : rem & (~0ull << e);
            }
            const int ns = __builtin_popcountll(chosen);
            int32_t q_ls = 0, q_lit = 0, q_off = 0, q_ml = 0, q_ob = 0, q_pb = 0;   // sequence k in lane k
            int32_t acc = 0, pacc = 0;
            if (ns > 0) {
                // every picked lane at once: its anchor is the previous picked
                // lane's match end (or the carried anchor), then catch-up over
                // the pending literals (lz4.c:1080), sizes, prefix sums, and a
                // compaction of sequence k into lane k
                const bool isch = (chosen >> lane) & 1u;
                const uint64_t below = chosen & (lane ? (~0ull >> (64 - lane)) : 0ull);
                const int32_t p = p0 + (int32_t)lane;
                const int prevl = below ? 63 - __builtin_clzll(below) : 0;
                const int32_t pend = __shfl(p + Lx, prevl);
                const int32_t anc = below ? pend : anchor;
                int32_t st = p, c = A.cand, len = Lx, bk = back;
                if (isch) {
                    if (bk > st - anc) bk = st - anc;
                    if (bk == 4) {
                        while (st - bk > anc && c - bk > 0 && s[st - bk - 1] == s[c - bk - 1]) ++bk;
                    }
                }
                st -= bk;
                c -= bk;
                len += bk;
                const int32_t lit = st - anc;
                const int32_t sz = isch ? seq_size<BIG>(lit, len) : 0;
                const int32_t psz = isch ? (lit >= kLongLit ? sz - lit : sz) : 0;
                int32_t isz, ipsz;
                if (BIG) {
                    isz = wave_incl_sum(sz);
                    ipsz = wave_incl_sum(psz);
                } else {
                    // one scan for both: a step's byte-parallel total stays
                    // far below 2^14 (short literals, tokens, offsets, length
                    // bytes of <= 64 KiB matches) and its output below 2^18
                    const int32_t both = wave_incl_sum((sz << 14) | psz);
                    isz = (int32_t)((uint32_t)both >> 14);
                    ipsz = both & 0x3FFF;
                }
                acc = rdl(isz, 63);
                pacc = rdl(ipsz, 63);
                const int addr = (isch ? count_below(chosen) : 63) << 2;
                q_ls = __builtin_amdgcn_ds_permute(addr, anc);
                q_lit = __builtin_amdgcn_ds_permute(addr, lit);
                q_off = __builtin_amdgcn_ds_permute(addr, st - c);
                q_ml = __builtin_amdgcn_ds_permute(addr, len);
                q_ob = __builtin_amdgcn_ds_permute(addr, isz - sz);
                q_pb = __builtin_amdgcn_ds_permute(addr, ipsz - psz);
                anchor = cur;
            }
            issue_b();
            int32_t LB = 0, backB = 0;
            uint64_t maskB = 0;
            if (ns > 0) {
                if (SEG && f_lit < 0) {
                    f_lit = rdl(q_lit, 0);
                    f_ml = rdl(q_ml, 0);
                }
                const int32_t w = emit_seqs<BIG>(s, d, op, cap, ns, q_ls, q_lit, q_off, q_ml, q_ob, q_pb, acc, pacc, p0,
                                            A.v, vprev, lane);
                if (w < 0) {
                    fail = true;
                    break;
                }
                op += w;
            }
            if (has_next) maskB = chunk_finish(B, p0 + 64, matchlimit, LB, backB, lane);
            if (!has_next) break;
            vprev = A.v;
            A.v = B.v;
            A.cand = B.cand;
            mask = maskB;
            L = LB;
            back = backB;
            wnext = wafter;
        }
        if (!fail && fin) {   // last literals (lz4.c:1266-1293)
            const int32_t lit = N - anchor;
            if (SEG && f_lit < 0) f_lit = lit;
            const int32_t sz = seq_size<BIG>(lit, 0);
            const int32_t w = emit_seqs<BIG>(s, d, op, cap, 1, anchor, lit, 0, 0, 0, 0, sz,
                                        lit >= kLongLit ? sz - lit : sz, 1 << 30, 0u, 0u, lane);
            if (w < 0) {
                fail = true;
            } else {
                op += w;
            }
        }
        if (lane == 0) {
            if (SEG)
                reinterpret_cast<int4*>(seg_meta)[b] = make_int4(fail ? -1 : op, anchor, f_lit, f_ml);
            else
                out_len[b] = fail ? 0 : op;
        }
    }
}

// len bytes from s to d by the wave, 16 per lane, four loads in flight
__device__ __forceinline__ void wave_copy(uint8_t* __restrict__ d, const uint8_t* __restrict__ s, int32_t len,
                                          uint32_t lane) {
    int32_t x = 16 * (int32_t)lane;
    for (; x + 3 * 1024 + 16 <= len; x += 4 * 1024) {
        const u32x4 a = ld16(s + x), b = ld16(s + x + 1024), c = ld16(s + x + 2048), e = ld16(s + x + 3072);
        st16(d + x, a);
        st16(d + x + 1024, b);
        st16(d + x + 2048, c);
        st16(d + x + 3072, e);
    }
    for (; x < len; x += 1024) {
        if (x + 16 <= len) {
            st16(d + x, ld16(s + x));
        } else {
            for (int32_t y = x; y < len; ++y) d[y] = s[y];
        }
    }
}

// Joins a block's segment slots (SEG above): segment k's first sequence
// takes the literals from the previous segments' end anchor c_k (the last
// segment with a sequence before it; 0 for the first), so its token and
// length bytes are rewritten and those literals copied from the source; the
// rest of the slot is copied as it is.  The block fails (0) if a segment
// failed or the joined size exceeds dst_cap.
__global__ __launch_bounds__(64) void pcompress_stitch_kernel(const uint8_t* __restrict__ src,
                                                              const int64_t* __restrict__ src_off,
                                                              const int32_t* __restrict__ src_len,
                                                              uint8_t* __restrict__ dst,
                                                              const int64_t* __restrict__ dst_off,
                                                              const int32_t* __restrict__ dst_cap,
                                                              int32_t* __restrict__ out_len, int64_t n,
                                                              const uint8_t* __restrict__ slots,
                                                              const int32_t* __restrict__ seg_meta, int64_t seg_cap,
                                                              int32_t segs) {
    const uint32_t lane = threadIdx.x;
    for (int64_t b = blockIdx.x; b < n; b += gridDim.x) {
        const int32_t NB = src_len[b];
        if (NB < 0) {
            if (lane == 0) out_len[b] = 0;
            continue;
        }
        const int32_t seg = NB > 0 ? seg_len(NB) : kSegMin;
        const int nseg = seg_count(NB);
        int4 m = make_int4(0, 0, -1, 0);
        if ((int)lane < nseg && (int)lane < segs) m = reinterpret_cast<const int4*>(seg_meta)[b * segs + lane];
        const bool bad = nseg > segs || __ballot((int)lane < nseg && m.x < 0) != 0;
        // c_k: the end anchor of the last segment before k with a sequence
        int32_t c = 0, my_c = 0;
        for (int k = 0; k < nseg; ++k) {
            if ((int)lane == k) my_c = c;
            if (rdl(m.z, k) >= 0) c = rdl(m.y, k);
        }
        int32_t L1 = 0, nk = 0;
        const bool has = (int)lane < nseg && m.z >= 0;
        if (has) {
            L1 = (int32_t)lane * seg + m.z - my_c;   // merged literal run of the first sequence
            nk = 1 + ext_len<true>(L1) + L1 + (m.x - 1 - ext_len<true>(m.z) - m.z);
        }
        const int32_t incl = wave_incl_sum(nk), total = rdl(incl, 63);
        if (bad || total > dst_cap[b]) {
            if (lane == 0) out_len[b] = 0;
            continue;
        }
        const uint8_t* s = src + src_off[b];
        uint8_t* d = dst + dst_off[b];
        for (int k = 0; k < nseg; ++k) {
            if (rdl(m.z, k) < 0) continue;
            const int32_t F = rdl(incl - nk, k), L = rdl(L1, k), ck = rdl(my_c, k), ml = rdl(m.w, k);
            const int32_t l0 = rdl(m.z, k), o = rdl(m.x, k);
            const int32_t E = ext_len<true>(L);
            const uint32_t tok = (uint32_t)(((L < 15 ? L : 15) << 4) | (ml ? (ml - 4 < 15 ? ml - 4 : 15) : 0));
            uint8_t* q = d + F;
            for (int32_t x = (int32_t)lane; x <= E; x += 64)
                q[x] = (uint8_t)(x == 0 ? tok : x < E ? 255u : (uint32_t)(L - 15 - 255 * (E - 1)));
            wave_copy(q + 1 + E, s + ck, L, lane);
            const int32_t h0 = 1 + ext_len<true>(l0) + l0;   // the slot's own first token, length bytes, literals
            wave_copy(q + 1 + E + L, slots + (b * segs + k) * seg_cap + h0, o - h0, lane);
        }
        if (lane == 0) out_len[b] = total;
    }
}

// slots per block = the longest block's segment count (1 for
// blocks up to 256 KiB: ~1x the input, not kSegs x)
extern "C" size_t lz4m_pcompress_large_workspace_size(int64_t n, int32_t max_len) {
    if (n <= 0 || max_len < 0) return 0;
    const int64_t segs = seg_count(max_len);
    const int64_t meta = (n * segs * 16 + 255) & ~(int64_t)255;
    return (size_t)(meta + n * segs * seg_slot(max_len > 0 ? seg_len(max_len) : kSegMin));
}

extern "C" int lz4m_pcompress_large_batch(const uint8_t* d_src, const int64_t* d_src_off, const int32_t* d_src_len,
                                          uint8_t* d_dst, const int64_t* d_dst_off, const int32_t* d_dst_cap,
                                          int32_t* d_out_len, int64_t n, int32_t max_len, void* d_work,
                                          size_t work_bytes, lz4m_stream_t stream) {
    if (n < 0 || max_len < 0) return LZ4M_EINVAL;
    if (n == 0) return 0;
    if (d_work == nullptr || work_bytes < lz4m_pcompress_large_workspace_size(n, max_len)) return LZ4M_EINVAL;
    hipStream_t st = (hipStream_t)stream;
    const int32_t segs = seg_count(max_len);
    int32_t* meta = (int32_t*)d_work;
    uint8_t* slots = (uint8_t*)d_work + ((n * segs * 16 + 255) & ~(int64_t)255);
    const int64_t cap = seg_slot(max_len > 0 ? seg_len(max_len) : kSegMin);
    const int64_t items = n * segs;
    const uint32_t grid = (uint32_t)(items < (1ll << 30) ? items : (1ll << 30));
    // 12 hash bits (r05ba: 13 bits gained 1.9 % ratio at 1.6x the time)
    hipLaunchKernelGGL((pcompress_kernel<true, 12, true, true>), dim3(grid), dim3(64), 0, st, d_src, d_src_off,
                       d_src_len, slots, nullptr, nullptr, nullptr, n, meta, cap, segs);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return (int)e;
    const uint32_t sgrid = (uint32_t)(n < (1ll << 30) ? n : (1ll << 30));
    hipLaunchKernelGGL(pcompress_stitch_kernel, dim3(sgrid), dim3(64), 0, st, d_src, d_src_off, d_src_len, d_dst,
                       d_dst_off, d_dst_cap, d_out_len, n, slots, meta, cap, segs);
    return (int)hipGetLastError();
}

// variant: 0 = blocks <= 64 KiB, 12-bit u16 table; 1 = the same with 13 bits;
// 2 = any block size: a windowed 13-bit u16 table (r05ay: 303 -> 167 ms on
// config 4 against a u32 table, same size)
int pcompress_launch(const uint8_t* d_src, const int64_t* d_src_off, const int32_t* d_src_len, uint8_t* d_dst,
                     const int64_t* d_dst_off, const int32_t* d_dst_cap, int32_t* d_out_len, int64_t n, int variant,
                     hipStream_t stream) {
    const uint32_t grid = (uint32_t)(n < (1ll << 30) ? n : (1ll << 30));
    if (variant == 2) {
        hipLaunchKernelGGL((pcompress_kernel<true, 13, true>), dim3(grid), dim3(64), 0, stream, d_src, d_src_off,
                           d_src_len, d_dst, d_dst_off, d_dst_cap, d_out_len, n);
    } else if (variant == 1) {
        hipLaunchKernelGGL((pcompress_kernel<false, 13>), dim3(grid), dim3(64), 0, stream, d_src, d_src_off,
                           d_src_len, d_dst, d_dst_off, d_dst_cap, d_out_len, n);
    } else {
        hipLaunchKernelGGL((pcompress_kernel<false, 12>), dim3(grid), dim3(64), 0, stream, d_src, d_src_off,
                           d_src_len, d_dst, d_dst_off, d_dst_cap, d_out_len, n);
    }
    return (int)hipGetLastError();
}

}  // namespace lz4m
