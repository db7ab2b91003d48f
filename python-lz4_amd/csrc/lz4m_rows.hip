// lz4m_rows.hip -- the large-batch LZ4 block decoder: parse, then row execution.
//
// Bit-exact restatement of LZ4_decompress_safe (reference lz4libs/lz4.c:
// 1936-2339, fast loop :1996-2109) in three stream-ordered kernels:
//
//  1. rows_parse_kernel  -- one LANE per block walks the token chain only (no
//     copies): for every sequence the reference provably decodes inside its
//     fast loop and without error, it records the sequence's compressed length
//     (one byte; 255 = "long, re-parse it") and stops at the first sequence
//     that is not such ("good") -- the block's tail, or any error.  A serial
//     parse costs a lane ~25 instructions per sequence, 64 blocks per wave.
//  2. rows_exec_kernel   -- one 16-lane ROW per block (4 blocks per wave):
//     round after round, lane j of the row takes the row's next sequence j,
//     its start found by a row prefix sum of the recorded lengths (no
//     speculative parse, no chain walk).  Output is assembled in the row's
//     LDS history buffer (the block's last 1-2 KiB of output); a DPP prefix sum
//     places each sequence, literals are written, and matches are copied in
//     readiness passes (a match waits while an earlier pending match of the
//     same round writes into its source; rounds of 16 keep those chains ~3
//     deep).  Sources older than the buffer come from HBM (the block's own
//     flushed output).  Finished 16-byte chunks leave for HBM in one coalesced
//     store per row and round.
//  3. the finisher (decompress_kernel<false, true>, lz4m_decompress.hip) --
//     one lane per block resumes the reference's exact state machine at the
//     first non-good sequence, so the tail, errors and error positions are the
//     reference's.
//
// Scratch (caller-provided, lz4m_decompress_workspace_size): counters, one
// 32-byte record per block, and the per-block length bytes (<= one per three
// compressed bytes).  A block whose length bytes do not fit is decoded by the
// finisher alone (correct, slower).
#include "lz4m_common.h"
#include "lz4m_rows.h"

#include <limits.h>

namespace lz4m {
typedef __attribute__((address_space(3))) u32x4 lds_u32x4;

// s_waitcnt vmcnt(0) (expcnt and lgkmcnt left at their maximum)
__device__ __forceinline__ void wait_vm0() { __builtin_amdgcn_s_waitcnt(0x0F70); }

// ------------------------------------------------------------- row helpers
// A row = 16 consecutive lanes; DPP row_shr stays inside a row and
// row_newbcast:n (gfx90a+) broadcasts lane n of each row to the whole row.
__device__ __forceinline__ int32_t row_incl_sum(int32_t v) {
    v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xF, 0xF, false);   // row_shr:1
    v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xF, 0xF, false);   // row_shr:2
    v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xF, 0xF, false);   // row_shr:4
    v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xF, 0xF, false);   // row_shr:8
    return v;
}
// two inclusive row prefix sums at once (the chains interleave: no wait
// states between dependent DPP steps)
__device__ __forceinline__ void row_incl_sum2(int32_t& a, int32_t& b) {
    a += __builtin_amdgcn_update_dpp(0, a, 0x111, 0xF, 0xF, false);
    b += __builtin_amdgcn_update_dpp(0, b, 0x111, 0xF, 0xF, false);
    a += __builtin_amdgcn_update_dpp(0, a, 0x112, 0xF, 0xF, false);
    b += __builtin_amdgcn_update_dpp(0, b, 0x112, 0xF, 0xF, false);
    a += __builtin_amdgcn_update_dpp(0, a, 0x114, 0xF, 0xF, false);
    b += __builtin_amdgcn_update_dpp(0, b, 0x114, 0xF, 0xF, false);
    a += __builtin_amdgcn_update_dpp(0, a, 0x118, 0xF, 0xF, false);
    b += __builtin_amdgcn_update_dpp(0, b, 0x118, 0xF, 0xF, false);
}
__device__ __forceinline__ int32_t row_last(int32_t v) { return __builtin_amdgcn_update_dpp(0, v, 0x15F, 0xF, 0xF, false); }
__device__ __forceinline__ int32_t row_first(int32_t v) { return __builtin_amdgcn_update_dpp(0, v, 0x150, 0xF, 0xF, false); }

// max of v over the lanes below in the row (-1 for lane 0); v >= -1
__device__ __forceinline__ int32_t row_excl_max(int32_t v) {
    int32_t x = __builtin_amdgcn_update_dpp(-1, v, 0x111, 0xF, 0xF, false);
    x = max(x, __builtin_amdgcn_update_dpp(-1, x, 0x111, 0xF, 0xF, false));
    x = max(x, __builtin_amdgcn_update_dpp(-1, x, 0x112, 0xF, 0xF, false));
    x = max(x, __builtin_amdgcn_update_dpp(-1, x, 0x114, 0xF, 0xF, false));
    x = max(x, __builtin_amdgcn_update_dpp(-1, x, 0x118, 0xF, 0xF, false));
    return x;
}
// min of v over the lanes below in the row (INT_MAX for lane 0)
__device__ __forceinline__ int32_t row_excl_min(int32_t v) {
    int32_t x = __builtin_amdgcn_update_dpp(INT_MAX, v, 0x111, 0xF, 0xF, false);
    x = min(x, __builtin_amdgcn_update_dpp(INT_MAX, x, 0x111, 0xF, 0xF, false));
    x = min(x, __builtin_amdgcn_update_dpp(INT_MAX, x, 0x112, 0xF, 0xF, false));
    x = min(x, __builtin_amdgcn_update_dpp(INT_MAX, x, 0x114, 0xF, 0xF, false));
    x = min(x, __builtin_amdgcn_update_dpp(INT_MAX, x, 0x118, 0xF, 0xF, false));
    return x;
}

// Two exclusive max-scans over the row at once (values >= 0, 0 = none):
// max of a and of b over the lanes below (0 for lane 0).  Identity 0 lets
// each step fold into one v_max_i32_dpp; the two chains interleave.
__device__ __forceinline__ void row_excl_max2(int32_t a, int32_t b, int32_t& xa, int32_t& xb) {
    int32_t x = __builtin_amdgcn_update_dpp(0, a, 0x111, 0xF, 0xF, false);
    int32_t y = __builtin_amdgcn_update_dpp(0, b, 0x111, 0xF, 0xF, false);
    x = max(x, __builtin_amdgcn_update_dpp(0, x, 0x111, 0xF, 0xF, false));
    y = max(y, __builtin_amdgcn_update_dpp(0, y, 0x111, 0xF, 0xF, false));
    x = max(x, __builtin_amdgcn_update_dpp(0, x, 0x112, 0xF, 0xF, false));
    y = max(y, __builtin_amdgcn_update_dpp(0, y, 0x112, 0xF, 0xF, false));
    x = max(x, __builtin_amdgcn_update_dpp(0, x, 0x114, 0xF, 0xF, false));
    y = max(y, __builtin_amdgcn_update_dpp(0, y, 0x114, 0xF, 0xF, false));
    x = max(x, __builtin_amdgcn_update_dpp(0, x, 0x118, 0xF, 0xF, false));
    y = max(y, __builtin_amdgcn_update_dpp(0, y, 0x118, 0xF, 0xF, false));
    xa = x;
    xb = y;
}

// Exactly k bytes (k >= 16: 16) of v at global address p.
__device__ __forceinline__ void gbl_put(uint8_t* p, u32x4 v, int32_t k) {
    if (k >= 16) {
        st16(p, v);
        return;
    }
    if (k <= 0) return;
    uint32_t o = 0;
    if (k & 8) {
        const uint64_t x = ((uint64_t)v.y << 32) | v.x;
        __builtin_memcpy(p, &x, 8);
        o = 8;
    }
    if (k & 4) {
        const uint32_t x = window_dword(v, o);
        __builtin_memcpy(p + o, &x, 4);
        o += 4;
    }
    if (k & 2) {
        const uint16_t x = (uint16_t)window_dword(v, o);
        __builtin_memcpy(p + o, &x, 2);
        o += 2;
    }
    if (k & 1) p[o] = (uint8_t)window_dword(v, o);
}

// the 4 bytes at k (0..28) of the 32-byte window a|b, the dwords selected by
// a tree on the index bits
__device__ __forceinline__ uint32_t dword32_tree(u32x4 a, u32x4 b, uint32_t k) {
    const uint32_t q = k >> 2;
    const bool q1 = (q & 1u) != 0, q2 = (q & 2u) != 0, q4 = (q & 4u) != 0;
    // dword q: pairs (x, y), (z, w) of a and b by bit 0, then by bit 1, then bit 2
    const uint32_t l0 = q1 ? a.y : a.x, l1 = q1 ? a.w : a.z, l2 = q1 ? b.y : b.x, l3 = q1 ? b.w : b.z;
    const uint32_t lo = q4 ? (q2 ? l3 : l2) : (q2 ? l1 : l0);
    // dword q + 1 (0 past the window)
    const uint32_t h0 = q1 ? a.z : a.y, h1 = q1 ? b.x : a.w, h2 = q1 ? b.z : b.y, h3 = q1 ? 0u : b.w;
    const uint32_t hi = q4 ? (q2 ? h3 : h2) : (q2 ? h1 : h0);
    return __builtin_amdgcn_alignbyte(hi, lo, k & 3);
}


// ------------------------------------------------------------ 1. the parse
// One lane per block.  The compressed block is read through a 128-byte LDS
// ring per lane holding stream bytes [wb, wb + 128) (wb a multiple of 64; a
// 16-byte read wraps per aligned 8-byte piece), and the
// next 64 bytes [wb + 128, wb + 192) are requested ahead into registers.  The
// inner loop is the common sequence only -- literal <= 12 bytes, at most one
// match-length byte, inside the ring, good -- as straight-line code: the
// token byte, then the aligned dword pair holding offset and length byte (two
// dependent LDS reads, ~30 VALU and ~9 SALU per step; the round-5 step read
// 16 bytes and selected from them: ~65 VALU, ~33 SALU, r06l/m: 24.3 -> 20.1
// ms per 1 M probe blocks).  A lane that meets anything else (the ring's
// end, a longer literal or length, a full length stage, the block's end)
// stops; once too few lanes go on, the wave runs one general step: every
// lane past the first half of its ring rotates the requested bytes in and
// requests the next 64, waiting lanes parse one sequence with the general
// parse.  Recorded lengths are staged in a 32-entry LDS ring per lane and
// leave for HBM 16 at a time.  The ring refills are loaded by four lanes per
// block (one 64-byte request instead of four 16-byte ones).
constexpr int kPW = 128;                // ring bytes
typedef __attribute__((address_space(3))) volatile uint8_t lds_vu8;
typedef __attribute__((address_space(3))) volatile uint32_t lds_vu32;
constexpr int kPStage = 32;   // length ring (flushed in halves)
constexpr int kPWG = 64;      // parse workgroup (LDS is allocated per workgroup)
// a 64-bit address received from another lane, as a global pointer
__device__ __forceinline__ const uint8_t* readlane_safe_ptr(uint64_t a) {
    typedef __attribute__((address_space(1))) const uint8_t gu8;
    return (const uint8_t*)(gu8*)(uintptr_t)a;
}
constexpr int32_t kPRunCap = 16;        // length-byte runs longer than this end the good prefix (finisher)
constexpr int kPMinActive = 40;         // run the general step once fewer lanes than this can go on
constexpr int kPSteps = 4;              // fast steps per count of the lanes going (r06m: 20.60 ms, 2: 20.64)

// 64 stream bytes into ring half h (0: offsets 0-63; 1: 64-127)
__device__ __forceinline__ void ring_put(lds_u8* W, int32_t h, const u32x4* v) {
#pragma unroll
    for (int c = 0; c < 4; ++c) lds_st16(W + 64 * h + 16 * c, v[c]);
}

__device__ __forceinline__ void load64(const uint8_t* s, int32_t x, int32_t iend, u32x4* v) {
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        const int32_t y = x + 16 * c;
        v[c] = y + 16 <= iend ? ld16(s + y) : ld16_guarded(s + y, iend - y);
    }
}

// Whole-literal blocks (an incompressible block: one sequence whose literal
// runs exactly to the block's end) are decoded here, by the wave: the
// reference reads the literal length (read_variable_length(&ip, iend - 15, 1),
// lz4.c:1903-1928: every run byte read leaves ip <= iend - 15), finds
// ip + length > iend - 32 and takes the last-literals branch (lz4.c:2172-2229),
// whose result is `length` exactly when ip + length == iend and
// length <= oend.  The candidate lane f's block is checked here with those
// tests (anything else is left to the finisher, as before) and its literal
// copied by the wave, 8 KiB per round trip; the result is the decoded size
// (-1: not such a block), which the lane records as meta ip = -1 (done), op =
// the size.  The copy overlaps the other waves' parsing, which is
// latency-bound; in the finisher it ran at the device's copy rate after the
// row execution (~2.4 ms of the headline launch's 4 ms finisher).
__device__ __forceinline__ int64_t whole_literal_block(const uint8_t* s, int32_t iend, int32_t oend, uint8_t* d,
                                                       uint32_t lane) {
    typedef __attribute__((address_space(1))) const uint8_t gu8;
    // the token and the length-byte run: bytes [0, 1024), 16 per lane
    const int32_t y = 16 * (int32_t)lane;
    const u32x4 v = y + 16 <= iend ? ld16(s + y) : ld16_guarded(s + y, iend - y);
    const uint32_t tok = (uint32_t)__builtin_amdgcn_readlane((int32_t)v.x, 0) & 0xFFu;   // byte 0: lane 0's
    // the first byte other than 255 at position >= 1 in this lane's 16
    int32_t first = 16;
    for (int b = 15; b >= 0; --b)
        if (byte_of(v, b) != 255u && (lane != 0 || b != 0)) first = b;
    const uint64_t nz = __ballot(first < 16 && y + first < iend);
    if ((tok >> 4) != 15u || nz == 0) return -1;
    const int fl = __builtin_ctzll(nz);
    const int32_t pe = 16 * fl + __builtin_amdgcn_readlane(first, fl);   // the run's last byte
    const uint32_t bt = (uint32_t)__builtin_amdgcn_readlane((int32_t)byte_of(v, first & 15), fl);
    const int64_t L = 15 + 255 * (int64_t)(pe - 1) + bt;
    const int32_t q = pe + 1;
    if (q > iend - 15 || q + L != (int64_t)iend || L > oend) return -1;
    // (uniform bases, 32-bit lane offsets: 4 loads in flight per lane)
    const uint8_t* cs = (const uint8_t*)(gu8*)(s + q);
    const uint32_t Lf = (uint32_t)L & ~15u;   // whole 16-byte pieces
    for (uint32_t b = 0; b < Lf; b += 4096) {
        u32x4 w[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const uint32_t p = b + 1024u * u + (uint32_t)y;
            if (p < Lf) w[u] = ld16(cs + p);
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const uint32_t p = b + 1024u * u + (uint32_t)y;
            if (p < Lf) st16(d + p, w[u]);
        }
    }
    if ((uint32_t)L != Lf && lane == ((Lf >> 4) & 63u)) gbl_put(d + Lf, ld16_guarded(cs + Lf, (int32_t)L - (int32_t)Lf), (int32_t)L - (int32_t)Lf);
    return L;
}

__global__ __launch_bounds__(kPWG) void rows_parse_kernel(const uint8_t* __restrict__ src,
                                                         const int64_t* __restrict__ src_off,
                                                         const int32_t* __restrict__ src_len,
                                                         uint8_t* __restrict__ dst,
                                                         const int64_t* __restrict__ dst_off,
                                                         const int32_t* __restrict__ dst_cap, int64_t n,
                                                         RowMeta* __restrict__ meta, uint8_t* __restrict__ lens,
                                                         int64_t lens_cap, unsigned long long* __restrict__ ctr) {
    __shared__ __attribute__((aligned(kPW))) uint8_t wins[kPWG * kPW];
    __shared__ __attribute__((aligned(kPStage))) uint8_t stgs[kPWG * kPStage];
    const uint32_t lane = lane_id();
    lds_u8* W = (lds_u8*)(wins + threadIdx.x * kPW);
    const uint32_t Wa = (uint32_t)(uintptr_t)W;   // kPW-aligned: ring offsets are OR-ed in
    lds_u8* stg = (lds_u8*)(stgs + threadIdx.x * kPStage);
    const uint32_t Sa = (uint32_t)(uintptr_t)stg;   // (kPStage-aligned)
    const uint8_t* s = nullptr;
    int64_t idx = -1, loff = 0;
    int32_t iend = 0, oend = 0, ip = 0, op = 0, k = 0, kf = 0, wb = 0, sh = 0;
    u32x4 pf[4];   // stream bytes [wb + 128, wb + 192), requested ahead
    bool live = false, need = false, more = true, pfv = false, stall = false;
    while (true) {
        if (more) {
            // idle lanes take the next blocks: one queue atomic and one
            // length-space atomic per wave refill
            const uint64_t idle = __ballot(!live);
            if (idle != 0 && (uint32_t)__popcll(idle) >= 8u) {
                const int first = __builtin_ctzll(idle);
                const uint32_t cnt = (uint32_t)__popcll(idle);
                unsigned long long qb = 0;
                if ((int)lane == first) qb = atomicAdd(&ctr[0], (unsigned long long)cnt);
                qb = (unsigned long long)readlane64((int64_t)qb, first);
                if (qb + cnt >= (unsigned long long)n) more = false;
                int64_t wantb = 0;
                bool fresh = false;
                if (!live) {
                    const uint64_t below = lane == 0 ? 0 : (idle & (~0ull >> (64 - lane)));
                    idx = (int64_t)(qb + (unsigned long long)__popcll(below));
                    if (idx < n) {
                        // block positions are kept shifted by sh = the block's
                        // offset in its 64-byte line, so that every ring refill is
                        // one aligned 64-byte piece (not two partial ones); the
                        // bytes before the block are read, never parsed -- only
                        // where they lie inside the caller's buffer
                        const int64_t so = src_off[idx];
                        const int32_t il = src_len[idx];
                        sh = (int32_t)((uintptr_t)(src + so) & 63u);
                        if (so < sh) sh = 0;
                        s = src + so - sh;
                        iend = il + sh;
                        oend = dst_cap[idx];
                        ip = sh;
                        op = k = kf = 0;
                        wb = -4 * kPW;
                        pfv = false;
                        if (oend >= 64 && il > 0) {   // else: no fast loop (lz4.c:1990-1993) or a special case
                            // a good sequence takes >= 3 input and >= 4 output bytes;
                            // rounded up to 16 so that every 16-byte length store is
                            // aligned inside one 128-byte line (unaligned ones,
                            // straddling two lines, cost the parse 1.5 ms per 1 M
                            // blocks, r06zo)
                            const int32_t a = il / 3, b = oend / 4;
                            wantb = ((int64_t)(a < b ? a : b) + 1 + 15) & ~(int64_t)15;
                            fresh = true;
                        } else {
                            meta[idx] = RowMeta{0, 0, 0, 0, 0, 0};
                        }
                    }
                }
                int64_t incl = wantb;
#pragma unroll
                for (int dd = 1; dd < 64; dd <<= 1) {
                    const int64_t t = __shfl_up(incl, dd);
                    if ((int)lane >= dd) incl += t;
                }
                const int64_t total = readlane64(incl, 63);
                int64_t abase = 0;
                if (total > 0) {
                    if (lane == 0) abase = (int64_t)atomicAdd(&ctr[1], (unsigned long long)total);
                    abase = readlane64(abase, 0);
                }
                if (fresh) {
                    loff = abase + incl - wantb;
                    if (loff + wantb > lens_cap) {
                        meta[idx] = RowMeta{0, 0, 0, 0, 0, 0};   // no room: the finisher decodes the whole block
                    } else {
                        live = true;
                        need = true;
                    }
                }
            }
        }
        if (!__any(live)) {
            if (more) continue;
            break;
        }
        // ---- the general step
        // rotate requested bytes in (every lane past the first half of its ring)
        {
            // block b's 64 requested bytes are held by lanes 4 (b % 16) ..
            // + 3, 16 bytes each, in pf[b / 16]
            const uint64_t R = __ballot(live && pfv && ip >= wb + 64);
            if (R) {
#pragma unroll
                for (int c = 0; c < 4; ++c) {
                    const int bb = 16 * c + (int)(lane >> 2);
                    const int32_t wbb = __builtin_amdgcn_ds_bpermute(bb << 2, wb);
                    if ((R >> bb) & 1ull) {
                        lds_u8* Wb = (lds_u8*)(wins + bb * kPW);
                        const int32_t h = (wbb >> 6) & 1;
                        lds_st16(Wb + 64 * h + 16 * (int32_t)(lane & 3), pf[c]);
                    }
                }
                if ((R >> lane) & 1ull) {
                    wb += 64;
                    pfv = false;
                }
            }
        }
        // a lane stopped at its ring's end that the rotation could not serve
        // (nothing requested: the ring already ends at the input's end) takes
        // the general parse; every other stopped lane retries the fast loop
        if (live && stall && !need && ip + 16 > wb + kPW) need = true;
        stall = false;
        bool wl = false;   // a block start with a literal of >= 4 KiB: perhaps a whole-literal block
        if (live && need) {
            need = false;
            if (ip + 32 > wb + kPW) {   // no bytes ahead (block start, a long literal): load the ring now
                const int32_t nb = ip & ~63;
                u32x4 v0[4], v1[4];
                load64(s, nb, iend, v0);
                load64(s, nb + 64, iend, v1);
                ring_put(W, (nb >> 6) & 1, v0);
                ring_put(W, ((nb >> 6) + 1) & 1, v1);
                wb = nb;
                pfv = false;
            }
            // one sequence, general parse with the reference fast loop's tests
            // (lz4.c:2004-2086)
            bool good = true, slow = true;
            int32_t pe = 0;
            int64_t lit = 0, ml = 0;
            // straight-line from the 32 ring bytes at ip (the ring holds them:
            // loaded above if not): literal and match lengths with at most one
            // extension byte each, offset inside the 32 bytes -- the same
            // tests, in the same order, as the byte loop below, which takes
            // only what this cannot (a 255 extension byte, a literal of more
            // than 27 bytes)
            {
                // the token and the literal-length byte from the aligned dword
                // pair at ip, the offset and match-length byte from the pair at
                // ip + po (po <= 29: inside the 32 bytes the ring holds)
                const uint32_t x0 = __builtin_amdgcn_alignbyte(*(lds_vu32*)(size_t)(Wa | (((uint32_t)ip + 4u) & (kPW - 4))),
                                                               *(lds_vu32*)(size_t)(Wa | ((uint32_t)ip & (kPW - 4))), (uint32_t)ip);
                const uint32_t tok = x0 & 0xFFu;
                const int32_t l0 = (int32_t)(tok >> 4), mlc = (int32_t)(tok & 15u);
                int32_t q = 1, L = l0;
                bool g = true, sl = false;
                if (l0 == 15) {   // read_variable_length(&ip, iend - 15, 1), one byte of it
                    if (ip + 1 >= iend - 15) {
                        g = false;
                    } else {
                        const int32_t e = (int32_t)((x0 >> 8) & 0xFFu);
                        q = 2;
                        L += e;
                        if (ip + 2 > iend - 15) g = false;
                        else if (e == 255) sl = true;
                        if (g && !sl && (op + L > oend - 32 || ip + q + L > iend - 32)) g = false;   // :2016-2027
                    }
                } else if (ip + 1 > iend - 17) {   // :2034
                    g = false;
                }
                int32_t M = mlc, pq = 0;
                if (g && !sl) {
                    const int32_t po = q + L;   // the offset's byte in the 32
                    if (po + 3 > 32) {
                        sl = true;
                    } else {
                        const uint32_t ao = (uint32_t)(ip + po);
                        const uint32_t dw = __builtin_amdgcn_alignbyte(*(lds_vu32*)(size_t)(Wa | ((ao + 4u) & (kPW - 4))),
                                                                       *(lds_vu32*)(size_t)(Wa | (ao & (kPW - 4))), ao);
                        const int32_t off = (int32_t)(dw & 0xFFFFu);
                        pq = po + 2;
                        if (mlc == 15) {   // read_variable_length(&ip, iend - 4, 0), one byte of it
                            const int32_t e2 = (int32_t)((dw >> 16) & 0xFFu);
                            ++pq;
                            M += e2;
                            if (ip + pq > iend - 4) g = false;
                            else if (e2 == 255) sl = true;
                        }
                        M += 4;
                        if (g && !sl && (off == 0 || off > op + L || op + L + M >= oend - 64)) g = false;
                    }
                }
                slow = sl;
                if (!sl) {
                    good = g;
                    pe = ip + pq;
                    lit = L;
                    ml = M;
                }
            }
            if (slow) {   // (rare) byte by byte; bytes outside the ring come from HBM
#define PB(x) ((x) - wb < kPW ? (uint32_t)W[(x) & (kPW - 1)] : (uint32_t)s[(x)])
                good = true;
                const uint32_t tok = PB(ip);
                lit = tok >> 4;
                int32_t q = ip + 1;
                if (lit == 15) {   // read_variable_length(&ip, iend - 15, 1), lz4.c:1903-1928
                    if (q >= iend - 15) {
                        good = false;
                    } else {
                        uint32_t b;
                        int32_t run = 0;
                        do {
                            b = PB(q);
                            ++q;
                            lit += b;
                            if (q > iend - 15) good = false;
                            // a run past kPRunCap bytes (a literal of >= 4 KiB: an
                            // incompressible block's single literal is ~257) goes to
                            // the finisher: not read byte by byte here, mostly from HBM
                            if (++run >= kPRunCap && b == 255) {
                                good = false;
                                wl = k == 0;
                            }
                        } while (good && b == 255);
                        if (good && (op + lit > oend - 32 || q + lit > iend - 32)) good = false;   // :2016-2027
                    }
                } else if (q > iend - 17) {   // :2034
                    good = false;
                }
                if (good) {
                    const int32_t po = q + (int32_t)lit;
                    const uint32_t off = PB(po) | (PB(po + 1) << 8);
                    pe = po + 2;
                    ml = tok & 15;
                    if (ml == 15) {   // read_variable_length(&ip, iend - 4, 0)
                        uint32_t b;
                        int32_t run = 0;
                        do {
                            b = PB(pe);
                            ++pe;
                            ml += b;
                            if (pe > iend - 4) good = false;
                            if (++run >= kPRunCap && b == 255) good = false;   // (as above)
                        } while (good && b == 255);
                    }
                    ml += 4;
                    // offset 0 and offsets before the block start go to the exact
                    // path (lz4.c:2071, :2081); so do matches reaching oend - 64 (:2073, :2076)
                    if (good && (off == 0 || (int64_t)off > (int64_t)op + lit || (int64_t)op + lit + ml >= (int64_t)oend - 64))
                        good = false;
                }
#undef PB
            }
            if (good) {
                const int32_t adv = pe - ip;
                stg[k & (kPStage - 1)] = (uint8_t)(adv < 255 ? adv : 255);
                ip = pe;
                op += (int32_t)(lit + ml);
                ++k;
            } else {   // the first sequence that is not good: the finisher resumes here
                for (int32_t c = kf; c < k; c += 16) gbl_put(lens + loff + c, lds_ld16(stg + (c & (kPStage - 1))), k - c);
                meta[idx] = RowMeta{loff, k, ip - sh, op, 0, 0};
                live = false;
            }
        }
        // whole-literal blocks, checked and copied by the wave (whole_literal_block)
        for (uint64_t C = __ballot(wl); C != 0; C &= C - 1) {
            const int f = __builtin_ctzll(C);
            const int64_t fi = readlane64(idx, f);
            const int32_t fsh = __builtin_amdgcn_readlane(sh, f);
            const int64_t r = whole_literal_block(readlane_ptr(s, f) + fsh, __builtin_amdgcn_readlane(iend, f) - fsh,
                                                  __builtin_amdgcn_readlane(oend, f), dst + dst_off[fi], lane);
            if ((int)lane == f && r >= 0) meta[idx] = RowMeta{loff, 0, -1, (int32_t)r, 0, 0};
        }
        // flush full halves of the length ring
        if (live && k - kf >= kPStage / 2) {
            uint8_t* o = lens + loff + kf;
            st16(o, lds_ld16(stg + (kf & (kPStage - 1))));
            kf += kPStage / 2;
        }
        // request the next 64 bytes ahead
        {
            // four lanes per block, 16 contiguous bytes each: one 64-byte
            // request per block instead of four 16-byte ones
            const uint64_t Q = __ballot(live && !pfv && wb + kPW < iend);
            if (Q) {
                const uint64_t na = (uint64_t)(uintptr_t)(s + wb + kPW);
                const int32_t left = iend - (wb + kPW);
#pragma unroll
                for (int c = 0; c < 4; ++c) {
                    const int bb = 16 * c + (int)(lane >> 2);
                    const uint32_t lo = (uint32_t)__builtin_amdgcn_ds_bpermute(bb << 2, (int32_t)(uint32_t)na);
                    const uint32_t hi = (uint32_t)__builtin_amdgcn_ds_bpermute(bb << 2, (int32_t)(uint32_t)(na >> 32));
                    const int32_t lf = __builtin_amdgcn_ds_bpermute(bb << 2, left) - 16 * (int32_t)(lane & 3);
                    if ((Q >> bb) & 1ull) {
                        const uint8_t* q = readlane_safe_ptr(((uint64_t)hi << 32) | lo) + 16 * (lane & 3);
                        pf[c] = lf >= 16 ? ld16(q) : ld16_guarded(q, lf);
                    }
                }
                if ((Q >> lane) & 1ull) pfv = true;
            }
        }
        // ---- the common sequence, straight-line, until too few lanes can go on
        const int32_t thr = min(kPMinActive, (int)__popcll(__ballot(live)));
        const int32_t kfl = kf + kPStage - 1;   // the length ring is full at k == kfl
        // the sequence at (ip, op): the token byte, then the aligned dword
        // pair holding the offset and the match-length byte (each address
        // wrapped into the ring) -- two dependent LDS reads, no select tree
        auto peek = [&](int32_t& lit, int32_t& adv, int32_t& ml, int32_t& off, int32_t& oe) __attribute__((always_inline)) {
            const int32_t tok = (int32_t)*(lds_vu8*)(size_t)(Wa | ((uint32_t)ip & (kPW - 1)));
            lit = tok >> 4;
            const int32_t mlc = tok & 15;
            const int32_t ob = ip + 1 + lit;
            const uint32_t lo = *(lds_vu32*)(size_t)(Wa | ((uint32_t)ob & (kPW - 4)));
            const uint32_t hi = *(lds_vu32*)(size_t)(Wa | ((uint32_t)(ob + 4) & (kPW - 4)));
            const uint32_t dw = __builtin_amdgcn_alignbyte(hi, lo, (uint32_t)ob);
            const bool mlx = mlc == 15;
            off = (int32_t)(dw & 0xFFFFu);
            adv = 3 + lit + (int32_t)mlx;
            ml = mlc + 4 + (mlx ? (int32_t)((dw >> 16) & 0xFFu) : 0);   // 274: a 255 extension byte
            oe = op + lit + ml;
        };
        {
            // one condition per step for the lanes still going: the ring's
            // end and the block's end (ip <= iend - 20 covers both end tests
            // of the reference's fast loop for adv <= 16) as one bound
            const int32_t lim = min(wb + kPW - 16, iend - 20);
            const int32_t oendm = oend - 64;
            // kPSteps steps per count of the lanes still going; every lane runs
            // them all (predicated, no exec-mask branches), and a lane that
            // cannot take its sequence stops going
            bool go = live && !need && !stall;
            while (true) {
#pragma unroll
                for (int u = 0; u < kPSteps; ++u) {
                    int32_t lit, adv, ml, off, oe;
                    peek(lit, adv, ml, off, oe);
                    const bool take = go & (ip <= lim) & (k < kfl) & (lit <= 12) & (ml != 274) &
                                      ((uint32_t)(off - 1) < (uint32_t)(op + lit)) & (oe < oendm);
                    // slot k is free (one slot of the ring always is): written even
                    // when the sequence is not taken, then overwritten
                    *(lds_vu8*)(size_t)(Sa | ((uint32_t)k & (kPStage - 1))) = (uint8_t)adv;
                    ip += take ? adv : 0;
                    op = take ? oe : op;
                    k += (int32_t)take;
                    go = take;
                }
                if ((int)__popcll(__ballot(go)) < max(thr, 1)) break;
            }
            // a lane that stopped waits (`stall`) for the next general step to
            // rotate its ring or flush its lengths, or takes the general parse
            // (`need`) for a sequence the one-step test does not cover
            if (live && !need && !stall && !go) {
                int32_t lit, adv, ml, off, oe;
                peek(lit, adv, ml, off, oe);
                const bool fast = (lit <= 12) & (ml != 274) & (ip <= iend - 20) & (off != 0) & (off <= op + lit) &
                                  (oe < oendm);
                stall = true;
                need = (ip + 16 <= wb + kPW) & (k < kfl) & !fast;
            }
        }
    }
}

// ------------------------------------------------------- 2. row execution
// Per row: output [base, base + kRowsH) of the block in LDS (the history).
// Lane jj reads its sequence straight from HBM: 32 bytes at its start, which
// the row knows from the recorded lengths (row prefix sum).  The lengths and
// the 32 bytes of the NEXT round are requested while this round copies, so a
// round waits on at most one memory round trip (its far match sources).
// History per row (bytes).  Far sources (below the history) are HBM line
// fills, ~0.67 per sequence at 1 KiB (a 128-byte line for a 16-byte piece):
// aiming them all at one cached line took the launch 128.6 -> 112.1 ms
// (r06j, wrong output).  1280 B is the deepest history the LDS holds at 5
// waves per SIMD (30.8 KB per workgroup; 1392 B ran 4 workgroups per CU,
// 130.9 ms): 0.61 fills per sequence, 128.6-129.6 -> 127.0-127.3 ms (r06j/k).
constexpr int32_t kRowsH = 1280;
constexpr int32_t kRowsHS = kRowsH + 32;   // buffer stride (16-byte reads past the end stay inside)
constexpr int32_t kRowsRoom = 512;         // rebase when less room than this is left
constexpr int32_t kRowsKeep = kRowsH - kRowsRoom;   // history kept on a rebase
static_assert(kRowsKeep % 16 == 0 && kRowsKeep + kRowsRoom <= kRowsH && kRowsKeep + 16 <= 1024, "history split");

// Row-cooperative exact copies in HBM (16 lanes, lane j = jj).
__device__ __forceinline__ void row_copy_literal(uint8_t* d, const uint8_t* s, int32_t len, int32_t jj) {
    for (int32_t pos = 16 * jj; pos < len; pos += 256) {
        const u32x4 v = len - pos >= 16 ? ld16(s + pos) : ld16_guarded(s + pos, len - pos);
        gbl_put(d + pos, v, len - pos);
    }
}

__device__ __forceinline__ void row_copy_match(uint8_t* d, int32_t off, int32_t len, int32_t jj) {
    if (off >= 16) {
        // steps of w = the offset rounded down to 16 (no piece of a step reads
        // bytes the step writes), each step's pieces four loads per lane at a
        // time: a long far match (a zero run's, off ~ ml ~ 2 KB) is one or two
        // steps, not one fenced 256-byte step each (r06zc)
        const int32_t w = off & ~15;
        for (int32_t b = 0; b < len; b += w) {
            const int32_t e = min(b + w, len);
            for (int32_t p0 = b + 16 * jj; p0 < e; p0 += 1024) {
                u32x4 v[4];
#pragma unroll
                for (int u = 0; u < 4; ++u)
                    if (p0 + 256 * u < e) v[u] = ld16(d + p0 + 256 * u - off);
#pragma unroll
                for (int u = 0; u < 4; ++u)
                    if (p0 + 256 * u < e) gbl_put(d + p0 + 256 * u, v[u], len - (p0 + 256 * u));
            }
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
        }
        return;
    }
    const u32x4 pat = period_pattern(ld16(d - off), (uint32_t)off);
    const int32_t step = 16 - (16 % off);
    for (int32_t pos = step * jj; pos < len; pos += step * 16) gbl_put(d + pos, pat, len - pos);
}

// 32 bytes of block input at t (bytes at or past iend read as zero)
__device__ __forceinline__ void load32(const uint8_t* s, int32_t t, int32_t iend, bool valid, u32x4& a, u32x4& b) {
    a = u32x4{0, 0, 0, 0};
    b = a;
    if (!valid) return;
    a = t + 16 <= iend ? ld16(s + t) : ld16_guarded(s + t, iend - t);
    b = t + 32 <= iend ? ld16(s + t + 16) : ld16_guarded(s + t + 16, iend - t - 16);
}


#define LDS_PUT(p, v, k) lds_put_al((p), (v), (k), MT)

// Offsets inside a block's slots are never negative, so a 64-bit address is
// the base plus a zero-extended offset (no sign extension and no select of its
// high half per load; r06f: -0.6 % with the interleaved row sums below)
#define ROFF(x) ((uint32_t)(x))

// One round of a row, parsed: lane jj's sequence (literal at input position
// t, lit / off / ml), its output position o, the round's row totals and the
// far source requested from HBM; the literal's first 32 bytes go to XS.
// The literal's first 32 bytes go to the lane's LDS slot (two 16-byte
// aligned entries), not to registers: a parsed round waits there while the
// previous one executes, and the registers it frees hold the executor at 5
// waves per SIMD.
struct PSeq {
    int32_t t, lit, off, ml, o, dlt;  // t: the literal's input position
    int32_t opn, ipn;                 // uniform across the row
    uint32_t fl;                      // flags | (use << 8): the row takes its first `use` lanes
};
constexpr uint32_t kFlU = 1, kFlFar = 2, kFlLate = 4, kFlLitHbm = 8, kFlEsc = 16;

// The far source's first 32 bytes, requested when the round is parsed (two
// 16-byte pieces; the second only where a far match is longer than 16 bytes)
// and consumed by the round's passes.  Kept outside PSeq: after the passes
// the same registers take the next round's requests, with no copy between --
// a copy of a register with a load in flight waits for that load.
struct FarSrc {
    u32x4 g0, g1;
};

// Parse the row's round at (k0, ip, op): lane jj's length byte dlt, its
// start t and its 32 input bytes wa|wb (wb is clamped into the block, so
// bytes >= 16 are valid only if t + 32 <= iend).  bnext is the history base
// the round will run with; sources below it are requested now if they lie
// below F (flushed), else marked late (requested once flushed).
__device__ __forceinline__ void parse_round(PSeq& P, int32_t jj, int32_t r, int32_t k0, int32_t nseq, int32_t ip,
                                            int32_t op, int32_t bnext, int32_t F, const uint8_t* s, const uint8_t* d,
                                            int32_t iend, int32_t dlt, int32_t t, u32x4 wa, u32x4 wb, lds_u32x4* XS,
                                            FarSrc& FS, int32_t& incsum) {
    const bool act = k0 + jj < nseq;
    const bool esc = dlt == 255;   // length >= 255: the parse left it to be re-parsed
    const bool wbok = t + 32 <= iend;
    const uint32_t tok = wa.x & 0xFFu;
    const int32_t lit0 = (int32_t)(tok >> 4);
    const bool litx = lit0 == 15;
    const int32_t lit = lit0 + (litx ? (int32_t)byte_of(wa, 1) : 0);   // one extra byte unless escaped
    const int32_t lp = litx ? 2 : 1;
    const int32_t po = lp + lit;
    const int32_t mlc = (int32_t)(tok & 15u);
    // offset and first match-length byte: from wa for lit <= 12, else from wa|wb
    // the dword pair at pq selected by a tree on its three index bits (14
    // selects) for every lane, instead of a 16-byte and a 32-byte select chain
    // both computed and selected between
    const uint32_t pq = (uint32_t)(po < 28 ? po : 28);
    const uint32_t dwo = dword32_tree(wa, wb, pq);
    // (po > 29: past the 32 bytes, `slow` re-reads the offset: any shift in
    // 0..31 will do -- 8 * (po - pq) would reach 32 and be undefined)
    const uint32_t bsh = po > 28 ? 8u : 0u;
    int32_t off = (int32_t)((dwo >> bsh) & 0xFFFFu);
    const int32_t e0 = (int32_t)((dwo >> (bsh + 16)) & 0xFFu);
    int32_t ml = mlc + (mlc == 15 ? e0 : 0);
    const bool slow = (po + 3 > 32) | ((mlc == 15) & (e0 == 255)) | ((po + 3 > 16) & !wbok);
    if (slow && act && !esc) {   // a long match length, or the offset past the bytes at hand: from HBM
        const uint8_t* q = s + t;
        off = (int32_t)q[po] | ((int32_t)q[po + 1] << 8);
        ml = mlc;
        if (ml == 15) {
            int32_t pe = po + 2;
            uint32_t b;
            do {
                b = q[pe];
                ++pe;
                ml += (int32_t)b;
            } while (b == 255 && pe < iend - t);
        }
    }
    ml += 4;
    const int32_t len = act && !esc ? lit + ml : 0;
    // (with the next round's length-byte prefix sum, incsum: two chains)
    int32_t lsum = len;
    row_incl_sum2(lsum, incsum);
    const int32_t o = op + lsum - len;
    const int32_t mend = o + lit + ml;
    const bool ok = act & !esc & (mend <= bnext + kRowsH);
    const uint64_t nok = __ballot(!ok);
    int32_t use;
    bool u;
    if (nok == 0) {   // every row takes its 16 sequences: the ends of lane 15's
        use = 16;
        u = true;
        P.opn = row_last(o + len);
        P.ipn = row_last(t + dlt);
    } else {
        const uint32_t rb = (uint32_t)(nok >> (16 * r)) & 0xFFFFu;
        use = rb ? __builtin_ctz(rb) : 16;
        u = jj < use;
        P.opn = op + row_last(row_incl_sum(u ? len : 0));
        P.ipn = ip + row_last(row_incl_sum(u ? dlt : 0));
    }
    const int32_t s0 = o + lit - off;
    const bool far = u & (s0 < bnext);
    const bool late = far & (s0 + 32 > F);
    const bool pf = far & !late;
    // unconditional requests (lanes without a far source read the block start)
    FS.g0 = ld16(d + ROFF(pf ? s0 : 0));
    // the second piece [s0 + 16, s0 + 32) is flushed too (not late: s0 + 32 <= F)
    FS.g1 = ld16(d + ROFF((pf & (ml > 16)) ? s0 + 16 : 0));
    const uint32_t sh = (uint32_t)lp;
    XS[0] = u32x4{__builtin_amdgcn_alignbyte(wa.y, wa.x, sh), __builtin_amdgcn_alignbyte(wa.z, wa.y, sh),
                 __builtin_amdgcn_alignbyte(wa.w, wa.z, sh), __builtin_amdgcn_alignbyte(wb.x, wa.w, sh)};
    XS[1] = u32x4{__builtin_amdgcn_alignbyte(wb.y, wb.x, sh), __builtin_amdgcn_alignbyte(wb.z, wb.y, sh),
                 __builtin_amdgcn_alignbyte(wb.w, wb.z, sh), __builtin_amdgcn_alignbyte(0u, wb.w, sh)};
    P.t = t + lp;
    P.lit = lit;
    P.off = off;
    P.ml = ml;
    P.o = o;
    P.dlt = dlt;
    P.fl = ((uint32_t)use << 8) | (u ? kFlU : 0u) | (far ? kFlFar : 0u) | (late ? kFlLate : 0u) | (esc ? kFlEsc : 0u) |
           ((u & (lp + lit > 16) & ((lp + lit > 32) | !wbok)) ? kFlLitHbm : 0u);
}

// 16 * jj recomputed where it is used on the rare paths (block end, a
// sequence that does not fit): kept live across the loop it was spilled
__device__ __forceinline__ int32_t cold_j16(int32_t jj) {
    int32_t v = 16 * jj;
    asm volatile("" : "+v"(v));
    return v;
}

// history base a row runs its next round with, given the output position op
__device__ __forceinline__ int32_t next_base(int32_t op, int32_t base) {
    return op - base > kRowsH - kRowsRoom ? ((op - kRowsKeep) & ~15) : base;
}

// the round's inputs: 32 bytes at t (clamped into the block) and a length byte
__device__ __forceinline__ void load_in(const uint8_t* s, int32_t t, int32_t iend, u32x4& a, u32x4& b) {
    const int32_t ta = t + 16 <= iend ? t : 0;   // good sequences: t + 16 < iend
    const int32_t tb = t + 32 <= iend ? t + 16 : iend - 16;
    a = ld16(s + ROFF(ta));
    b = ld16(s + ROFF(tb));
}
// (no select on the loaded value: a lane past the block's good sequences
// reads the last length, and parse_round masks it by `act`; a select here
// waited for the load at once)
__device__ __forceinline__ int32_t load_len(const uint8_t* dl, int32_t k, int32_t nseq) {
    return (int32_t)dl[ROFF(k < nseq ? k : nseq - 1)];
}


// Rows in flight: round R executes while round R + 1 is already parsed
// (its far sources in flight) and round R + 2's inputs are requested, so a
// round waits on no memory latency of its own.  The registers are held to 5
// waves per SIMD (the LDS allows 5; 6 spilled, r05bg).
// kEWG: threads per workgroup.  The waves of a workgroup are independent (no
// barrier after the prologue); 256 shares the put-mask and period tables
// (1.6 KB of LDS) between four waves.
constexpr int kEWG = 256;
__global__ __launch_bounds__(kEWG) __attribute__((amdgpu_waves_per_eu(5, 8))) void rows_exec_kernel(const uint8_t* __restrict__ src,
                                                       const int64_t* __restrict__ src_off,
                                                       const int32_t* __restrict__ src_len, uint8_t* dst,
                                                       const int64_t* __restrict__ dst_off,
                                                       const RowMeta* __restrict__ meta,
                                                       const uint8_t* __restrict__ lens, int64_t n,
                                                       unsigned long long* __restrict__ ctr) {
    __shared__ __attribute__((aligned(16))) uint8_t hists[kEWG / 16 * kRowsHS];
    __shared__ __attribute__((aligned(16))) uint32_t mtab[kPutTab];
    __shared__ __attribute__((aligned(16))) uint32_t psel[16 * 8];
    __shared__ __attribute__((aligned(16))) u32x4 xsl[kEWG * 2];
    const uint32_t lane = threadIdx.x & 63u;   // lane of the wave
    const int32_t jj = (int32_t)(lane & 15), r = (int32_t)(lane >> 4);
    lds_u8* HB = (lds_u8*)(hists + (threadIdx.x >> 4) * kRowsHS);   // the row's history
    lds_put_table_init(mtab, threadIdx.x, kEWG);
    lds_cu32* MT = (lds_cu32*)mtab;
    period_sel_init(psel, threadIdx.x, kEWG);
    __syncthreads();   // tables written by other waves
    lds_cu32* PS = (lds_cu32*)psel;
    lds_u32x4* XSL = (lds_u32x4*)(xsl + 2 * threadIdx.x);
    // row state (uniform across the row's 16 lanes)
    const uint8_t* s = nullptr;
    uint8_t* d = nullptr;
    const uint8_t* dl = nullptr;
    int32_t iend = 0, nseq = 0, k0 = 0, ip = 0, op = 0, base = 0, F = 0;
    bool have = false, sync = true;
    PSeq P, Q;   // P: the round to execute; Q: the next one, parsed ahead
    FarSrc FS;   // P's far-source pieces (after P's passes: Q's)
    // the round after P (parsed next): its length bytes as their inclusive row
    // prefix sum incq (a computed value) and its 32 input bytes na|nb; lraw =
    // the raw length bytes of the round after that.  Every loaded value is
    // consumed before the same variable is loaded again, so none is copied
    // across the loop edge (a copy of a register with a load in flight waits
    // for it -- in order, for every younger request too: r05)
    int32_t incq = 0, lraw = 0;
    u32x4 na = u32x4{0, 0, 0, 0}, nb = na;
    while (true) {
        if (!have) {
            unsigned long long b = 0;
            if (jj == 0) b = atomicAdd(&ctr[2], 1ull);
            const uint32_t blo = (uint32_t)row_first((int32_t)(uint32_t)b);
            const uint32_t bhi = (uint32_t)row_first((int32_t)(uint32_t)(b >> 32));
            b = ((unsigned long long)bhi << 32) | blo;
            if (b >= (unsigned long long)n) break;
            const RowMeta mt = meta[b];
            if (mt.nseq == 0) continue;   // the finisher decodes the whole block
            s = src + src_off[b];
            d = dst + dst_off[b];
            iend = src_len[b];
            dl = lens + mt.loff;
            nseq = mt.nseq;
            k0 = ip = op = base = F = 0;
            have = true;
            sync = true;
        }
        if (sync && k0 >= nseq) {   // the block's good prefix is done: flush the rest exactly
            for (int32_t c = F + cold_j16(jj); c < op; c += 256) gbl_put(d + c, lds_ld16(HB + (c - base)), op - c);
            have = false;
            continue;
        }
        if (sync) {   // block start, or the last round stopped early: parse this round now
            // the length bytes of this round, the next and the one after at
            // once, then this round's inputs and -- as if it takes all 16 --
            // the next round's: two round trips before the parse (four were
            // dependent before, r06ze)
            const int32_t dc = load_len(dl, k0 + jj, nseq);
            const int32_t dq = load_len(dl, k0 + 16 + jj, nseq);
            lraw = load_len(dl, k0 + 32 + jj, nseq);
            int32_t incc = dc;
            incq = dq;
            row_incl_sum2(incc, incq);
            const int32_t tc = ip + incc - dc;
            u32x4 wa, wb;
            load_in(s, tc, iend, wa, wb);
            load_in(s, ip + row_last(incc) + incq - dq, iend, na, nb);   // = P.ipn + incq - dq when P takes 16
            int32_t dummy = 0;
            parse_round(P, jj, r, k0, nseq, ip, op, base, F, s, d, iend, dc, tc, wa, wb, XSL, FS, dummy);
            sync = false;
            // the loads just issued (this round's far sources among them) are
            // waited for here, once: left pending, the merge of this rare path
            // with the common one made every round wait for its newest
            // far-source request (r05a: -1.7 %).  A round that takes no
            // sequence goes to the one-sequence path, whose first fence waits.
            if ((P.fl >> 8) != 0) wait_vm0();
        }
        if ((P.fl >> 8) == 0) {
            sync = true;
            // one sequence that does not fit the buffers: flush, copy it in
            // HBM on the row, reload the history
            // (the parse verified it: every read below stays inside the block)
            int32_t L, q, ofs, qe, M;
            if (!(row_first((int32_t)P.fl) & kFlEsc)) {   // lane 0's sequence as parse_round read it: exact when not escaped
                L = row_first(P.lit);
                q = row_first(P.t);
                ofs = row_first(P.off);
                M = row_first(P.ml);
                // its end: length bytes are runs of 255 and one byte below 255
                qe = q + L + 2 + (M >= 19 ? (M - 19) / 255 + 1 : 0);
            } else {   // (rare) a sequence of >= 255 input bytes: byte by byte
                const uint32_t tk = s[ip];
                L = (int32_t)(tk >> 4);
                q = ip + 1;
                if (L == 15) {
                    uint32_t b;
                    do {
                        b = s[q];
                        ++q;
                        L += (int32_t)b;
                    } while (b == 255 && q < iend);
                }
                ofs = (int32_t)s[q + L] | ((int32_t)s[q + L + 1] << 8);
                qe = q + L + 2;
                M = (int32_t)(tk & 15u);
                if (M == 15) {
                    uint32_t b;
                    do {
                        b = s[qe];
                        ++qe;
                        M += (int32_t)b;
                    } while (b == 255 && qe < iend);
                }
                M += 4;
            }
            // the flush and the literal touch different bytes: one fence for both
            for (int32_t c = F + cold_j16(jj); c < op; c += 256) gbl_put(d + c, lds_ld16(HB + (c - base)), op - c);
            row_copy_literal(d + op, s + q, L, jj);
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
            row_copy_match(d + op + L, ofs, M, jj);
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
            op += L + M;
            ip = qe;
            k0 += 1;
            base = (op > kRowsKeep ? op - kRowsKeep : 0) & ~15;
            // op < oend - 64: the 16-byte reads stay inside the block's slot
            for (int32_t c = base + cold_j16(jj); c < op; c += 256) lds_st16(HB + (c - base), ld16(d + c));
            F = op;
            continue;
        }
        // ---- literals: bytes lp.. of the input (exact); longer ones rare
        {
            const bool u = (P.fl & kFlU) != 0;
            const int32_t lit = P.lit, o = P.o;
            if (u && lit > 0) LDS_PUT(HB + (o - base), XSL[0], lit);
            if (u && lit > 16) {
                if (!(P.fl & kFlLitHbm)) {
                    LDS_PUT(HB + (o - base + 16), XSL[1], lit - 16);
                } else {   // a literal beyond the bytes at hand: from HBM (inside the block: good)
                    for (int32_t i = 16; i < lit; i += 16) LDS_PUT(HB + (o - base + i), ld16(s + P.t + i), lit - i);
                }
            }
        }
        // ---- the next round, parsed ahead (its far sources are requested
        // then), and the inputs of the round after it are requested: after
        // this round's passes (below), so that no load the passes wait on (a
        // long far match's later pieces, a late source) is younger than these
        // requests -- gfx9 counts loads in order, and waiting for one load
        // waits for every older one (r05)
        const bool ahead = (P.fl >> 8) == 16 && k0 + 16 < nseq;
        auto parse_ahead = [&]() __attribute__((always_inline)) {
            if (ahead) {
                const int32_t bq = next_base(P.opn, base);
                // Q's length bytes from their prefix sum: lane j's minus lane j-1's
                const int32_t dq = incq - __builtin_amdgcn_update_dpp(0, incq, 0x111, 0xF, 0xF, true);
                int32_t inc2 = lraw;
                parse_round(Q, jj, r, k0 + 16, nseq, P.ipn, P.opn, bq, F, s, d, iend, dq, P.ipn + incq - dq, na, nb, XSL, FS, inc2);
                incq = inc2;
                load_in(s, Q.ipn + incq - lraw, iend, na, nb);
                lraw = load_len(dl, k0 + 48 + jj, nseq);
            }
        };
        // ---- execute round P
        const bool u = (P.fl & kFlU) != 0;
        const int32_t lit = P.lit, off = P.off, ml = P.ml, o = P.o;
        const int32_t m = o + lit, mend = m + ml, s0 = m - off;
        // readiness passes: a match is copied once no earlier pending match of
        // the round writes into its source [s0, se)
        const bool far = (P.fl & kFlFar) != 0, late = (P.fl & kFlLate) != 0;
        u32x4 g0 = FS.g0;
        const u32x4 g1 = FS.g1;
        if (__any(late)) {   // a source flushed only by the previous round (rare): load it now
            const u32x4 lv = ld16(d + ROFF(late ? s0 : 0));
            g0 = late ? lv : g0;
        }
        const int32_t se = s0 + (off < ml ? off : ml);
        const bool per = off < 16;   // period pattern (s0 >= base here: m - base >= off)
        // 16 - 16 % off for off 1..15 from a table (3 bits per offset; the
        // integer division was ~20 VALU per round)
        constexpr uint64_t kRem16 = (0ull << 3) | (0ull << 6) | (1ull << 9) | (0ull << 12) | (1ull << 15) |
                                    (4ull << 18) | (2ull << 21) | (0ull << 24) | (7ull << 27) | (6ull << 30) |
                                    (5ull << 33) | (4ull << 36) | (3ull << 39) | (2ull << 42) | (1ull << 45);
        const int32_t stp = per ? 16 - (int32_t)((kRem16 >> (3u * ((uint32_t)off & 15u))) & 7u) : 16;
        bool pend = u;
        // one match copy (exec-masked to the ready lanes: an LDS access costs per active lane)
        auto copy_match = [&]() __attribute__((always_inline)) {
            const u32x4 l0 = lds_ld16a(HB + (s0 >= base ? s0 - base : 0));
            u32x4 v0 = far ? g0 : l0;
            if (per) v0 = period_perm(l0, PS + 8 * off);
            LDS_PUT(HB + (m - base), v0, ml);
            if (ml > stp) {   // the rest (matches longer than one step)
                for (int32_t i = stp; i < ml; i += stp) {
                    u32x4 v = v0;
                    if (!per) {
                        const int32_t sp = s0 + i;
                        // sp < base: flushed (F >= base + kRowsKeep - 143); the
                        // second piece of a (not late) far source was requested
                        // with the first; later pieces are loaded now, only where
                        // some lane needs one (this wait then covers only loads
                        // older than the round's own requests)
                        v = lds_ld16a(HB + (sp >= base ? sp - base : 0));
                        const bool pc1 = (i == 16) & far & !late;
                        if (sp < base && pc1) v = g1;
                        const bool hb = (sp < base) & !pc1;
                        if (__any(hb)) {
                            const u32x4 x = ld16(d + ROFF(hb ? sp : 0));
                            v = hb ? x : v;
                        }
                    }
                    LDS_PUT(HB + (m - base + i), v, ml - i);
                }
            }
        };
        while (__any(pend)) {
            // x1 = 1 + the end of the nearest pending match below, y1 = BIG -
            // the start of the first pending match below (0: none)
            int32_t x1, y1;
            row_excl_max2(pend ? mend + 1 : 0, pend ? 0x3FFFFFFF - m : 0, x1, y1);
            const bool ready = pend & ((x1 <= s0 + 1) | (y1 <= 0x3FFFFFFF - se));
            if (ready) copy_match();
            pend = pend && !ready;
        }
        parse_ahead();
        // ---- flush, advance, rebase for the next round
        const int32_t opn = P.opn;
        {
            // whole 128-byte lines only, each written once (a line split over two
            // rounds' flushes was written twice: WRITE_SIZE -20 %, the
            // executor 94.4 -> 90.8 ms, r06x); F lags op by < 144 bytes, all
            // of them still in the history
            const int32_t fe = opn & ~127;
            for (int32_t c = F + 16 * jj; c + 16 <= fe; c += 256) st16(d + ROFF(c), lds_ld16(HB + (c - base)));
            if (fe > F) F += (fe - F) & ~15;
        }
        op = opn;
        ip = P.ipn;
        k0 += (int32_t)(P.fl >> 8);
        const int32_t nbse = next_base(op, base);
        if (nbse != base) {
            // one group (op - nbse < kRowsKeep + 16 <= 1024): every read of
            // the row's 16 lanes is issued before any write
            for (int32_t c0 = 0; c0 < op - nbse; c0 += 1024) {
                u32x4 v[4];
#pragma unroll
                for (int g = 0; g < 4; ++g) v[g] = lds_ld16(HB + (nbse - base) + c0 + 256 * g + 16 * jj);
#pragma unroll
                for (int g = 0; g < 4; ++g) lds_st16(HB + c0 + 256 * g + 16 * jj, v[g]);
            }
            // (the copy moved 1 KiB: bytes past op - nbse came from past the
            // old output, zero, or from past the row's buffer)
            base = nbse;
        }
        if (ahead) {
            P = Q;
        } else {
            sync = true;
        }
    }
}

}  // namespace lz4m

using namespace lz4m;


extern "C" size_t lz4m_rows_fixed_bytes(int64_t n) { return kRowsMeta + (size_t)n * sizeof(RowMeta); }

extern "C" int lz4m_rows_launch(const uint8_t* d_src, const int64_t* d_src_off, const int32_t* d_src_len,
                                uint8_t* d_dst, const int64_t* d_dst_off, const int32_t* d_dst_cap, int64_t n,
                                void* d_work, size_t work_bytes, int parse_grid, int exec_grid, hipStream_t stream) {
    const size_t fixed = lz4m_rows_fixed_bytes(n);
    if (work_bytes < fixed) return LZ4M_ROWS_ENOSPACE;
    unsigned long long* ctr = static_cast<unsigned long long*>(d_work);
    RowMeta* meta = reinterpret_cast<RowMeta*>(static_cast<uint8_t*>(d_work) + kRowsMeta);
    uint8_t* lens = static_cast<uint8_t*>(d_work) + fixed;
    const int64_t lens_cap = (int64_t)(work_bytes - fixed);
    hipError_t e = hipMemsetAsync(ctr, 0, 64, stream);
    if (e != hipSuccess) return (int)e;
    hipLaunchKernelGGL(rows_parse_kernel, dim3((uint32_t)parse_grid), dim3(kPWG), 0, stream, d_src, d_src_off,
                       d_src_len, d_dst, d_dst_off, d_dst_cap, n, meta, lens, lens_cap, ctr);
    hipLaunchKernelGGL(rows_exec_kernel, dim3((uint32_t)exec_grid), dim3(kEWG), 0, stream, d_src, d_src_off, d_src_len,
                       d_dst, d_dst_off, meta, lens, n, ctr);
    return (int)hipGetLastError();
}

extern "C" int lz4m_rows_grids(int64_t n, int* parse_grid, int* exec_grid) {
    int dev = 0, cus = 0, pk = 0, ek = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&pk, reinterpret_cast<const void*>(rows_parse_kernel), kPWG, 0);
    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&ek, reinterpret_cast<const void*>(rows_exec_kernel), kEWG, 0);
    if (cus <= 0) cus = 256;
    const int64_t ps = (int64_t)cus * (pk > 0 ? pk : 1), es = (int64_t)cus * (ek > 0 ? ek : 1);
    const int64_t pneed = (n + kPWG - 1) / kPWG, eneed = (n + kEWG / 16 - 1) / (kEWG / 16);
    *parse_grid = (int)(pneed < ps ? pneed : ps);
    *exec_grid = (int)(eneed < es ? eneed : es);
    return 0;
}
