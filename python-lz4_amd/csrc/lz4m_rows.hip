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

// Exactly k bytes (k >= 16: 16; k <= 0: none) of v at LDS address p.
__device__ __forceinline__ void lds_put(lds_u8* p, u32x4 v, int32_t k) {
    if (k >= 16) {
        lds_st16(p, v);
        return;
    }
    if (k <= 0) return;
    uint32_t o = 0;
    if (k & 8) {
        const uint64_t x = ((uint64_t)v.y << 32) | v.x;
        __builtin_memcpy((uint8_t*)p, &x, 8);
        o = 8;
    }
    if (k & 4) {
        const uint32_t x = window_dword(v, o);
        __builtin_memcpy((uint8_t*)(p + o), &x, 4);
        o += 4;
    }
    if (k & 2) {
        const uint16_t x = (uint16_t)window_dword(v, o);
        __builtin_memcpy((uint8_t*)(p + o), &x, 2);
        o += 2;
    }
    if (k & 1) p[o] = (uint8_t)window_dword(v, o);
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

// ------------------------------------------------------------ 1. the parse
// One lane per block.  The compressed block is read through a 128-byte LDS
// window per lane.  A lane parses sequences out of its window until it needs
// bytes beyond it; the wave then refills the windows of all lanes waiting,
// with all their loads in flight at once (one memory round trip per ~20
// sequences per lane instead of one per refill), and parsing resumes.  A
// sequence whose literal skips past the window is split: the token and
// literal length are parsed first, the offset and match length after the
// window moves to them.  Recorded lengths are staged 32 at a time in LDS and
// leave for HBM as whole 32-byte chunks.
constexpr int kPW = 128;                // window bytes
constexpr int kPWS = kPW + 16;          // window stride
constexpr int kPStage = 32;
#ifndef LZ4M_PARSE_MIN_ACTIVE
#define LZ4M_PARSE_MIN_ACTIVE 16        // refill once fewer lanes than this can still parse
#endif

__global__ __launch_bounds__(256) void rows_parse_kernel(const uint8_t* __restrict__ src,
                                                         const int64_t* __restrict__ src_off,
                                                         const int32_t* __restrict__ src_len,
                                                         const int32_t* __restrict__ dst_cap, int64_t n,
                                                         RowMeta* __restrict__ meta, uint8_t* __restrict__ lens,
                                                         int64_t lens_cap, unsigned long long* __restrict__ ctr) {
    __shared__ __attribute__((aligned(16))) uint8_t wins[256 * kPWS];
    __shared__ __attribute__((aligned(16))) uint8_t stgs[256 * kPStage];
    const uint32_t lane = lane_id();
    lds_u8* W = (lds_u8*)(wins + threadIdx.x * kPWS);
    lds_u8* stg = (lds_u8*)(stgs + threadIdx.x * kPStage);
    const uint8_t* s = nullptr;
    int64_t idx = -1, loff = 0;
    int32_t iend = 0, oend = 0, ip = 0, op = 0, k = 0, ib = 0;
    // a sequence split at its offset: po >= 0 is the offset position, ptok /
    // plit the token and literal length already parsed
    int32_t po = -1, plit = 0;
    uint32_t ptok = 0;
    int32_t want = 0;   // window wanted at this position (need)
    bool live = false, need = false, more = true;
    while (true) {
        if (more) {
            // idle lanes take the next blocks: one queue atomic and one
            // length-space atomic per wave refill
            const uint64_t idle = __ballot(!live);
            if (idle != 0 && (uint32_t)__popcll(idle) >= LZ4M_PARSE_MIN_ACTIVE / 2) {
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
                        s = src + src_off[idx];
                        iend = src_len[idx];
                        oend = dst_cap[idx];
                        ip = op = k = 0;
                        po = -1;
                        if (oend >= 64 && iend > 0) {   // else: no fast loop (lz4.c:1990-1993) or a special case
                            // a good sequence takes >= 3 input and >= 4 output bytes
                            const int32_t a = iend / 3, b = oend / 4;
                            wantb = (int64_t)(a < b ? a : b) + 1;
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
                        want = 0;
                    }
                }
            }
        }
        if (!__any(live)) {
            if (more) continue;
            break;
        }
        // refill every waiting window at once
        if (live && need) {
            const int32_t nb = want & ~15;
            u32x4 v[kPW / 16];
#pragma unroll
            for (int c = 0; c < kPW / 16; ++c) {
                const int32_t x = nb + 16 * c;
                v[c] = x + 16 <= iend ? ld16(s + x) : ld16_guarded(s + x, iend - x);
            }
#pragma unroll
            for (int c = 0; c < kPW / 16; ++c) lds_st16(W + 16 * c, v[c]);
            ib = nb;
            need = false;
        }
        // parse until too few lanes can go on
        while (true) {
            const bool go = live && !need;
            const uint64_t gm = __ballot(go);
            if (gm == 0 || (uint32_t)__popcll(gm) < (uint32_t)min(LZ4M_PARSE_MIN_ACTIVE, __popcll(__ballot(live))))
                break;
            if (!go) continue;
            // one sequence, with the reference fast loop's tests (lz4.c:2004-2086)
            bool good = true;
            if (po < 0) {
                if (ip + 16 > ib + kPW) {   // token + 15 bytes must be in the window
                    need = true;
                    want = ip;
                    continue;
                }
                const uint32_t tok = W[ip - ib];
                int64_t lit = tok >> 4;
                int32_t q = ip + 1;
                if (lit == 15) {   // read_variable_length(&ip, iend - 15, 1), lz4.c:1903-1928
                    if (q >= iend - 15) {
                        good = false;
                    } else {
                        uint32_t b;
                        do {
                            b = q - ib < kPW ? (uint32_t)W[q - ib] : (uint32_t)s[q];
                            ++q;
                            lit += b;
                            if (q > iend - 15) good = false;
                        } while (good && b == 255);
                        if (good && (op + lit > oend - 32 || q + lit > iend - 32)) good = false;   // :2016-2027
                    }
                } else if (q > iend - 17) {   // :2034
                    good = false;
                }
                if (good) {
                    po = q + (int32_t)lit;
                    plit = (int32_t)lit;
                    ptok = tok;
                }
            }
            if (good) {
                if (po + 3 > ib + kPW) {   // the offset and first length byte must be in the window
                    need = true;
                    want = po;
                    continue;
                }
                const uint32_t off = (uint32_t)W[po - ib] | ((uint32_t)W[po + 1 - ib] << 8);
                int32_t pe = po + 2;
                int64_t ml = ptok & 15;
                if (ml == 15) {   // read_variable_length(&ip, iend - 4, 0)
                    uint32_t b;
                    do {
                        b = pe - ib < kPW ? (uint32_t)W[pe - ib] : (uint32_t)s[pe];
                        ++pe;
                        ml += b;
                        if (pe > iend - 4) good = false;
                    } while (good && b == 255);
                }
                ml += 4;
                // offset 0 and offsets before the block start go to the exact
                // path (lz4.c:2071, :2081); so do matches reaching oend - 64 (:2073, :2076)
                if (good && (off == 0 || (int64_t)off > (int64_t)op + plit ||
                             (int64_t)op + plit + ml >= (int64_t)oend - 64))
                    good = false;
                if (good) {
                    const int32_t adv = pe - ip;
                    stg[k & (kPStage - 1)] = (uint8_t)(adv < 255 ? adv : 255);
                    if ((k & (kPStage - 1)) == kPStage - 1) {
                        uint8_t* o = lens + loff + (k & ~(kPStage - 1));
#pragma unroll
                        for (int c = 0; c < kPStage / 16; ++c) st16(o + 16 * c, lds_ld16(stg + 16 * c));
                    }
                    ip = pe;
                    op += plit + (int32_t)ml;
                    ++k;
                    po = -1;
                    continue;
                }
            }
            // the first sequence that is not good: the finisher resumes here
            const int32_t rest = k & (kPStage - 1);
            uint8_t* o = lens + loff + (k & ~(kPStage - 1));
            for (int c = 0; c < rest; c += 16) gbl_put(o + c, lds_ld16(stg + c), rest - c);
            meta[idx] = RowMeta{loff, k, ip, op, 0, 0};
            live = false;
        }
    }
}

// ------------------------------------------------------- 2. row execution
// Per row: output [base, base + kRowsH) of the block in LDS (the history).
// Lane jj reads its sequence straight from HBM: 32 bytes at its start, which
// the row knows from the recorded lengths (row prefix sum).  The lengths and
// the 32 bytes of the NEXT round are requested while this round copies, so a
// round waits on at most one memory round trip (its far match sources).
#ifndef LZ4M_ROWS_H
#define LZ4M_ROWS_H 2048
#endif
constexpr int32_t kRowsH = LZ4M_ROWS_H;
constexpr int32_t kRowsHS = kRowsH + 32;   // buffer stride (16-byte reads past the end stay inside)
constexpr int32_t kRowsKeep = kRowsH / 2;   // history kept on a rebase
constexpr int32_t kRowsRoom = 512;          // rebase when less room than this is left

// Row-cooperative exact copies in HBM (16 lanes, lane j = jj).
__device__ __forceinline__ void row_copy_literal(uint8_t* d, const uint8_t* s, int32_t len, int32_t jj) {
    for (int32_t pos = 16 * jj; pos < len; pos += 256) {
        const u32x4 v = len - pos >= 16 ? ld16(s + pos) : ld16_guarded(s + pos, len - pos);
        gbl_put(d + pos, v, len - pos);
    }
}

__device__ __forceinline__ void row_copy_match(uint8_t* d, int32_t off, int32_t len, int32_t jj) {
    if (off >= 16) {
        const int32_t w = (off < 256 ? off : 256) & ~15;   // rows whose sources all precede them
        for (int32_t b = 0; b < len; b += w) {
            const int32_t pos = b + 16 * jj;
            if (16 * jj < w && pos < len) gbl_put(d + pos, ld16(d + pos - off), len - pos);
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

// the 4 bytes at k (0..28) of the 32-byte window a|b
__device__ __forceinline__ uint32_t dword32(u32x4 a, u32x4 b, uint32_t k) {
    const uint32_t q = k >> 2;
    const uint32_t lo = q == 0 ? a.x : q == 1 ? a.y : q == 2 ? a.z : q == 3 ? a.w : q == 4 ? b.x : q == 5 ? b.y : q == 6 ? b.z : b.w;
    const uint32_t hi = q == 0 ? a.y : q == 1 ? a.z : q == 2 ? a.w : q == 3 ? b.x : q == 4 ? b.y : q == 5 ? b.z : q == 6 ? b.w : 0u;
    return __builtin_amdgcn_alignbyte(hi, lo, k & 3);
}

__global__ __launch_bounds__(64) void rows_exec_kernel(const uint8_t* __restrict__ src,
                                                       const int64_t* __restrict__ src_off,
                                                       const int32_t* __restrict__ src_len, uint8_t* dst,
                                                       const int64_t* __restrict__ dst_off,
                                                       const RowMeta* __restrict__ meta,
                                                       const uint8_t* __restrict__ lens, int64_t n,
                                                       unsigned long long* __restrict__ ctr) {
    __shared__ __attribute__((aligned(16))) uint8_t hists[4 * kRowsHS];
    const uint32_t lane = threadIdx.x;
    const int32_t jj = (int32_t)(lane & 15), r = (int32_t)(lane >> 4);
    lds_u8* HB = (lds_u8*)(hists + r * kRowsHS);
    // row state (uniform across the row's 16 lanes)
    const uint8_t* s = nullptr;
    uint8_t* d = nullptr;
    const uint8_t* dl = nullptr;
    int32_t iend = 0, nseq = 0, k0 = 0, ip = 0, op = 0, base = 0, F = 0;
    bool have = false, pf = false;
    // this round's inputs (valid when pf): length dc, start tc, bytes wa|wb;
    // dn = the next round's length
    int32_t dc = 0, tc = 0, dn = 0;
    u32x4 wa = u32x4{0, 0, 0, 0}, wb = wa;
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
            pf = false;
        }
        // keep kRowsRoom bytes of room; never drop unflushed bytes (F >= op - 15)
        if (op - base > kRowsH - kRowsRoom) {
            const int32_t nb = (op - kRowsKeep) & ~15;
            for (int32_t c = 16 * jj; c < op - nb; c += 256) lds_st16(HB + c, lds_ld16(HB + (nb - base) + c));
            base = nb;
        }
        // ---- the round: lane jj takes sequence k0 + jj
        const int32_t k = k0 + jj;
        const bool act = k < nseq;
        if (!pf) {   // block start, or the last round stopped early: load now
            dc = act ? (int32_t)dl[k] : 0;
            tc = ip + row_incl_sum(dc) - dc;
            load32(s, tc, iend, act, wa, wb);
            dn = k + 16 < nseq ? (int32_t)dl[k + 16] : 0;
        }
        const int32_t t = tc, dlt = dc;
        const bool esc = dlt == 255;   // length >= 255: the parse left it to be re-parsed
        const uint32_t tok = wa.x & 0xFFu;
        int32_t lit = (int32_t)(tok >> 4), lp = 1;
        if (lit == 15) {
            lit += (int32_t)byte_of(wa, 1);   // one extra byte unless the length escaped
            lp = 2;
        }
        const int32_t po = lp + lit;
        int32_t off = 0, ml = (int32_t)(tok & 15u);
        bool slow = false;
        if (lit <= 12) {
            off = (int32_t)(window_dword(wa, (uint32_t)po) & 0xFFFFu);
            if (ml == 15) {
                const int32_t e = (int32_t)byte_of(wa, po + 2);
                ml += e;
                slow = e == 255;
            }
        } else if (po + 3 <= 32) {
            off = (int32_t)(dword32(wa, wb, (uint32_t)po) & 0xFFFFu);
            if (ml == 15) {
                const int32_t e = (int32_t)((dword32(wa, wb, (uint32_t)(po + 2 < 28 ? po + 2 : 28)) >> (8 * (po + 2 - (po + 2 < 28 ? po + 2 : 28)))) & 0xFFu);
                ml += e;
                slow = e == 255;
            }
        } else {
            slow = true;
        }
        if (slow && act && !esc) {   // a long match length or the offset past 32 bytes: from HBM
            const uint8_t* q = s + t;
            off = (int32_t)q[po] | ((int32_t)q[po + 1] << 8);
            ml = (int32_t)(tok & 15u);
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
        const int32_t o = op + row_incl_sum(len) - len;
        const int32_t m = o + lit, mend = m + ml;
        const bool ok = act && !esc && mend <= base + kRowsH;
        const uint32_t rb = (uint32_t)(__ballot(!ok) >> (16 * r)) & 0xFFFFu;
        const int32_t use = rb ? __builtin_ctz(rb) : 16;
        if (use == 0) {
            pf = false;
            if (k0 >= nseq) {   // the block's good prefix is done: flush the rest exactly
                for (int32_t c = F + 16 * jj; c < op; c += 256) gbl_put(d + c, lds_ld16(HB + (c - base)), op - c);
                have = false;
                continue;
            }
            // one sequence that does not fit the buffers: flush, copy it in
            // HBM on the row, reload the history
            // (the parse verified it: every read below stays inside the block)
            const uint32_t tk = s[ip];
            int32_t L = (int32_t)(tk >> 4), q = ip + 1;
            if (L == 15) {
                uint32_t b;
                do {
                    b = s[q];
                    ++q;
                    L += (int32_t)b;
                } while (b == 255 && q < iend);
            }
            const int32_t ofs = (int32_t)s[q + L] | ((int32_t)s[q + L + 1] << 8);
            int32_t qe = q + L + 2, M = (int32_t)(tk & 15u);
            if (M == 15) {
                uint32_t b;
                do {
                    b = s[qe];
                    ++qe;
                    M += (int32_t)b;
                } while (b == 255 && qe < iend);
            }
            M += 4;
            for (int32_t c = F + 16 * jj; c < op; c += 256) gbl_put(d + c, lds_ld16(HB + (c - base)), op - c);
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
            row_copy_literal(d + op, s + q, L, jj);
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
            row_copy_match(d + op + L, ofs, M, jj);
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
            op += L + M;
            ip = qe;
            k0 += 1;
            base = (op > kRowsKeep ? op - kRowsKeep : 0) & ~15;
            // op < oend - 64: the 16-byte reads stay inside the block's slot
            for (int32_t c = base + 16 * jj; c < op; c += 256) lds_st16(HB + (c - base), ld16(d + c));
            F = op;
            continue;
        }
        const bool u = jj < use;
        const int32_t opn = op + row_last(row_incl_sum(u ? len : 0));
        const int32_t ipn = ip + row_last(row_incl_sum(u ? dlt : 0));
        // the next round's lengths and bytes, requested now (valid if this
        // round takes all 16 sequences)
        const bool pfn = use == 16;
        int32_t tn = 0, dn2 = 0;
        u32x4 na = u32x4{0, 0, 0, 0}, nb2 = na;
        if (pfn) {
            const int32_t kn = k0 + 16 + jj;
            tn = ipn + row_incl_sum(dn) - dn;
            load32(s, tn, iend, kn < nseq, na, nb2);
            dn2 = kn + 16 < nseq ? (int32_t)dl[kn + 16] : 0;
        }
        const int32_t s0 = m - off;
        // sources older than the buffer: their first 32 bytes are requested now
        const bool far = u && s0 < base;
        u32x4 pre0 = u32x4{0, 0, 0, 0}, pre1 = pre0;
        if (far) {
            pre0 = ld16(d + s0);
            if (ml > 16) pre1 = ld16(d + s0 + 16);
        }
        if (u && lit > 0) {
            if (lit <= 12) {
                lds_put(HB + (o - base), window_shift1(wa), lit);
            } else if (lp + lit <= 32) {
                const uint32_t sh = (uint32_t)lp;
                const u32x4 x0 = u32x4{__builtin_amdgcn_alignbyte(wa.y, wa.x, sh), __builtin_amdgcn_alignbyte(wa.z, wa.y, sh),
                                       __builtin_amdgcn_alignbyte(wa.w, wa.z, sh), __builtin_amdgcn_alignbyte(wb.x, wa.w, sh)};
                const u32x4 x1 = u32x4{__builtin_amdgcn_alignbyte(wb.y, wb.x, sh), __builtin_amdgcn_alignbyte(wb.z, wb.y, sh),
                                       __builtin_amdgcn_alignbyte(wb.w, wb.z, sh), __builtin_amdgcn_alignbyte(0u, wb.w, sh)};
                lds_put(HB + (o - base), x0, lit);
                if (lit > 16) lds_put(HB + (o - base + 16), x1, lit - 16);
            } else {   // a literal beyond the 32 bytes: from HBM (inside the block: good)
                for (int32_t i = 0; i < lit; i += 16) lds_put(HB + (o - base + i), ld16(s + t + lp + i), lit - i);
            }
        }
        // readiness passes: a match is copied once no earlier pending match of
        // the round writes into its source [s0, se)
        const int32_t se = s0 + (off < ml ? off : ml);
        bool pend = u;
        while (__any(pend)) {
            const int32_t x = row_excl_max(pend ? mend : -1);
            const int32_t y = row_excl_min(pend ? m : INT_MAX);
            const bool ready = pend && (x <= s0 || se <= y);
            if (ready) {
                if (off >= 16) {
                    for (int32_t i = 0; i < ml; i += 16) {
                        const int32_t sp = s0 + i;
                        // sp < base: flushed (F >= base + kRowsKeep - 16)
                        const u32x4 v = (far && i < 32) ? (i == 0 ? pre0 : pre1)
                                                        : sp >= base ? lds_ld16(HB + (sp - base)) : ld16(d + sp);
                        lds_put(HB + (m - base + i), v, ml - i);
                    }
                } else {   // s0 >= base: m - base >= off here
                    const u32x4 pat = period_pattern(lds_ld16(HB + (s0 - base)), (uint32_t)off);
                    const int32_t step = 16 - (16 % off);
                    for (int32_t i = 0; i < ml; i += step) lds_put(HB + (m - base + i), pat, ml - i);
                }
            }
            pend = pend && !ready;
        }
        if (pfn) {
            dc = dn;
            tc = tn;
            wa = na;
            wb = nb2;
            dn = dn2;
        }
        pf = pfn;
        for (int32_t c = F + 16 * jj; c + 16 <= opn; c += 256) st16(d + c, lds_ld16(HB + (c - base)));
        F += (opn - F) & ~15;
        op = opn;
        ip = ipn;
        k0 += use;
    }
}

}  // namespace lz4m

using namespace lz4m;

extern "C" size_t lz4m_rows_fixed_bytes(int64_t n) { return 64 + (size_t)n * sizeof(RowMeta); }

extern "C" int lz4m_rows_launch(const uint8_t* d_src, const int64_t* d_src_off, const int32_t* d_src_len,
                                uint8_t* d_dst, const int64_t* d_dst_off, const int32_t* d_dst_cap, int64_t n,
                                void* d_work, size_t work_bytes, int parse_grid, int exec_grid, hipStream_t stream) {
    const size_t fixed = lz4m_rows_fixed_bytes(n);
    if (work_bytes < fixed) return LZ4M_ROWS_ENOSPACE;
    unsigned long long* ctr = static_cast<unsigned long long*>(d_work);
    RowMeta* meta = reinterpret_cast<RowMeta*>(static_cast<uint8_t*>(d_work) + 64);
    uint8_t* lens = static_cast<uint8_t*>(d_work) + fixed;
    const int64_t lens_cap = (int64_t)(work_bytes - fixed);
    hipError_t e = hipMemsetAsync(ctr, 0, 64, stream);
    if (e != hipSuccess) return (int)e;
    hipLaunchKernelGGL(rows_parse_kernel, dim3((uint32_t)parse_grid), dim3(256), 0, stream, d_src, d_src_off,
                       d_src_len, d_dst_cap, n, meta, lens, lens_cap, ctr);
    hipLaunchKernelGGL(rows_exec_kernel, dim3((uint32_t)exec_grid), dim3(64), 0, stream, d_src, d_src_off, d_src_len,
                       d_dst, d_dst_off, meta, lens, n, ctr);
    return (int)hipGetLastError();
}

extern "C" int lz4m_rows_grids(int64_t n, int* parse_grid, int* exec_grid) {
    int dev = 0, cus = 0, pk = 0, ek = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&pk, reinterpret_cast<const void*>(rows_parse_kernel), 256, 0);
    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&ek, reinterpret_cast<const void*>(rows_exec_kernel), 64, 0);
    if (cus <= 0) cus = 256;
    const int64_t ps = (int64_t)cus * (pk > 0 ? pk : 1), es = (int64_t)cus * (ek > 0 ? ek : 1);
    const int64_t pneed = (n + 255) / 256, eneed = (n + 3) / 4;
    *parse_grid = (int)(pneed < ps ? pneed : ps);
    *exec_grid = (int)(eneed < es ? eneed : es);
    return 0;
}
