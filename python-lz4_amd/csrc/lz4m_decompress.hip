// lz4m_decompress.hip -- batched LZ4 block decoder for MI355X (gfx950).
//
// Bit-exact restatement of LZ4_decompress_safe / _usingDict (reference
// lz4libs/lz4.c:1936-2339, x86_64 build with LZ4_FAST_DEC_LOOP=1): same
// decoded bytes, same accept/reject decisions, same error position.
//
// Mapping.  One LANE owns one block and walks its sequences with the
// reference's two-phase state machine (fast phase while >= 64 bytes of
// output room, sticky switch to the safe phase).  A 64-lane wavefront thus
// parses 64 blocks at once, so the serial token chain of each block costs one
// lane, not one wave.  Short copies (the common case on compressible data:
// literals <= 14 B, matches <= 18 B) are done by the owning lane with 16-byte
// unaligned loads/stores.  Copies longer than kCoopMin are deferred: after
// every sequence step the wave runs a cooperative phase in which all 64 lanes
// execute each deferred copy at 1 KiB per wave instruction (coalesced), in
// lane order, literal before match.  Incompressible blocks (one long literal
// run) and run-length-heavy blocks therefore stream at wave width.
//
// Memory: compressed input is read once; the decoded output is written once
// and match sources are re-read from the block's own output (L1/L2 hits, the
// window is <= 64 KiB behind).  Algorithmic HBM bytes per block =
// compressed size + decoded size.
#include "lz4m_common.h"
#include "lz4m_rows.h"
#include "lz4m_worker.h"
#include "../../include/lz4m.h"

#include <stdlib.h>
#include <string.h>

#include <atomic>
#include <mutex>

namespace lz4m {

constexpr int64_t kCoopMin = 64;     // copies longer than this go wave-cooperative

enum CopyKind : int { kNone = 0, kLiteral = 1, kMatch = 2 };

struct Copy {
    int kind;
    int64_t dpos;    // destination position in the block's output
    int64_t arg;     // literal: source position in the input; match: offset
    int64_t len;
};

struct Lane {
    const uint8_t* src;
    uint8_t* dst;
    const uint8_t* dict_end;
    int64_t iend, oend, dict_len;
    int64_t ip, op;
    int32_t result;
    bool fast, live;
};

// Store exactly k (0..16) bytes of v at p (any alignment).
__device__ __forceinline__ void put_exact(uint8_t* p, u32x4 v, uint32_t k) {
    if (k == 16) {
        st16(p, v);
        return;
    }
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

// ------------------------------------------------ input reads (general path)
// The general state machine reads the compressed block byte by byte (length
// bytes, offsets) and in 16-byte pieces (token window, literals).
__device__ __forceinline__ uint32_t in_byte(const Lane& L, int64_t p) { return L.src[p]; }

__device__ __forceinline__ u32x4 in16(const Lane& L, int64_t p) { return ld16_guarded(L.src + p, L.iend - p); }

__device__ __forceinline__ uint32_t in_le16(const Lane& L, int64_t p) {
    return in_byte(L, p) | (in_byte(L, p + 1) << 8);
}

// ---------------------------------------------------------------- lane copies
// Non-overlapping copy by the owning lane.  Reads never pass s_room, writes
// never pass d_room (the block's own buffers); inside those bounds the tail
// may be copied as a full 16-byte chunk, like the reference's wild copies.
__device__ __forceinline__ void lane_copy(uint8_t* d, const uint8_t* s, int64_t len, int64_t d_room,
                                          int64_t s_room) {
    for (int64_t i = 0; i < len; i += 16) {
        if (len - i >= 16 || (d_room - i >= 16 && s_room - i >= 16)) {
            st16(d + i, ld16(s + i));
        } else {
            for (int64_t k = i; k < len; ++k) d[k] = s[k];
        }
    }
}

// Overlapping LZ77 copy d[j] = d[j - off] (zeros when off == 0, lz4.c:478-485,
// 2300-2307), by the owning lane.
__device__ __forceinline__ void lane_match(uint8_t* d, int64_t off, int64_t len, int64_t room) {
    if (off >= 16) {
        for (int64_t i = 0; i < len; i += 16) {
            if (len - i >= 16 || room - i >= 16) {
                st16(d + i, ld16(d + i - off));
            } else {
                for (int64_t k = i; k < len; ++k) d[k] = d[k - off];
            }
        }
        return;
    }
    u32x4 pat;
    int64_t step;
    if (off == 0) {
        pat = u32x4{0, 0, 0, 0};
        step = 16;
    } else {
        // the `off` bytes before d are final; read them (never past the slot)
        const u32x4 w = ld16_guarded(d - off, off + (room < 16 - off ? room : 16 - off));
        pat = period_pattern(w, (uint32_t)off);
        step = 16 - (16 % off);
    }
    for (int64_t i = 0; i < len; i += step) {
        if (room - i >= 16) {
            st16(d + i, pat);
        } else {
            const int64_t e = len - i < 16 ? len - i : 16;
            for (int k = 0; k < e; ++k) d[i + k] = (uint8_t)byte_of(pat, k);
        }
    }
}

// ---------------------------------------------------------- wave copies
// All 64 lanes execute the same copy (uniform arguments).
// Literal bytes never overlap their destination, so each lane requests four
// 16-byte pieces before storing any: a long literal (a stored-looking block's
// 64 KiB) waits on one memory round trip per 4 KiB instead of per 1 KiB.
// SL: s points into LDS (the lone-block decoder's staged input): LDS reads,
// which wait on no store, where a flat read of LDS waits for every store the
// wave has in flight (one L2 write round trip per 4 KiB of a long literal).
template <int kU = 4, bool SL = false>   // kU: pieces per lane per round trip (1 where registers are short: the dictionary kernel)
__device__ __forceinline__ void wave_literal(uint8_t* d, const uint8_t* s, int64_t len, int64_t d_room,
                                             int64_t s_room, uint32_t lane) {
    for (int64_t base = 0; base < len; base += 16 * kWave * kU) {
        u32x4 v[kU];
#pragma unroll
        for (int u = 0; u < kU; ++u) {
            const int64_t pos = base + 16 * kWave * u + 16 * (int64_t)lane;
            const bool whole = pos < len && (len - pos >= 16 || s_room - pos >= 16);
            if constexpr (SL)
                v[u] = whole ? lds_ld16a((const lds_u8*)(s + pos)) : u32x4{0, 0, 0, 0};
            else
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

__device__ __forceinline__ void wave_match(uint8_t* d, int64_t off, int64_t len, int64_t room, uint32_t lane) {
    if (off >= 16) {
        // rows of W bytes whose sources all lie before the row: W <= off
        const int64_t w_bytes = ((off < 16 * kWave ? off : 16 * kWave) / 16) * 16;
        for (int64_t base = 0; base < len; base += w_bytes) {
            const int64_t pos = base + 16 * (int64_t)lane;
            if (16 * (int64_t)lane < w_bytes && pos < len) {
                if (len - pos >= 16 || room - pos >= 16) {
                    st16(d + pos, ld16(d + pos - off));
                } else {
                    for (int64_t k = pos; k < len; ++k) d[k] = d[k - off];
                }
            }
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
        }
        return;
    }
    u32x4 pat;
    int64_t step;
    if (off == 0) {
        pat = u32x4{0, 0, 0, 0};
        step = 16;
    } else {
        const u32x4 w = ld16_guarded(d - off, off + (room < 16 - off ? room : 16 - off));
        pat = period_pattern(w, (uint32_t)off);
        step = 16 - (16 % off);
    }
    for (int64_t base = 0; base < len; base += step * kWave) {
        const int64_t pos = base + step * (int64_t)lane;
        if (pos < len) {
            if (room - pos >= 16) {
                st16(d + pos, pat);
            } else {
                const int64_t e = len - pos < 16 ? len - pos : 16;
                for (int k = 0; k < e; ++k) d[pos + k] = (uint8_t)byte_of(pat, k);
            }
        }
    }
}

// ------------------------------------------------------------ lane decode
// read_variable_length (lz4.c:1903-1928).  On failure *ip is the position
// the reference reports.
__device__ __forceinline__ bool read_len(const Lane& L, int64_t& ip, int64_t ilimit, bool initial_check,
                                         int64_t& out) {
    if (initial_check && ip >= ilimit) return false;
    {
        // 16 bytes per load: a run of 255s (a long literal or match, e.g. the
        // 257 length bytes of a stored-looking 64 KiB block) costs one memory
        // round trip per 16 bytes instead of per byte.  Same outcome as the
        // byte loop below: reading the byte at ilimit fails with
        // ip = ilimit + 1 (ilimit < iend, so every byte up to it is readable;
        // ld16_guarded zero-fills past iend, i.e. past ilimit).
        if (ip >= ilimit) {   // the first byte read already fails (ip + 1)
            ++ip;
            return false;
        }
        int64_t len = 0;
        for (;;) {
            const u32x4 v = ld16_guarded(L.src + ip, L.iend - ip);
            const uint32_t n0 = ~v.x, n1 = ~v.y, n2 = ~v.z, n3 = ~v.w;
            const uint32_t q = n0 ? 0u : n1 ? 1u : n2 ? 2u : n3 ? 3u : 4u;
            if (q < 4) {
                const uint32_t nw = q == 0 ? n0 : q == 1 ? n1 : q == 2 ? n2 : n3;
                const uint32_t bi = (uint32_t)__builtin_ctz(nw) >> 3;
                const uint32_t j = 4 * q + bi;   // first byte != 255
                if (ip + (int64_t)j >= ilimit) {
                    ip = ilimit + 1;
                    return false;
                }
                len += 255 * (int64_t)j + (int64_t)((~nw >> (8 * bi)) & 0xFFu);   // no indexed access: no scratch
                ip += j + 1;
                out = len;
                return true;
            }
            if (ip + 16 > ilimit) {   // the run reaches ilimit
                ip = ilimit + 1;
                return false;
            }
            len += 255 * 16;
            ip += 16;
        }
    }
}

__device__ __forceinline__ void emit_literal(Lane& L, int64_t ip, int64_t op, int64_t lit, Copy& c,
                                             bool deferred) {
    if (lit == 0) return;
    if (deferred || lit > kCoopMin) {
        c = Copy{kLiteral, op, ip, lit};
    } else {
        lane_copy(L.dst + op, L.src + ip, lit, L.oend - op, L.iend - ip);
    }
}

__device__ __forceinline__ void emit_match(Lane& L, int64_t op, int64_t off, int64_t ml, Copy& c, bool deferred) {
    if (deferred || ml > kCoopMin) {
        c = Copy{kMatch, op, off, ml};
    } else {
        lane_match(L.dst + op, off, ml, L.oend - op);
    }
}

// Literal bytes 1..lit (lit <= 14) of the token window.
__device__ __forceinline__ void window_literal(Lane& L, int64_t op, u32x4 w, int64_t lit) {
    st16(L.dst + op, window_shift1(w));   // wild 16-byte store, inside the oend-32 margin
}

// Match that starts inside the external dictionary (lz4.c:2252-2277).
// Rare; done by the owning lane.
__device__ __noinline__ void dict_match(Lane& L, int64_t op, int64_t off, int64_t ml) {
    const int64_t in_dict = off - op;
    uint8_t* d = L.dst + op;
    const uint8_t* s = L.dict_end - in_dict;
    if (ml <= in_dict) {
        for (int64_t k = 0; k < ml; ++k) d[k] = s[k];
    } else {
        for (int64_t k = 0; k < in_dict; ++k) d[k] = s[k];
        const int64_t rest = ml - in_dict;
        uint8_t* d2 = d + in_dict;
        const int64_t off2 = op + in_dict;   // continues from the block start
        for (int64_t k = 0; k < rest; ++k) d2[k] = d2[k - off2];
    }
}

// One sequence of block L.  Deferred copies land in lc / mc.
template <bool DICT>
__device__ __forceinline__ void decode_step(Lane& L, Copy& lc, Copy& mc) {
    const u32x4 w = in16(L, L.ip);
    const uint32_t tok = w.x & 0xFFu;
    int64_t ip = L.ip + 1;
    int64_t op = L.op;
    int64_t lit = tok >> 4, ml, off, add;
    bool deferred = false;
    const int64_t iend = L.iend, oend = L.oend;
    const int64_t dlen = DICT ? L.dict_len : 0;
    const bool check_window = dlen < 65536;
#define OOW(o) (check_window && (o) > op + dlen)

    if (L.fast) {   // lz4.c:1996-2109
        if (lit == 15) {
            if (!read_len(L, ip, iend - 15, true, add)) goto fail;
            lit += add;
            if (op + lit > oend - 32 || ip + lit > iend - 32) {
                L.fast = false;
                goto literal_tail;
            }
            emit_literal(L, ip, op, lit, lc, false);
            deferred = lc.kind != kNone;
            ip += lit;
            op += lit;
            off = in_le16(L, ip);
        } else {
            if (ip > iend - 17) {
                L.fast = false;
                goto literal_tail;
            }
            // literals are bytes 1..lit of the token window
            window_literal(L, op, w, lit);
            off = lit <= 13 ? (window_dword(w, (uint32_t)(1 + lit)) & 0xFFFFu) : in_le16(L, ip + lit);
            ip += lit;
            op += lit;
        }
        ip += 2;
        ml = tok & 15;
        if (ml == 15) {
            if (!read_len(L, ip, iend - 4, false, add)) goto fail;
            ml += add + 4;
            if (OOW(off)) goto fail;
            if (op + ml >= oend - 64) {
                L.fast = false;
                goto match_tail;
            }
        } else {
            ml += 4;
            if (op + ml >= oend - 64) {
                L.fast = false;
                goto match_tail;
            }
            if (off >= 8 && off <= op) {
                emit_match(L, op, off, ml, mc, deferred);
                op += ml;
                goto done;
            }
        }
        if (OOW(off)) goto fail;
        if (DICT && off > op) {
            if (op + ml > oend - 5) goto fail;
            if (deferred) goto defer_dict;
            dict_match(L, op, off, ml);
            op += ml;
            goto done;
        }
        emit_match(L, op, off, ml, mc, deferred);
        op += ml;
        goto done;
    }

    // safe phase, lz4.c:2114-2329
    if (lit != 15 && ip < iend - 16 && op <= oend - 32) {   // shortcut, lz4.c:2128-2158
        window_literal(L, op, w, lit);
        off = lit <= 13 ? (window_dword(w, (uint32_t)(1 + lit)) & 0xFFFFu) : in_le16(L, ip + lit);
        op += lit;
        ip += lit + 2;
        ml = tok & 15;
        if (ml != 15 && off >= 8 && off <= op) {
            lane_match(L.dst + op, off, ml + 4, oend - op);
            op += ml + 4;
            goto done;
        }
        goto match_length;
    }
    if (lit == 15) {
        if (!read_len(L, ip, iend - 15, true, add)) goto fail;
        lit += add;
    }
literal_tail:   // lz4.c:2172-2229
    if (op + lit > oend - 12 || ip + lit > iend - 8) {
        if (ip + lit != iend || op + lit > oend) goto fail;
        emit_literal(L, ip, op, lit, lc, false);   // last literals: exact (never past oend / iend)
        op += lit;
        L.result = (int32_t)op;
        L.live = false;
        L.op = op;
        return;
    }
    emit_literal(L, ip, op, lit, lc, false);
    deferred = lc.kind != kNone;
    ip += lit;
    op += lit;
    off = in_le16(L, ip);
    ip += 2;
    ml = tok & 15;
match_length:   // lz4.c:2238-2245
    if (ml == 15) {
        if (!read_len(L, ip, iend - 4, false, add)) goto fail;
        ml += add;
    }
    ml += 4;
match_tail:   // lz4.c:2248-2328
    if (OOW(off)) goto fail;
    if (DICT && off > op) {
        if (op + ml > oend - 5) goto fail;
        if (deferred) goto defer_dict;
        dict_match(L, op, off, ml);
        op += ml;
        goto done;
    }
    if (op + ml > oend - 5) goto fail;
    emit_match(L, op, off, ml, mc, deferred);
    op += ml;
done:
    L.ip = ip;
    L.op = op;
    return;
defer_dict:
    // a dictionary match behind a deferred literal: run it right after the
    // cooperative phase by re-entering with a pending marker
    mc = Copy{kMatch, op, -off, ml};   // negative offset marks "dictionary"
    op += ml;
    goto done;
fail:
    L.result = (int32_t)(-ip - 1);
    L.live = false;
    return;
#undef OOW
}

// RESUME (the finisher of the large-batch decoder, lz4m_rows.hip): every
// block starts at the reference's state after its good prefix, resume[i].ip /
// .op, which rows_exec_kernel has already written to dst.
template <bool DICT, bool RESUME = false>
__global__ __launch_bounds__(256) void decompress_kernel(const uint8_t* __restrict__ src,
                                                         const int64_t* __restrict__ src_off,
                                                         const int32_t* __restrict__ src_len, uint8_t* dst,
                                                         const int64_t* __restrict__ dst_off,
                                                         const int32_t* __restrict__ dst_cap,
                                                         const uint8_t* __restrict__ dict,
                                                         const int64_t* __restrict__ dict_off,
                                                         const int32_t* __restrict__ dict_len,
                                                         int32_t* __restrict__ status, int64_t n,
                                                         const RowMeta* __restrict__ resume = nullptr) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t lane = lane_id();
    Lane L;
    L.live = false;
    L.result = -1;
    if (i < n) {
        L.src = src + src_off[i];
        L.dst = dst + dst_off[i];
        L.iend = src_len[i];
        L.oend = dst_cap[i];
        L.ip = 0;
        L.op = 0;
        L.dict_len = 0;
        L.dict_end = nullptr;
        if (DICT) {
            L.dict_len = dict_len[i];
            L.dict_end = dict + dict_off[i] + L.dict_len;
        }
        if (L.oend < 0) {
            L.result = -1;   // lz4.c:1950
        } else if (L.oend == 0) {
            L.result = (L.iend == 1 && L.src[0] == 0) ? 0 : -1;   // lz4.c:1978-1982
        } else if (L.iend <= 0) {
            L.result = -1;   // lz4.c:1983
        } else {
            L.fast = L.oend >= 64;
            L.live = true;
            if (RESUME) {
                L.ip = resume[i].ip;
                L.op = resume[i].op;
                if (L.ip < 0) {   // a whole-literal block, decoded by rows_parse_kernel: op = its size
                    L.result = L.op;
                    L.live = false;
                }
            }
        }
    }

    while (__any(L.live)) {
        Copy lc{kNone, 0, 0, 0}, mc{kNone, 0, 0, 0};
        if (L.live) decode_step<DICT>(L, lc, mc);
        uint64_t pend = __ballot(lc.kind != kNone || mc.kind != kNone);
        if (pend == 0) continue;
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");   // lane stores visible to the wave
        while (pend) {
            const int l = __builtin_ctzll(pend);
            pend &= pend - 1;
            uint8_t* d = readlane_ptr(L.dst, l);
            const int64_t oend = readlane64(L.oend, l);
            const int lk = __builtin_amdgcn_readlane(lc.kind, l);
            if (lk != kNone) {
                const uint8_t* s = readlane_ptr(L.src, l);
                const int64_t iend = readlane64(L.iend, l);
                const int64_t dp = readlane64(lc.dpos, l), sp = readlane64(lc.arg, l), ln = readlane64(lc.len, l);
                wave_literal(d + dp, s + sp, ln, oend - dp, iend - sp, lane);
                __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
            }
            const int mk = __builtin_amdgcn_readlane(mc.kind, l);
            if (mk != kNone) {
                const int64_t dp = readlane64(mc.dpos, l), off = readlane64(mc.arg, l), ln = readlane64(mc.len, l);
                if (DICT && off < 0) {
                    if (lane == (uint32_t)l) dict_match(L, dp, -off, ln);
                } else {
                    wave_match(d + dp, off, ln, oend - dp, lane);
                }
                __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
            }
        }
    }
    if (i < n) status[i] = L.result;
}



// ------------------------------------------------- cooperative (small batches)
// One wavefront per block, for batches too small to fill the lane decoder
// (it needs ~1 M blocks for full rate: a lane decodes 64 KiB in ~34 ms) --
// single-block calls, and frames of 4 MiB blocks (2 048 lanes).  The wave
// decodes the block's fast-loop prefix cooperatively, then lane 0 finishes the
// block with the exact state machine (decode_step, as the chain kernel does).
//
// A round takes up to 64 sequences: the wave stages 1 KiB of input in LDS,
// every lane parses a speculative sequence at position pos + lane, and a
// readlane walk follows the chain of starts; sequence k is then re-parsed in
// lane k, a prefix sum places it, literals are written, and matches are copied
// in passes (a match is ready once its source ends before the first pending
// match's start, so everything it reads is final).  Longer literals run one
// sequence at a time on the whole wave.  A sequence is taken only when the
// reference provably stays in its fast loop and succeeds on it (lz4.c:2004-2110:
// ip + 1 <= iend - 17 or the long-literal margins, a single match-length byte
// inside iend - 4, 1 <= offset <= output so far, op + ml < oend - 64);
// anything else -- the tail, offset 0, errors -- goes to the exact path with
// the state the reference would have, so bytes and statuses are identical.
constexpr int kCoopIn = 1024;

__device__ __forceinline__ void coop_put(uint8_t* p, u32x4 v, int32_t k) {
    if (k >= 16) {
        st16(p, v);
    } else if (k > 0) {
        put_exact(p, v, (uint32_t)k);
    }
}

__device__ __forceinline__ int32_t coop_incl_sum(int32_t v) {
    v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xF, 0xF, false);   // row_shr:1
    v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xF, 0xF, false);   // row_shr:2
    v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xF, 0xF, false);   // row_shr:4
    v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xF, 0xF, false);   // row_shr:8
    v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xA, 0xF, false);   // row_bcast:15
    v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xC, 0xF, false);   // row_bcast:31
    return v;
}

// Exact-length whole-wave copies (no wild bytes: other sequences' output may
// already sit right after them).
template <bool SL = false>   // SL: s points into LDS (as wave_literal)
__device__ __forceinline__ void coop_copy_literal(uint8_t* d, const uint8_t* s, int32_t len, uint32_t lane) {
    constexpr int kU = 4;   // four pieces requested before any is stored (as wave_literal)
    for (int32_t base = 0; base < len; base += 16 * kWave * kU) {
        u32x4 v[kU];
#pragma unroll
        for (int u = 0; u < kU; ++u) {
            const int32_t pos = base + 16 * kWave * u + 16 * (int32_t)lane;
            if constexpr (SL)
                v[u] = pos < len ? lds_ld16a((const lds_u8*)(s + pos)) : u32x4{0, 0, 0, 0};
            else
                v[u] = pos < len ? ld16(s + pos) : u32x4{0, 0, 0, 0};
        }
#pragma unroll
        for (int u = 0; u < kU; ++u) {
            const int32_t pos = base + 16 * kWave * u + 16 * (int32_t)lane;
            if (pos < len) coop_put(d + pos, v[u], len - pos);
        }
    }
}

__device__ __forceinline__ void coop_copy_match(uint8_t* d, int32_t off, int32_t len, uint32_t lane) {
    if (off >= 16) {
        const int32_t w = (off < 16 * kWave ? off : 16 * kWave) & ~15;   // rows whose sources precede them
        for (int32_t base = 0; base < len; base += w) {
            const int32_t pos = base + 16 * (int32_t)lane;
            if (pos < base + w && pos < len) coop_put(d + pos, ld16(d + pos - off), len - pos);
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
        }
        return;
    }
    const u32x4 pat = period_pattern(ld16(d - off), (uint32_t)off);
    const int32_t step = 16 - (16 % off);
    for (int32_t pos = step * (int32_t)lane; pos < len; pos += step * kWave) coop_put(d + pos, pat, len - pos);
}

// The sequence starting at t (relative to the LDS input window), w = its
// first 16 bytes.  `simple`: parallel-path material -- at most one extra
// length byte each for literal and match (< 255), and the whole sequence
// inside the window.  Literals of <= 12 bytes come from w, longer ones from LDS.
struct CoopSeq {
    int32_t lit, litpos, off, ml, adv;
    bool simple, litx, mlx;
};

__device__ __forceinline__ CoopSeq coop_parse(const lds_u8* IN, int32_t t, u32x4 w) {
    CoopSeq q;
    const uint32_t tok = w.x & 0xFFu, mlc = tok & 15u;
    int32_t lit = (int32_t)(tok >> 4);
    q.litx = lit == 15;
    q.mlx = mlc == 15;
    q.simple = true;
    if (lit <= 12) {
        q.lit = lit;
        q.litpos = t + 1;
        q.off = (int32_t)(window_dword(w, (uint32_t)(1 + lit)) & 0xFFFFu);
        q.ml = (int32_t)mlc + 4;
        q.adv = 3 + lit;
        if (q.mlx) {
            const uint32_t e = byte_of(w, 3 + lit);
            q.simple = e != 255u;
            q.ml = 19 + (int32_t)e;
            q.adv += 1;
        }
        return q;
    }
    int32_t lp = t + 1;
    if (q.litx) {
        const uint32_t b = IN[t + 1];
        q.simple = b != 255u;
        lit += (int32_t)b;
        lp = t + 2;
    }
    q.lit = lit;
    q.litpos = lp;
    const int32_t po = lp + lit;   // offset position
    q.simple = q.simple && po + 3 + 16 <= kCoopIn;
    const int32_t pc = q.simple ? po : 0;
    q.off = (int32_t)IN[pc] | ((int32_t)IN[pc + 1] << 8);
    q.ml = (int32_t)mlc + 4;
    q.adv = po + 2 - t;
    if (q.mlx) {
        const uint32_t e = IN[pc + 2];
        q.simple = q.simple && e != 255u;
        q.ml = 19 + (int32_t)e;
        q.adv += 1;
    }
    return q;
}

// The block's rest from (ip, op) with the exact state machine on lane 0 and
// long copies on the whole wave (as decompress_chain_kernel); returns the
// reference's result (decoded size or -(error position)-1).  Output [0, op)
// must already be in HBM and visible to the wave.
// DICT: the dlen bytes before dict_end are the block's dictionary
// (LZ4_decompress_safe_usingDict, as decompress_kernel<true>).  SL: s points
// into LDS (long literals read as LDS, wave_literal).
template <bool DICT = false, bool SL = false>
__device__ __forceinline__ int32_t coop_finish(const uint8_t* s, uint8_t* d, int32_t iend, int32_t oend, int32_t ip,
                                               int32_t op, bool fast, uint32_t lane, int32_t dlen = 0,
                                               const uint8_t* dict_end = nullptr) {
    Lane L;
    L.live = false;
    L.result = -1;
    if (lane == 0) {
        L.src = s;
        L.dst = d;
        L.iend = iend;
        L.oend = oend;
        L.ip = ip;
        L.op = op;
        L.dict_len = DICT ? dlen : 0;
        L.dict_end = DICT ? dict_end : d;
        L.fast = fast;
        L.live = true;
    }
    while (__any(L.live)) {
        Copy lc{kNone, 0, 0, 0}, mc{kNone, 0, 0, 0};
        if (L.live) decode_step<DICT>(L, lc, mc);
        if (__ballot(lc.kind != kNone || mc.kind != kNone) == 0) continue;
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
        const int64_t oe = readlane64(L.oend, 0);
        if (__builtin_amdgcn_readlane(lc.kind, 0) != kNone) {
            const int64_t ie = readlane64(L.iend, 0);
            const int64_t dp = readlane64(lc.dpos, 0), sp = readlane64(lc.arg, 0), ln = readlane64(lc.len, 0);
            wave_literal<DICT ? 1 : 4, SL>(d + dp, s + sp, ln, oe - dp, ie - sp, lane);   // DICT: registers are short
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
        }
        if (__builtin_amdgcn_readlane(mc.kind, 0) != kNone) {
            const int64_t dp = readlane64(mc.dpos, 0), mo = readlane64(mc.arg, 0), ln = readlane64(mc.len, 0);
            if (DICT && mo < 0) {   // starts in the dictionary (the chain kernel's convention)
                if (lane == 0) dict_match(L, dp, -mo, ln);
            } else {
                wave_match(d + dp, mo, ln, oe - dp, lane);
            }
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
        }
    }
    return __builtin_amdgcn_readlane(L.result, 0);
}

// ------------------------------------ cooperative with on-chip history
// hist_decompress_kernel: the cooperative decoder above with the block's
// output assembled in an 8 KiB LDS buffer per wave instead of in HBM.  The
// buffer holds output [base, base + kHistW); a round's literals and matches
// are written there with exact byte counts, the readiness passes read match
// sources from it (an LDS round trip per pass instead of an HBM one), and
// only sources older than `base` (more than ~4 KiB back) come from HBM.  After
// each round the finished 16-byte chunks leave for HBM in one coalesced pass
// ([0, F) is in HBM).  When the buffer fills, its last kHistKeep bytes move to
// the front (rebase).  Long literals and the exact tail run on HBM as in the
// cooperative kernel: everything is flushed first and the history reloaded
// after.  The accept/reject rules are the cooperative kernel's plus "fits in
// the buffer", so statuses and bytes are identical.
constexpr int32_t kHistW = 8192;
constexpr int32_t kHistKeep = 4096;      // history kept on a rebase
constexpr int32_t kHistRebase = kHistW - 2048;
constexpr int32_t kHistRestage = 384;    // restage below this many window bytes

__device__ __forceinline__ void lds_wait() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

// A length-byte run read 32 bytes per memory round trip (wave-uniform; the
// one-sequence path of a long literal, e.g. the 257 length bytes of a stored-
// looking 64 KiB block): the same outcome as the byte loop
//   do { x = s[q++]; len += x; } while (x == 255 && q < lim)   (entered with q < lim)
// -- true with q past the first byte < 255 if that byte lies before lim, else
// false (the caller then leaves the sequence to the exact path).
__device__ __forceinline__ bool run_len32(const uint8_t* s, int32_t& q, int32_t lim, int32_t iend, int32_t& len) {
    while (q < lim) {
        u32x4 v[2];
#pragma unroll
        for (int c = 0; c < 2; ++c) {
            const int32_t x = q + 16 * c;
            v[c] = x + 16 <= iend ? ld16(s + x) : ld16_guarded(s + x, iend - x);
        }
        int32_t j = 32;   // first byte != 255 of the 32
#pragma unroll
        for (int c = 1; c >= 0; --c) {
            const uint32_t n0 = ~v[c].x, n1 = ~v[c].y, n2 = ~v[c].z, n3 = ~v[c].w;
            const int32_t w = n0 ? 0 : n1 ? 1 : n2 ? 2 : n3 ? 3 : 4;
            if (w < 4) {
                const uint32_t nw = w == 0 ? n0 : w == 1 ? n1 : w == 2 ? n2 : n3;
                j = 16 * c + 4 * w + (int32_t)(__builtin_ctz(nw) >> 3);
            }
        }
        if (q + j >= lim) return false;   // no byte < 255 before lim
        if (j < 32) {
            const u32x4 vc = j < 16 ? v[0] : v[1];
            len += 255 * j + (int32_t)byte_of(vc, j & 15);
            q += j + 1;
            return true;
        }
        len += 255 * 32;
        q += 32;
    }
    return false;
}


// DICT (linked frames, lz4m_decompress_batch_prefix): block b's dictionary
// is the dict_len[b] bytes ending at d + ddelta, where d is its output slot
// (ddelta = the distance from the output buffer to an equally laid-out
// dictionary buffer: the previous round of a linked frame).  A match whose
// whole source lies in the dictionary takes the parallel path (its bytes are
// read from there); anything else that reaches before the block goes to the
// exact state machine with the same dictionary (decode_step<true>).
// SOLO (lz4m_decompress_solo, the single-call API: n == 1, input <=
// kSoloIn bytes): the workgroup first stages the whole compressed block in
// LDS, and every input read -- the speculative parse windows, length runs,
// long literals, the exact state machine -- is an LDS read.  A lone block is
// latency-bound (a stored-looking 64 KiB block waits on ~40 dependent memory
// round trips); the batch instances are unchanged.
constexpr int32_t kSoloIn = 66 * 1024;   // > LZ4_compressBound(65536) + 64
constexpr int kSoloU = 4;               // 16-byte pieces in flight per lane when staging / copying out
template <bool DICT, bool SOLO = false>
__device__ __forceinline__ void hist_decompress_body(const uint8_t* __restrict__ src,
                                                     const int64_t* __restrict__ src_off,
                                                     const int32_t* __restrict__ src_len, uint8_t* dst,
                                                     const int64_t* __restrict__ dst_off,
                                                     const int32_t* __restrict__ dst_cap,
                                                     int32_t* __restrict__ status, int64_t n,
                                                     const int32_t* __restrict__ dict_len, int64_t ddelta,
                                                     uint8_t* solo_out, int32_t* solo_done) {
    __shared__ __attribute__((aligned(16))) uint8_t ins[4][kCoopIn + 64];
    __shared__ __attribute__((aligned(16))) uint8_t outs[4][kHistW + 32];
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    lds_u8* IN = (lds_u8*)ins[wv];
    lds_u8* OB = (lds_u8*)outs[wv];
    __shared__ __attribute__((aligned(16))) uint32_t mtab[kPutTab];
    lds_put_table_init(mtab, threadIdx.x, 256);
    __syncthreads();
    lds_cu32* MT = (lds_cu32*)mtab;
#define HPUT(p, v, k) lds_put_al((p), (v), (k), MT)
#define HLD(p) lds_ld16a(p)
    const uint8_t* solo_src = nullptr;
    __shared__ int32_t solo_r, solo_lit, solo_lip;   // SOLO: result; the stored-like fast path's length and start
    uint32_t* ts = SOLO && solo_done ? reinterpret_cast<uint32_t*>(solo_done + 1) : nullptr;   // CallMeta::work
    (void)ts;
    if constexpr (SOLO) {
        LZ4M_WTS(ts, 0);
        __shared__ __attribute__((aligned(16))) uint8_t sblk[kSoloIn];
        const uint8_t* g = src + src_off[0];
        const int32_t len = src_len[0];   // <= kSoloIn - 64 (host-checked); zeros past it
        constexpr int32_t kStep = 16 * 256;
        const int32_t lim = len + 64 < kSoloIn ? len + 64 : kSoloIn;   // the block and 64 zero bytes
        for (int32_t base0 = 0; base0 < lim; base0 += kSoloU * kStep) {   // four pieces in flight per lane (16 measured no faster over PCIe)
            u32x4 v[kSoloU];
#pragma unroll
            for (int u = 0; u < kSoloU; ++u) {
                const int32_t p = base0 + u * kStep + 16 * (int32_t)threadIdx.x;
                v[u] = p + 16 <= len ? ld16(g + p) : ld16_guarded(g + p, len - p);
            }
#pragma unroll
            for (int u = 0; u < kSoloU; ++u) {
                const int32_t p = base0 + u * kStep + 16 * (int32_t)threadIdx.x;
                if (p < lim) lds_st16((lds_u8*)sblk + p, v[u]);
            }
        }
        __syncthreads();
        LZ4M_WTS(ts, 1);
        solo_src = (const uint8_t*)sblk;
        // A stored-like block -- one literal run to the end of the input, what
        // LZ4 makes of incompressible data -- is one length read and one copy
        // in the reference too (lz4.c:2000-2010 read_variable_length, then the
        // last-literals branch :2205-2229 with ip + length == iend, op +
        // length <= oend).  With the token's literal nibble 15, length L >= 15
        // and the run ending exactly at iend, every check the reference makes
        // on the way passes (the length bytes end at iend - L <= iend - 15, the
        // read limit) and the result is L; anything else takes the decoder.
        // Wave 0 finds the length run 64 bytes per ballot; every thread then
        // copies the literal from LDS to the output and the caller's buffer.
        if (threadIdx.x < kWave) {
            const int32_t iend = src_len[0], oend = dst_cap[0];
            int32_t q = -1, L = 15;
            if (iend >= 17 && oend >= 15 && (sblk[0] >> 4) == 15) {
                for (int32_t base = 1; base < iend; base += kWave) {
                    const int32_t p = base + (int32_t)lane;
                    const uint32_t bt = p < iend ? (uint32_t)sblk[p] : 0u;
                    const uint64_t stop = __ballot(bt != 255u);
                    if (stop == 0) {
                        L += 255 * kWave;
                        continue;
                    }
                    const int f = __builtin_ctzll(stop);
                    L += 255 * f + __builtin_amdgcn_readlane((int)bt, f);
                    q = base + f + 1;
                    break;
                }
            }
            if (lane == 0) solo_lit = (q > 0 && q + L == iend && L <= oend) ? L : -1, solo_lip = q;
        }
        __syncthreads();
        if (solo_lit >= 0) {
            const int32_t L = solo_lit;
            const lds_u8* lit = (const lds_u8*)sblk + solo_lip;
            uint8_t* d0 = dst + dst_off[0];
            for (int32_t p = 16 * (int32_t)threadIdx.x; p < L; p += 16 * 256) {
                const u32x4 v = lds_ld16a(lit + p);
                if (p + 16 <= L) {
                    st16(d0 + p, v);
                    if (solo_out != nullptr) st16(solo_out + p, v);
                } else {
                    put_exact(d0 + p, v, (uint32_t)(L - p));
                    if (solo_out != nullptr) put_exact(solo_out + p, v, (uint32_t)(L - p));
                }
            }
            if (threadIdx.x == 0) {
                status[0] = L;
                solo_r = L;
            }
        }
    }
    for (int64_t b = (int64_t)blockIdx.x * 4 + wv; b < n && !(SOLO && solo_lit >= 0); b += (int64_t)gridDim.x * 4) {
        const uint8_t* s = SOLO ? solo_src : src + src_off[b];
        uint8_t* d = dst + dst_off[b];
        const int32_t iend = src_len[b], oend = dst_cap[b];
        if (oend < 0 || iend <= 0 || oend == 0) {   // lz4.c:1950, :1978-1983
            const int32_t r0 = (oend == 0 && iend == 1 && s[0] == 0) ? 0 : -1;
            if (lane == 0) status[b] = r0;
            if (SOLO && lane == 0) solo_r = r0;
            continue;
        }
        const bool fast = oend >= 64;
        const int32_t dlen = DICT ? dict_len[b] : 0;
        int32_t ip = 0, op = 0, base = 0, F = 0, ib = -kCoopIn;
        bool fit_cut = false;   // the last round stopped at a sequence that only did not fit the buffer
        while (fast) {
            if (op - base > kHistRebase || (fit_cut && op - base > kHistKeep)) {   // keep the last kHistKeep bytes
                const int32_t nb = (op - kHistKeep) & ~15;
                // the move distance (> 2 KiB) exceeds the 1 KiB a wave moves per pass
                for (int32_t c = 16 * (int32_t)lane; c < op - nb; c += 16 * kWave) {
                    const u32x4 v = lds_ld16(OB + (nb - base) + c);
                    lds_wait();
                    lds_st16(OB + c, v);
                }
                base = nb;
            }
            // the 1 KiB input window serves several rounds (~3.5 input bytes per
            // sequence): restage only when fewer than kHistRestage bytes remain
            if (ip - ib > kCoopIn - kHistRestage) {
                ib = ip & ~15;
                const int32_t x = ib + 16 * (int32_t)lane;
                const u32x4 v = x + 16 <= iend ? ld16(s + x) : ld16_guarded(s + x, iend - x);
                lds_st16(IN + 16 * lane, v);
                __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
            }
            // speculative parse + walk: lane k gets the k-th sequence start
            int32_t myseq = 0;
            int nseq = 0;
            int32_t pos = ip - ib;
            // The chain of starts by pointer jumping instead of a serial readlane
            // walk.  Each lane parses two positions (pos + lane, pos + 64 + lane);
            // J[p] = the 2^t-th successor of position p at step t (>= 128: left the
            // parsed positions; kNoSeq: after a non-simple sequence).  Lane nseq + k
            // applies bit t of k with J at step t while J is doubled for step t + 1,
            // so the chain costs six dependent gathers.
            while (nseq < 64 && pos + 144 <= kCoopIn) {
                const int32_t ta = pos + (int32_t)lane, tb = ta + 64;
                const CoopSeq qa = coop_parse(IN, ta, HLD(IN + ta));
                const CoopSeq qb = coop_parse(IN, tb, HLD(IN + tb));
                const uint64_t sa = __ballot(qa.simple), sb = __ballot(qb.simple);
                constexpr int32_t kNoSeq = 1023;
                int32_t ja = qa.simple ? (int32_t)lane + qa.adv : kNoSeq;
                int32_t jb = qb.simple ? (int32_t)lane + 64 + qb.adv : kNoSeq;
                const int32_t kk = (int32_t)lane - nseq;
                int32_t c = kk >= 0 ? 0 : kNoSeq;
#pragma unroll
                for (int t = 0; t < 6; ++t) {
                    const int32_t ca = __builtin_amdgcn_ds_bpermute((c & 63) << 2, ja);
                    const int32_t cb = __builtin_amdgcn_ds_bpermute((c & 63) << 2, jb);
                    if (t < 5) {
                        const int32_t aa = __builtin_amdgcn_ds_bpermute((ja & 63) << 2, ja);
                        const int32_t ab = __builtin_amdgcn_ds_bpermute((ja & 63) << 2, jb);
                        const int32_t ba = __builtin_amdgcn_ds_bpermute((jb & 63) << 2, ja);
                        const int32_t bb = __builtin_amdgcn_ds_bpermute((jb & 63) << 2, jb);
                        if (((kk >> t) & 1) && c < 128) c = c < 64 ? ca : cb;
                        ja = ja < 128 ? (ja < 64 ? aa : ab) : ja;
                        jb = jb < 128 ? (jb < 64 ? ba : bb) : jb;
                    } else if (((kk >> t) & 1) && c < 128) {
                        c = c < 64 ? ca : cb;
                    }
                }
                const bool valid = c < 128 && (((c < 64 ? sa : sb) >> (c & 63)) & 1ull);
                if (valid) myseq = pos + c;
                const int nn = nseq + (int)__builtin_popcountll(__ballot(valid));
                if (nn >= 64) {
                    nseq = 64;
                    break;
                }
                const int32_t cv = __builtin_amdgcn_readlane(c, nn);   // the first start not taken
                nseq = nn;
                if (cv < 128) break;   // a non-simple sequence
                pos += cv;
            }
            if (nseq == 0) {
                // one sequence with literal > 12 bytes (or a long length), whole wave, on HBM
                const uint32_t tok = s[ip];
                int32_t lit = (int32_t)(tok >> 4), ml = (int32_t)(tok & 15u), q = ip + 1;
                if (lit == 15) {
                    if (q >= iend - 48 || !run_len32(s, q, iend - 48, iend, lit)) break;
                    if (q + lit > iend - 32 || op + lit > oend - 32) break;   // lz4.c:2016-2027
                } else if (q > iend - 17) {
                    break;   // lz4.c:2034
                }
                const int32_t opm = op + lit;
                const int32_t off = (int32_t)s[q + lit] | ((int32_t)s[q + lit + 1] << 8);
                int32_t qe = q + lit + 2;
                if (ml == 15) {
                    if (qe >= iend - 5 || !run_len32(s, qe, iend - 5, iend, ml)) break;
                    if (qe > iend - 5) break;
                }
                ml += 4;
                if (off < 1 || off > opm || opm + ml >= oend - 64) break;
                for (int32_t c = F + 16 * (int32_t)lane; c < op; c += 16 * kWave)
                    coop_put(d + c, lds_ld16(OB + (c - base)), op - c);
                __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
                coop_copy_literal<SOLO>(d + op, s + q, lit, lane);
                __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
                coop_copy_match(d + opm, off, ml, lane);
                __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
                op = opm + ml;
                ip = qe;
                // reload the history (op < oend - 64, so the 16-byte reads stay in dst)
                base = (op > kHistKeep ? op - kHistKeep : 0) & ~15;
                for (int32_t c = base + 16 * (int32_t)lane; c < op; c += 16 * kWave)
                    lds_st16(OB + (c - base), ld16(d + c));
                F = op;
                continue;
            }
            // sequence k in lane k
            const bool act = (int)lane < nseq;
            const int32_t tk = act ? myseq : 0;
            const u32x4 w = HLD(IN + tk);
            const CoopSeq q = coop_parse(IN, tk, w);
            const int32_t lit = q.lit, off = q.off, ml = q.ml, adv = q.adv;
            const int32_t len = act ? lit + ml : 0;
            const int32_t o = op + coop_incl_sum(len) - len;
            const int32_t sabs = ib + myseq;
            // the reference's fast-loop margins (lz4.c:2004-2110, as fast_seq / decode_step)
            const bool lit_ok = q.litx ? ib + q.litpos + lit <= iend - 32 && o + lit <= oend - 32
                                       : sabs + 1 <= iend - 17;
            // DICT: a source entirely in the dictionary
            const bool in_dict = DICT && off > o + lit && off <= o + lit + dlen && off >= 16 && o + lit - off + ml <= 0;
            const bool ok_nofit = act && q.simple && lit_ok && (!q.mlx || sabs + adv <= iend - 4) && off >= 1 &&
                                  (off <= o + lit || in_dict) && o + len < oend - 64;
            const bool ok = ok_nofit && o + len <= base + kHistW;
            const uint64_t bad = __ballot(act) & ~__ballot(ok);
            const int use = bad ? __builtin_ctzll(bad) : nseq;
            // a round cut only because the buffer is full goes on after a rebase;
            // margins and errors go to the exact path
            const bool fit_only = bad && ((__ballot(ok_nofit) >> use) & 1ull);
            if (use == 0 && !(fit_only && !fit_cut && op - base > kHistKeep)) break;
            fit_cut = fit_only;
            if (use == 0) continue;
            const bool u = (int)lane < use;
            const int32_t m = o + lit;
            // sources older than the buffer: their first 16 bytes are requested now,
            // so the HBM round trip overlaps the literal phase
            const bool far = u && m - off < base;
            u32x4 pre = u32x4{0, 0, 0, 0};
            if (far) pre = ld16(d + (m - off) + (DICT && m - off < 0 ? ddelta : 0));
            if (u && lit > 0) {
                if (lit <= 12) {
                    HPUT(OB + (o - base), window_shift1(w), lit);
                } else {
                    for (int32_t i = 0; i < lit; i += 16)
                        HPUT(OB + (o - base + i), HLD(IN + q.litpos + i), lit - i);
                }
            }
            lds_wait();
            const int32_t src_end = m - off + (off < ml ? off : ml);
            // A match is ready when no pending match writes into its source: its
            // source ends before the first pending match, or the nearest pending
            // match below it (pending destinations are disjoint and ordered) ends
            // before its source starts.
            const int32_t mend = m + ml;
            uint64_t pend = __ballot(u);
            while (pend) {
                const int32_t E = __builtin_amdgcn_readlane(m, __builtin_ctzll(pend));
                const bool mine = (pend >> lane) & 1ull;
                // end of the nearest pending match below: exclusive max-scan (DPP)
                int32_t x = __builtin_amdgcn_update_dpp(-1, mine ? mend : -1, 0x138, 0xF, 0xF, false);   // wave_shr:1
                x = max(x, __builtin_amdgcn_update_dpp(-1, x, 0x111, 0xF, 0xF, false));   // row_shr:1
                x = max(x, __builtin_amdgcn_update_dpp(-1, x, 0x112, 0xF, 0xF, false));   // row_shr:2
                x = max(x, __builtin_amdgcn_update_dpp(-1, x, 0x114, 0xF, 0xF, false));   // row_shr:4
                x = max(x, __builtin_amdgcn_update_dpp(-1, x, 0x118, 0xF, 0xF, false));   // row_shr:8
                x = max(x, __builtin_amdgcn_update_dpp(-1, x, 0x142, 0xA, 0xF, false));   // row_bcast:15
                x = max(x, __builtin_amdgcn_update_dpp(-1, x, 0x143, 0xC, 0xF, false));   // row_bcast:31
                const bool ready = mine && (src_end <= E || x <= m - off);
                if (ready) {
                    const int32_t s0 = m - off;
                    if (off >= 16) {
                        for (int32_t i = 0; i < ml; i += 16) {
                            const int32_t sp = s0 + i;   // < base: flushed long ago (base <= F - 4 K)
                            const u32x4 v = (i == 0 && far)   ? pre
                                            : sp >= base          ? HLD(OB + (sp - base))
                                                                  : ld16(d + sp + (DICT && sp < 0 ? ddelta : 0));
                            HPUT(OB + (m - base + i), v, ml - i);
                        }
                    } else {   // s0 > m - 16 >= base
                        const u32x4 pat = period_pattern(HLD(OB + (s0 - base)), (uint32_t)off);
                        const int32_t step = 16 - (16 % off);
                        for (int32_t i = 0; i < ml; i += step) HPUT(OB + (m - base + i), pat, ml - i);
                    }
                }
                lds_wait();
                pend &= ~__ballot(ready);
            }
            op = __builtin_amdgcn_readlane(o + len, use - 1);
            ip = ib + __builtin_amdgcn_readlane(myseq + adv, use - 1);
            // finished 16-byte chunks to HBM
            for (int32_t c = F + 16 * (int32_t)lane; c + 16 <= op; c += 16 * kWave)
                st16(d + c, lds_ld16(OB + (c - base)));
            F += (op - F) & ~15;
            if (use < nseq && !fit_only) break;
        }
        // flush the rest exactly, then the exact state machine from (ip, op)
        if (SOLO) LZ4M_WTS(ts, 4);
        for (int32_t c = F + 16 * (int32_t)lane; c < op; c += 16 * kWave)
            coop_put(d + c, lds_ld16(OB + (c - base)), op - c);
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
        if (SOLO) LZ4M_WTS(ts, 5);
        const int32_t r = coop_finish<DICT, SOLO>(s, d, iend, oend, ip, op, fast, lane, dlen, d + ddelta);
        if (SOLO) LZ4M_WTS(ts, 6);
        if (lane == 0) status[b] = r;
        if (SOLO && lane == 0) solo_r = r;
    }
    if constexpr (SOLO) {
        // the decoded bytes to the caller's mapped host buffer, all four waves
        // (wave 0 decoded; the others skipped the loop), so the call needs no
        // device-to-host copy of its own
        __syncthreads();
        LZ4M_WTS(ts, 2);
        const int32_t r = solo_r;
        if (solo_out != nullptr && r > 0 && solo_lit < 0) {   // (the stored-like path wrote solo_out itself)
            // through LDS (the staged input is no longer needed): every wave
            // first loads a chunk of the output into LDS, then stores it from
            // LDS, so no load waits behind the stores to host memory in flight
            // (a wave's memory counter retires in order)
            const uint8_t* d0 = dst + dst_off[0];
            constexpr int32_t kStep = 16 * 256, kChunk = 16 * kStep;   // 64 KiB <= kSoloIn
            lds_u8* bounce = (lds_u8*)const_cast<uint8_t*>(solo_src);   // the staging buffer (kSoloIn)
            for (int32_t c0 = 0; c0 < r; c0 += kChunk) {
                const int32_t m = r - c0 < kChunk ? r - c0 : kChunk;
                for (int32_t base0 = 0; base0 < m; base0 += kSoloU * kStep) {
                    u32x4 v[kSoloU];
#pragma unroll
                    for (int u = 0; u < kSoloU; ++u) {
                        const int32_t p = base0 + u * kStep + 16 * (int32_t)threadIdx.x;
                        v[u] = p + 16 <= m ? ld16(d0 + c0 + p) : ld16_guarded(d0 + c0 + p, m - p);
                    }
#pragma unroll
                    for (int u = 0; u < kSoloU; ++u) {
                        const int32_t p = base0 + u * kStep + 16 * (int32_t)threadIdx.x;
                        if (p < m) lds_st16(bounce + p, v[u]);
                    }
                }
                __syncthreads();
                for (int32_t p = 16 * (int32_t)threadIdx.x; p < m; p += kStep) {
                    const u32x4 v = lds_ld16(bounce + p);
                    if (p + 16 <= m) {
                        st16(solo_out + c0 + p, v);
                    } else {
                        put_exact(solo_out + c0 + p, v, (uint32_t)(m - p));
                    }
                }
                __syncthreads();
            }
        }
        if (solo_done != nullptr) {   // all of the above visible to the host, then the flag it polls
            // every storing thread releases its own solo_out stores at system
            // scope before the barrier, then one thread stores the flag
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
            __syncthreads();
            LZ4M_WTS(ts, 3);
            if (threadIdx.x == 0) __hip_atomic_store(solo_done, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
#undef HPUT
#undef HLD
}

// (the body is shared with the single-call worker, lz4m_worker.hip)
template <bool DICT, bool SOLO = false>
__global__ __launch_bounds__(256, 4) void hist_decompress_kernel(const uint8_t* __restrict__ src,
                                                                 const int64_t* __restrict__ src_off,
                                                                 const int32_t* __restrict__ src_len, uint8_t* dst,
                                                                 const int64_t* __restrict__ dst_off,
                                                                 const int32_t* __restrict__ dst_cap,
                                                                 int32_t* __restrict__ status, int64_t n,
                                                                 const int32_t* __restrict__ dict_len, int64_t ddelta,
                                                                 uint8_t* solo_out, int32_t* solo_done) {
    hist_decompress_body<DICT, SOLO>(src, src_off, src_len, dst, dst_off, dst_cap, status, n, dict_len, ddelta,
                                     solo_out, solo_done);
}

// The single-call decompress worker: one persistent workgroup that serves
// the lone-block requests of one host thread from its mailbox with the
// SOLO body above (input and record read from mapped pinned memory, output
// written back into it, done flag released), until told to quit or idle.
__global__ __launch_bounds__(256) void decompress_worker(Mailbox* mb, uint8_t* hd, uint8_t* dbuf, uint64_t idle,
                                                        uint64_t life) {
    __shared__ uint32_t cmd[8];
    __shared__ int64_t zero_off;   // the record's offsets and sizes, read by the body from LDS, not over PCIe
    uint64_t birth = 0;
    uint32_t last = worker_init(mb, cmd, birth);
    if (threadIdx.x == 0) zero_off = 0;
    for (;;) {
        if (worker_next(mb, last, idle, birth, life, cmd) == 0) break;
        const int32_t rec_off = (int32_t)cmd[1];
        CallMeta* rec = reinterpret_cast<CallMeta*>(hd + rec_off);
        const int32_t* len_cap = reinterpret_cast<const int32_t*>(cmd + 2);   // cmd[2] = src_len, cmd[3] = dst_cap
        hist_decompress_body<false, true>(hd, &zero_off, len_cap, dbuf, &zero_off, len_cap + 1, &rec->result,
                                          (int64_t)1, nullptr, (int64_t)0, hd + rec_off + kCallMeta, &rec->done);
    }
}

// Linked-block frames (lz4frame.c:1853-1856, LZ4F_updateDict): block i may
// reference the output of blocks < i, so the chain decodes in order on one
// wavefront, contiguously into dst.  Lane 0 parses; the wave runs the long
// copies.  Prefix semantics = LZ4_decompress_safe_usingDict with the
// previous output as a contiguous prefix (withSmallPrefix / withPrefix64k,
// lz4.c:2612-2625): offsets may reach min(prefix, 64 KiB) before the block.
__global__ __launch_bounds__(64) void decompress_chain_kernel(const uint8_t* __restrict__ src,
                                                              const int64_t* __restrict__ src_off,
                                                              const int32_t* __restrict__ src_len,
                                                              const uint8_t* __restrict__ raw_flag, uint8_t* dst,
                                                              int32_t* __restrict__ status, int64_t n,
                                                              int32_t max_block) {
    const uint32_t lane = threadIdx.x;
    int64_t running = 0;
    for (int64_t b = 0; b < n; ++b) {
        const int64_t len = src_len[b];
        const uint8_t* s = src + src_off[b];
        uint8_t* d = dst + running;
        if (raw_flag[b]) {
            wave_literal(d, s, len, len, len, lane);
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
            if (lane == 0) status[b] = (int32_t)len;
            running += len;
            continue;
        }
        Lane L;
        L.live = false;
        L.result = -1;
        if (lane == 0) {
            L.src = s;
            L.dst = d;
            L.iend = len;
            L.oend = max_block;
            L.ip = 0;
            L.op = 0;
            L.dict_len = running < 65536 ? running : 65536;
            L.dict_end = d;
            if (L.iend <= 0) {
                L.result = -1;
            } else {
                L.fast = L.oend >= 64;
                L.live = true;
            }
        }
        while (__any(L.live)) {
            Copy lc{kNone, 0, 0, 0}, mc{kNone, 0, 0, 0};
            if (L.live) decode_step<true>(L, lc, mc);
            const uint64_t pend = __ballot(lc.kind != kNone || mc.kind != kNone);
            if (pend == 0) continue;
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
            uint8_t* dd = readlane_ptr(L.dst, 0);
            const int64_t oend = readlane64(L.oend, 0);
            if (__builtin_amdgcn_readlane(lc.kind, 0) != kNone) {
                const uint8_t* ss = readlane_ptr(L.src, 0);
                const int64_t iend = readlane64(L.iend, 0);
                const int64_t dp = readlane64(lc.dpos, 0), sp = readlane64(lc.arg, 0), ln = readlane64(lc.len, 0);
                wave_literal(dd + dp, ss + sp, ln, oend - dp, iend - sp, lane);
                __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
            }
            if (__builtin_amdgcn_readlane(mc.kind, 0) != kNone) {
                const int64_t dp = readlane64(mc.dpos, 0), off = readlane64(mc.arg, 0), ln = readlane64(mc.len, 0);
                if (off < 0) {
                    if (lane == 0) dict_match(L, dp, -off, ln);
                } else {
                    wave_match(dd + dp, off, ln, oend - dp, lane);
                }
                __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
            }
        }
        const int32_t r = __builtin_amdgcn_readlane(L.result, 0);
        if (lane == 0) status[b] = r;
        if (r < 0) {
            for (int64_t k = b + 1 + lane; k < n; k += kWave) status[k] = -1;
            return;
        }
        running += r;
    }
}

}  // namespace lz4m

using namespace lz4m;

namespace {

int current_device() {
    int dev = 0;
    (void)hipGetDevice(&dev);
    return dev >= 0 && dev < 64 ? dev : 0;
}

int env_int(const char* name, int dflt) {
    const char* e = getenv(name);
    const int v = e != nullptr ? atoi(e) : 0;
    return v > 0 ? v : dflt;
}

// the values are the C-ABI's decoder ids (include/lz4m.h); 1, 2, 5 and 6
// were retired decoders and are rejected
enum Decoder { kAuto = 0, kHistDec = 3, kRowsDec = 4 };   // 7 was the block-resident experiment (removed round 5)

// LZ4M_DECODER forces a decoder (A/B measurements, tests): hist | rows;
// unset = by batch size and scratch.
int decoder_env() {
    static const int mode = [] {
        const char* e = getenv("LZ4M_DECODER");
        if (e == nullptr) return (int)kAuto;
        if (strcmp(e, "hist") == 0) return (int)kHistDec;
        if (strcmp(e, "rows") == 0) return (int)kRowsDec;
        return (int)kAuto;
    }();
    return mode;
}

}  // namespace

extern "C" size_t lz4m_decompress_workspace_bytes(void) { return 64; }

extern "C" size_t lz4m_decompress_workspace_size(int64_t n, int64_t src_bytes) {
    if (n <= 0) return 64;
    const size_t lens = (size_t)(src_bytes > 0 ? src_bytes : 0) / 3 + 17 * (size_t)n + 64;   // + 16 per block: 16-aligned lengths
    return (lz4m_rows_fixed_bytes(n) + lens + 255) & ~(size_t)255;
}

extern "C" int lz4m_decompress_batch_sel(const uint8_t* d_src, const int64_t* d_src_off, const int32_t* d_src_len,
                                         uint8_t* d_dst, const int64_t* d_dst_off, const int32_t* d_dst_cap,
                                         int32_t* d_status, int64_t n, void* d_work, size_t work_bytes, int decoder,
                                         lz4m_stream_t stream) {
    if (n < 0 || !(decoder == kAuto || decoder == kHistDec || decoder == kRowsDec))
        return LZ4M_EINVAL;
    if (n == 0) return 0;
    hipStream_t st = (hipStream_t)stream;
    if (decoder == kAuto) decoder = decoder_env();
    if (d_work == nullptr || work_bytes < lz4m_decompress_workspace_bytes() || ((uintptr_t)d_work & 7) != 0)
        return LZ4M_EINVAL;
    // the large-batch decoder needs scratch for its per-block records and
    // sequence lengths (lz4m_decompress_workspace_size); without it (or for
    // small batches) the one-wavefront-per-block decoder takes any batch
    const bool rows_fit = work_bytes >= lz4m_rows_fixed_bytes(n) + 64;
    // LZ4M_ROWS_MIN_BLOCKS: smallest batch sent to the row decoder (tuning)
    static const int rows_min = env_int("LZ4M_ROWS_MIN_BLOCKS", 32768);   // crossover measured, DESIGN 3.1
    if (decoder == kAuto) decoder = rows_fit && n >= rows_min ? kRowsDec : kHistDec;
    if (decoder != kHistDec && !rows_fit) decoder = kHistDec;
    if (decoder == kRowsDec) {
        int pg = 1, eg = 1;
        lz4m_rows_grids(n, &pg, &eg);
        const int rc = lz4m_rows_launch(d_src, d_src_off, d_src_len, d_dst, d_dst_off, d_dst_cap, n, d_work, work_bytes,
                                        pg, eg, st);
        if (rc != 0) return rc;
        const RowMeta* meta = reinterpret_cast<const RowMeta*>(static_cast<const uint8_t*>(d_work) + kRowsMeta);
        const int64_t grid = (n + 255) / 256;
        hipLaunchKernelGGL((decompress_kernel<false, true>), dim3((uint32_t)grid), dim3(256), 0, st, d_src, d_src_off,
                           d_src_len, d_dst, d_dst_off, d_dst_cap, nullptr, nullptr, nullptr, d_status, n, meta);
        return (int)hipGetLastError();
    }
    const int64_t grid = (n + 3) / 4;
    hipLaunchKernelGGL(hist_decompress_kernel<false>, dim3((uint32_t)(grid < 65536 ? grid : 65536)), dim3(256), 0, st,
                       d_src, d_src_off, d_src_len, d_dst, d_dst_off, d_dst_cap, d_status, n, nullptr, (int64_t)0, nullptr, nullptr);
    return (int)hipGetLastError();
}

extern "C" int lz4m_decompress_solo(const uint8_t* d_src, const int64_t* d_src_off, const int32_t* d_src_len,
                                    uint8_t* d_dst, const int64_t* d_dst_off, const int32_t* d_dst_cap,
                                    int32_t* d_status, int32_t src_len_host, uint8_t* h_out, int32_t* h_done,
                                    lz4m_stream_t stream) {
    if (src_len_host < 0 || src_len_host > kSoloIn - 64) return LZ4M_EINVAL;
    hipLaunchKernelGGL((hist_decompress_kernel<false, true>), dim3(1), dim3(256), 0, (hipStream_t)stream, d_src,
                       d_src_off, d_src_len, d_dst, d_dst_off, d_dst_cap, d_status, (int64_t)1, nullptr, (int64_t)0, h_out, h_done);
    return (int)hipGetLastError();
}

extern "C" int lz4m_worker_launch(int kind, Mailbox* mb, uint8_t* hd, uint8_t* dbuf, uint64_t idle_ticks,
                                  uint64_t life_ticks, hipStream_t stream) {
    if (kind == 1) return lz4m_compress_worker_launch(mb, hd, dbuf, idle_ticks, life_ticks, stream);
    if (kind != 0) return LZ4M_EINVAL;
    hipLaunchKernelGGL(decompress_worker, dim3(1), dim3(256), 0, stream, mb, hd, dbuf, idle_ticks, life_ticks);
    return (int)hipGetLastError();
}

extern "C" int lz4m_decompress_batch_ws(const uint8_t* d_src, const int64_t* d_src_off, const int32_t* d_src_len,
                                        uint8_t* d_dst, const int64_t* d_dst_off, const int32_t* d_dst_cap,
                                        int32_t* d_status, int64_t n, void* d_work, size_t work_bytes,
                                        lz4m_stream_t stream) {
    return lz4m_decompress_batch_sel(d_src, d_src_off, d_src_len, d_dst, d_dst_off, d_dst_cap, d_status, n, d_work,
                                     work_bytes, kAuto, stream);
}

extern "C" int lz4m_decompress_batch(const uint8_t* d_src, const int64_t* d_src_off, const int32_t* d_src_len,
                                     uint8_t* d_dst, const int64_t* d_dst_off, const int32_t* d_dst_cap,
                                     int32_t* d_status, int64_t n, lz4m_stream_t stream) {
    if (n < 0) return LZ4M_EINVAL;
    if (n == 0) return 0;
    // no scratch: the one-wavefront-per-block decoder (any batch size)
    const int64_t grid = (n + 3) / 4;
    hipLaunchKernelGGL(hist_decompress_kernel<false>, dim3((uint32_t)(grid < 65536 ? grid : 65536)), dim3(256), 0,
                       (hipStream_t)stream, d_src, d_src_off, d_src_len, d_dst, d_dst_off, d_dst_cap, d_status, n,
                       nullptr, (int64_t)0, nullptr, nullptr);
    return (int)hipGetLastError();
}

extern "C" int lz4m_decompress_batch_dict(const uint8_t* d_src, const int64_t* d_src_off, const int32_t* d_src_len,
                                          uint8_t* d_dst, const int64_t* d_dst_off, const int32_t* d_dst_cap,
                                          const uint8_t* d_dict, const int64_t* d_dict_off,
                                          const int32_t* d_dict_len, int32_t* d_status, int64_t n,
                                          lz4m_stream_t stream) {
    if (n < 0) return LZ4M_EINVAL;
    if (n == 0) return 0;
    const int64_t grid = (n + 255) / 256;
    hipLaunchKernelGGL(decompress_kernel<true>, dim3((uint32_t)grid), dim3(256), 0, (hipStream_t)stream, d_src,
                       d_src_off, d_src_len, d_dst, d_dst_off, d_dst_cap, d_dict, d_dict_off, d_dict_len, d_status,
                       n, nullptr);
    return (int)hipGetLastError();
}

extern "C" int lz4m_decompress_batch_prefix(const uint8_t* d_src, const int64_t* d_src_off, const int32_t* d_src_len,
                                            uint8_t* d_dst, const int64_t* d_dst_off, const int32_t* d_dst_cap,
                                            const uint8_t* d_dict_base, const int32_t* d_dict_len,
                                            int32_t* d_status, int64_t n, lz4m_stream_t stream) {
    if (n < 0 || (n > 0 && d_dict_base == nullptr)) return LZ4M_EINVAL;
    if (n == 0) return 0;
    const int64_t grid = (n + 3) / 4;
    const int64_t delta = (int64_t)((intptr_t)d_dict_base - (intptr_t)d_dst);
    hipLaunchKernelGGL(hist_decompress_kernel<true>, dim3((uint32_t)(grid < 65536 ? grid : 65536)), dim3(256), 0,
                       (hipStream_t)stream, d_src, d_src_off, d_src_len, d_dst, d_dst_off, d_dst_cap, d_status, n,
                       d_dict_len, delta, nullptr, nullptr);
    return (int)hipGetLastError();
}

extern "C" int lz4m_decompress_chain(const uint8_t* d_src, const int64_t* d_src_off, const int32_t* d_src_len,
                                     const uint8_t* d_raw_flag, uint8_t* d_dst, int32_t* d_status, int64_t n,
                                     int32_t max_block, lz4m_stream_t stream) {
    if (n < 0 || max_block < 0) return LZ4M_EINVAL;
    if (n == 0) return 0;
    hipLaunchKernelGGL(decompress_chain_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, d_src, d_src_off,
                       d_src_len, d_raw_flag, d_dst, d_status, n, max_block);
    return (int)hipGetLastError();
}

