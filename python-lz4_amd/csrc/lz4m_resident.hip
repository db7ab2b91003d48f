// lz4m_resident.hip -- the block-resident executor of the large-batch decoder.
//
// Reference: LZ4_decompress_safe (lz4libs/lz4.c:2344-2350) ->
// LZ4_decompress_generic (:1936-2339), fast loop :1996-2109.  Bit-exact in
// three stream-ordered kernels; the first and the last are the row decoder's
// (lz4m_rows.hip, lz4m_decompress.hip):
//  1. rows_parse_kernel: one lane per block walks the token chain and
//     records every "good" sequence's compressed length (one byte, 255 =
//     re-parse it) -- a sequence the reference provably decodes inside its
//     fast loop without error -- and the state at the first one that is not;
//  2. res_exec_kernel (this file) places and copies the good sequences;
//  3. the finisher (decompress_kernel<false, true>) runs the reference's
//     exact state machine from there: the tail, every error and its position.
//
// Why resident.  The row executor keeps 1 KiB of each block's recent output
// on chip and reads every older match source back from HBM -- half of all
// matches on the silesia-like mix, 16-byte sources that each fetch a 128-byte
// line: 7.6x the algorithmic bytes per launch (round 3).  Here one 256-thread
// workgroup owns one block at a time and keeps the block's whole output
// (<= 64 KiB) in LDS, two blocks per CU: every match source is an LDS read
// and the output leaves for HBM once, coalesced, when the block is done.
//
// Work split.  The block's good sequences are cut into chunks of 64, one
// sequence per lane; wave w takes chunks w, w + 4, w + 8, ...  Two running
// positions chain the chunks in order through LDS handoff slots: the input
// position (a wave prefix sum of the recorded lengths, run two chunks ahead
// of execution so each lane's 32 input bytes are requested early) and the
// output position (a prefix sum of literal + match lengths once a chunk is
// parsed).  Dependencies between matches need no passes and no scans: a
// bitmap holds one bit per output byte, set after the byte is written (in
// the writing wave's LDS order), and a lane copies its match once every bit
// of its source is set.  The four waves thus run four consecutive chunks at
// once and a match waits exactly for the bytes it reads.  Copies longer than
// kResLong bytes run on the whole wave, up to 1 KiB per step.
//
// Blocks whose good prefix would reach past the LDS output (capacities above
// 64 KiB) are cut at the first sequence ending beyond kResLim: the record's
// resume point moves there and the finisher decodes the rest.
#include "lz4m_common.h"
#include "lz4m_rows.h"

namespace lz4m {

#ifndef LZ4M_RES_W
#define LZ4M_RES_W 4
#endif
constexpr int kResW = LZ4M_RES_W;             // waves per workgroup (one block)
constexpr int kResT = 64 * kResW;             // threads per workgroup
constexpr int32_t kResOut = 65536;            // output bytes held in LDS
constexpr int32_t kResLim = kResOut - 64;     // placed sequences end at or below this
constexpr int kResBitW = kResOut / 32 + 4;    // written-byte bitmap (dwords; word k + 1 of any read stays inside)
constexpr uint32_t kResStop = 0x7FFFFFFFu;    // output position handed on after a cut
#ifndef LZ4M_RES_LONG
#define LZ4M_RES_LONG 64
#endif
constexpr int32_t kResLong = LZ4M_RES_LONG;   // longer copies run on the whole wave

// LZ4M_RES_PROF (diagnostic builds only): per-phase wave-cycle sums and
// event counts, read with lz4m_res_prof
#ifdef LZ4M_RES_PROF
__device__ unsigned long long g_res_prof[16];
#define RS_DECL uint64_t rs[16] = {0}; uint64_t rs_t = clock64();
#define RS_MARK(i) do { const uint64_t _t = clock64(); rs[i] += _t - rs_t; rs_t = _t; } while (0)
#define RS_COUNT(i, x) rs[i] += (uint64_t)(x)
#define RS_FLUSH() do { if (lane == 0) for (int _i = 0; _i < 16; ++_i) atomicAdd(&g_res_prof[_i], (unsigned long long)rs[_i]); } while (0)
#else
#define RS_DECL
#define RS_MARK(i) do {} while (0)
#define RS_COUNT(i, x) do {} while (0)
#define RS_FLUSH() do {} while (0)
#endif

typedef __attribute__((address_space(3))) volatile uint32_t lds_vu32a;
typedef __attribute__((address_space(3))) volatile uint64_t lds_vu64a;

// 64-lane inclusive sum: DPP row shifts, then row broadcasts
__device__ __forceinline__ int32_t wave_incl_sum(int32_t v) {
    v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xF, 0xF, false);   // row_shr:1
    v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xF, 0xF, false);   // row_shr:2
    v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xF, 0xF, false);   // row_shr:4
    v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xF, 0xF, false);   // row_shr:8
    v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xA, 0xF, false);   // row_bcast:15
    v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xC, 0xF, false);   // row_bcast:31
    return v;
}

// Handoff slot: {tag, value} as one naturally aligned 8-byte LDS word
// (written by one lane with one ds_write_b64, so a reader sees both or
// neither).  Tag k + 1 carries chunk k's end position.
__device__ __forceinline__ void slot_put(lds_vu64a* s, uint32_t tag, uint32_t v) {
    *s = ((uint64_t)tag << 32) | (uint64_t)v;
}
// Spins are bounded (kResSpin polls, ~0.5 s): a protocol bug ends the
// kernel with wrong bytes, which the tests catch, instead of a hung GPU.
constexpr int32_t kResSpin = 1 << 23;
__device__ __forceinline__ uint32_t slot_wait(lds_vu64a* s, uint32_t tag, uint32_t dflt) {
    for (int32_t it = 0; it < kResSpin; ++it) {
        const uint64_t x = *s;
        if ((uint32_t)__builtin_amdgcn_readfirstlane((int32_t)(uint32_t)(x >> 32)) == tag)
            return (uint32_t)__builtin_amdgcn_readfirstlane((int32_t)(uint32_t)x);
        __builtin_amdgcn_s_sleep(1);
    }
    return dflt;
}

// ---------------------------------------------------- written-byte bitmap
// bits r .. r + L - 1 (1 <= L <= 32, 0 <= r <= 31) of a 64-bit pair
__device__ __forceinline__ uint64_t span_mask(int32_t r, int32_t L) { return (((uint64_t)1 << L) - 1) << r; }
// ds_or_b32 (no return): issued after the bytes' own writes, in this wave's
// LDS order, so a reader that sees the bit reads the bytes
#define LZ4M_DSOR(addr, x) asm volatile("ds_or_b32 %0, %1" ::"v"(addr), "v"(x) : "memory")
__device__ __forceinline__ void bits_set(lds_vu32a* B, int32_t p, int32_t L) {   // 1 <= L <= 32
    const uint64_t msk = span_mask(p & 31, L);
    const uint32_t a = lds_addr((const lds_u8*)(B + (p >> 5)));
    LZ4M_DSOR(a, (uint32_t)msk);
    if ((uint32_t)(msk >> 32) != 0u) LZ4M_DSOR(a + 4u, (uint32_t)(msk >> 32));
}
// [p, p + L), any L >= 0, by one lane: one OR per dword
__device__ __forceinline__ void bits_fill(lds_vu32a* B, int32_t p, int32_t L) {
    for (int32_t x = 0; x < L;) {
        const int32_t q = p + x;
        const int32_t k = min(32 - (q & 31), L - x);
        bits_set(B, q, k);
        x += k;
    }
}
// [p, p + L), any L >= 0, by the whole wave (uniform arguments)
__device__ __forceinline__ void bits_fill_wave(lds_vu32a* B, int32_t p, int32_t L, uint32_t lane) {
    if (L <= 0) return;
    const int32_t k0 = p >> 5, k1 = (p + L - 1) >> 5;
    for (int32_t k = k0 + (int32_t)lane; k <= k1; k += 64) {
        const int32_t lo = max(p, 32 * k) - 32 * k, hi = min(p + L, 32 * k + 32) - 32 * k;
        const uint32_t m = hi - lo >= 32 ? ~0u : ((1u << (hi - lo)) - 1u) << lo;
        LZ4M_DSOR(lds_addr((const lds_u8*)(B + k)), m);
    }
}

// ------------------------------------------------ one-round-trip LDS access
// A match attempt needs the written-byte bits of its source and the source
// bytes, read in that order (a reader that sees a bit must read the byte
// after it).  Both are issued back to back and waited for once: the bits of
// [p, p + 32) (two dwords) and the 40 bytes at p & ~7 (five aligned 8-byte
// reads: any 32-byte window at p).  The compiler knows nothing of these
// loads, hence the explicit wait inside the asm.
struct SrcRead {
    uint64_t bits, w0, w1, w2, w3, w4;
};
__device__ __forceinline__ void src_read(uint32_t baddr, uint32_t daddr, SrcRead& r) {
    // volatile: issued in program order (bits first); the empty asm after the
    // last one is a scheduling boundary, so nothing that waits for the bits
    // is placed between the loads
    typedef __attribute__((address_space(3))) volatile uint32_t vu32;
    const vu32* B = (const vu32*)(uintptr_t)baddr;
    const lds_vu64a* D = (const lds_vu64a*)(uintptr_t)daddr;
    const uint32_t b0 = B[0], b1 = B[1];
    r.w0 = D[0];
    r.w1 = D[1];
    r.w2 = D[2];
    r.w3 = D[3];
    r.w4 = D[4];
    asm volatile("" ::: "memory");
    r.bits = (uint64_t)b0 | ((uint64_t)b1 << 32);
}
// 16 bytes at byte q (0..7) of the 24-byte run x0|x1|x2
__device__ __forceinline__ u32x4 funnel16(uint64_t x0, uint64_t x1, uint64_t x2, uint32_t q) {
    const bool h = (q & 4u) != 0;
    const uint32_t r = q & 3u;
    const uint32_t c0 = (uint32_t)x0, c1 = (uint32_t)(x0 >> 32), c2 = (uint32_t)x1, c3 = (uint32_t)(x1 >> 32),
                   c4 = (uint32_t)x2, c5 = (uint32_t)(x2 >> 32);
    const uint32_t e0 = h ? c1 : c0, e1 = h ? c2 : c1, e2 = h ? c3 : c2, e3 = h ? c4 : c3, e4 = h ? c5 : c4;
    return u32x4{__builtin_amdgcn_alignbyte(e1, e0, r), __builtin_amdgcn_alignbyte(e2, e1, r),
                 __builtin_amdgcn_alignbyte(e3, e2, r), __builtin_amdgcn_alignbyte(e4, e3, r)};
}
// are the bits r .. r + L - 1 (1 <= L <= 32, 0 <= r <= 31) of w all set
__device__ __forceinline__ bool bits_in(uint64_t w, int32_t r, int32_t L) {
    const uint64_t msk = span_mask(r, L);
    return (w & msk) == msk;
}
// mask of the low n (0..4) bytes of a dword
__device__ __forceinline__ uint32_t low_bytes(int32_t n) { return n >= 4 ? ~0u : ((1u << (8 * n)) - 1u); }
// Exactly k (>= 1; >= 16: 16) bytes of v at LDS byte address a: five masked
// ORs on the enclosing aligned dwords (atomic per dword, so neighbouring
// sequences sharing a dword may write it at once), masks computed in
// registers (no table read: one LDS round trip less per put).
__device__ __forceinline__ void lds_put_ar(uint32_t a, u32x4 v, int32_t k) {
    const uint32_t r = a & 3u;
    const int32_t e = (int32_t)r + min(k, 16);
    const uint32_t s = (4u - r) & 3u;
    const bool z = r == 0;
    const uint32_t d0 = __builtin_amdgcn_alignbyte(v.x, z ? v.x : 0u, s);
    const uint32_t d1 = __builtin_amdgcn_alignbyte(v.y, z ? v.y : v.x, s);
    const uint32_t d2 = __builtin_amdgcn_alignbyte(v.z, z ? v.z : v.y, s);
    const uint32_t d3 = __builtin_amdgcn_alignbyte(v.w, z ? v.w : v.z, s);
    const uint32_t d4 = __builtin_amdgcn_alignbyte(0u, z ? 0u : v.w, s);
    const uint32_t m0 = low_bytes(min(e, 4)) & ~low_bytes((int32_t)r);
    const uint32_t m1 = low_bytes(min(max(e - 4, 0), 4)), m2 = low_bytes(min(max(e - 8, 0), 4));
    const uint32_t m3 = low_bytes(min(max(e - 12, 0), 4)), m4 = low_bytes(max(e - 16, 0));
    const uint32_t b4 = a & ~3u;
    LZ4M_MSKOR(b4, 0, m0, d0);
    LZ4M_MSKOR(b4, 4, m1, d1);
    LZ4M_MSKOR(b4, 8, m2, d2);
    LZ4M_MSKOR(b4, 12, m3, d3);
    LZ4M_MSKOR(b4, 16, m4, d4);
}

// ------------------------------------------------------------- sequences
// compressed length of the sequence at p (a good sequence: every byte read
// lies inside the block)
__device__ __forceinline__ int32_t seq_clen(const uint8_t* p, int32_t xl) {   // reads p[0 .. xl]
    const uint32_t tok = p[0];
    int32_t x = 1, lit = (int32_t)(tok >> 4);
    if (lit == 15) {
        uint32_t b;
        do {
            b = p[min(x, xl)];
            ++x;
            lit += (int32_t)b;
        } while (b == 255 && x <= xl);
    }
    x += lit + 2;
    if ((tok & 15u) == 15u) {
        uint32_t b;
        do {
            b = p[min(x, xl)];
            ++x;
        } while (b == 255 && x <= xl);
    }
    return x;
}

// 32 bytes of block input at t (a | b; b is clamped into the block, so its
// bytes are valid only when t + 32 <= iend; good sequences have t + 18 <= iend)
__device__ __forceinline__ void res_load_in(const uint8_t* s, int32_t t, int32_t iend, u32x4& a, u32x4& b) {
    const int32_t ta = t + 16 <= iend ? t : 0;
    const int32_t tb = t + 32 <= iend ? t + 16 : iend - 16;
    a = ld16(s + ta);
    b = ld16(s + tb);
}

// the 4 bytes at k (0..28) of the 32-byte window a|b
__device__ __forceinline__ uint32_t win32_dword(u32x4 a, u32x4 b, uint32_t k) {
    const uint32_t q = k >> 2;
    const uint32_t lo = q == 0 ? a.x : q == 1 ? a.y : q == 2 ? a.z : q == 3 ? a.w : q == 4 ? b.x : q == 5 ? b.y : q == 6 ? b.z : b.w;
    const uint32_t hi = q == 0 ? a.y : q == 1 ? a.z : q == 2 ? a.w : q == 3 ? b.x : q == 4 ? b.y : q == 5 ? b.z : q == 6 ? b.w : 0u;
    return __builtin_amdgcn_alignbyte(hi, lo, k & 3);
}

// One lane's sequence, parsed from its 32 input bytes (the row decoder's
// parse_round, lz4m_rows.hip) or, for the rare long forms, from HBM.
struct ResSeq {
    int32_t lit, off, ml, lp;   // lp: the literal's first byte relative to the token
    bool litg;                  // literal bytes beyond the 32 at hand (read from HBM)
};
__device__ __forceinline__ void res_parse(const uint8_t* s, int32_t t, int32_t iend, bool act, bool esc, u32x4 wa,
                                          u32x4 wb, ResSeq& q) {
    const bool wbok = t + 32 <= iend;
    const uint32_t tok = wa.x & 0xFFu;
    const int32_t lit0 = (int32_t)(tok >> 4);
    const bool litx = lit0 == 15;
    int32_t lit = lit0 + (litx ? (int32_t)byte_of(wa, 1) : 0);   // one extra byte unless escaped
    int32_t lp = litx ? 2 : 1;
    const int32_t po = lp + lit;
    const int32_t mlc = (int32_t)(tok & 15u);
    // offset and first match-length byte: from wa for lit <= 12 (po <= 13), else from wa|wb
    const uint32_t pq = (uint32_t)(po < 28 ? po : 28);
    const uint32_t dwo = lit <= 12 ? window_dword(wa, (uint32_t)po) : win32_dword(wa, wb, pq);
    const uint32_t dws = dwo >> min(8u * ((uint32_t)po - pq), 24u);
    int32_t off = (int32_t)(dws & 0xFFFFu);
    const int32_t e0 = (int32_t)((dws >> 16) & 0xFFu);
    int32_t ml = mlc + (mlc == 15 ? e0 : 0);
    const bool slow = esc | (po + 3 > 32) | ((mlc == 15) & (e0 == 255)) | ((po + 3 > 16) & !wbok);
    if (slow && act) {   // a long literal or match length, or the offset past the bytes at hand
        const uint8_t* p = s + t;
        const int32_t xl = iend - t - 1;   // reads stay inside the block
        int32_t x = 1;
        lit = lit0;
        if (lit == 15) {
            uint32_t b;
            do {
                b = p[min(x, xl)];
                ++x;
                lit += (int32_t)b;
            } while (b == 255 && x <= xl);
        }
        lp = x;
        x += lit;
        off = (int32_t)p[min(x, xl)] | ((int32_t)p[min(x + 1, xl)] << 8);
        x += 2;
        ml = mlc;
        if (ml == 15) {
            uint32_t b;
            do {
                b = p[min(x, xl)];
                ++x;
                ml += (int32_t)b;
            } while (b == 255 && x <= xl);
        }
    }
    q.lit = lit;
    q.off = off;
    q.ml = ml + 4;
    q.lp = lp;
    q.litg = (lp + lit > 16) & ((lp + lit > 32) | !wbok);
}

// exactly k (1..16) bytes of v at global address p
__device__ __forceinline__ void res_gput(uint8_t* p, u32x4 v, int32_t k) {
    if (k >= 16) {
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

// ------------------------------------------------------------ the kernel
__global__ __launch_bounds__(kResT, kResW / 2) void res_exec_kernel(const uint8_t* __restrict__ src,
                                                           const int64_t* __restrict__ src_off,
                                                           const int32_t* __restrict__ src_len, uint8_t* dst,
                                                           const int64_t* __restrict__ dst_off, RowMeta* meta,
                                                           const uint8_t* __restrict__ lens, int64_t n,
                                                           unsigned long long* __restrict__ ctr) {
    __shared__ __attribute__((aligned(16))) uint8_t outb[kResOut + 64];
    __shared__ __attribute__((aligned(16))) uint32_t bitw[kResBitW];
    __shared__ __attribute__((aligned(16))) uint64_t slots[8];   // 0-3: input positions, 4-7: output positions
    __shared__ int64_t nxt_s;                                     // the next block
    __shared__ int32_t opg_s;                                     // the block's good output end (after a cut)
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wv = tid >> 6;
    for (int k = (int)tid; k < kResBitW; k += kResT) bitw[k] = 0;
    if (tid < 8) slots[tid] = 0;
    if (tid == 0) nxt_s = (int64_t)atomicAdd(&ctr[2], 1ull);
    __syncthreads();
    lds_u8* OUT = (lds_u8*)outb;
    lds_vu32a* B = (lds_vu32a*)bitw;
    const uint32_t obase = lds_addr(OUT), bbase = lds_addr((const lds_u8*)B);
    lds_vu64a* IPS = (lds_vu64a*)slots;
    lds_vu64a* OPS = IPS + 4;
    RS_DECL
    while (true) {
        const int64_t b = readlane64(nxt_s, 0);
        if (b >= n) break;
        const RowMeta mt = meta[b];
        const int32_t nseq = __builtin_amdgcn_readfirstlane(mt.nseq);
        uint8_t* d = dst + dst_off[b];
        RS_COUNT(12, 1);
        if (nseq > 0) {
            if (tid == 0) opg_s = mt.op;
            const uint8_t* s = src + src_off[b];
            const int32_t iend = __builtin_amdgcn_readfirstlane(src_len[b]);
            const uint8_t* dl = lens + mt.loff;
            const int32_t nch = (nseq + 63) >> 6;
            // the recorded length of chunk k's lane (an unconditional load; lanes
            // past the block's end are masked where the value is used)
            auto lens_at = [&](int32_t k) -> int32_t {
                const int32_t i = 64 * k + (int32_t)lane;
                return (int32_t)dl[i < nseq ? i : nseq - 1];
            };
            // Prepare chunk k: input positions from its recorded lengths (the
            // input-position chain), then its 32 input bytes per lane requested.
            auto prepare = [&](int32_t k, int32_t dlv, int32_t& t, int32_t& clen, u32x4& a, u32x4& bb) {
                t = 0;
                clen = 0;
                if (k >= nch) return;
                const int32_t cnt = min(64, nseq - 64 * k);
                const bool act = (int32_t)lane < cnt;
                int32_t dlt = act ? dlv : 0;
                const uint32_t ip0 = k == 0 ? 0u : slot_wait(IPS + ((k - 1) & 3), (uint32_t)k, 0u);
                uint64_t esc = __ballot(act && dlt == 255);
                while (esc != 0) {   // lengths >= 255 were left to re-parse: serially, rare
                    const int e = __builtin_ctzll(esc);
                    esc &= esc - 1;
                    const int32_t pre = wave_incl_sum(dlt) - dlt;
                    if ((int)lane == e) {
                        const int32_t te = min((int32_t)ip0 + pre, iend - 18);
                        dlt = seq_clen(s + te, iend - te - 1);
                    }
                }
                const int32_t incl = wave_incl_sum(dlt);
                const int32_t tot = __builtin_amdgcn_readlane(incl, 63);
                if (lane == 0) slot_put(IPS + (k & 3), (uint32_t)(k + 1), ip0 + (uint32_t)tot);
                t = min((int32_t)ip0 + incl - dlt, iend - 18);   // good sequences: t + 18 <= iend
                clen = dlt;
                res_load_in(s, act ? t : 0, iend, a, bb);
            };
            // Three register sets, each {t, clen, a, b} of one prepared chunk,
            // and three length registers: iteration i runs set i % 3 and
            // prepares two chunks ahead into set (i + 2) % 3.  The loop is
            // unrolled three times so that no register still waiting for its
            // load is ever copied (a copy waits for every older load).
            struct PSet {
                int32_t t, clen;
                u32x4 a, b;
            };
            PSet S0, S1, S2;
            int32_t L0 = 0, L1 = 0, L2;
            {
                const int32_t l0 = lens_at((int32_t)wv), l1 = lens_at((int32_t)wv + kResW);
                prepare((int32_t)wv, l0, S0.t, S0.clen, S0.a, S0.b);
                prepare((int32_t)wv + kResW, l1, S1.t, S1.clen, S1.a, S1.b);
            }
            L2 = lens_at((int32_t)wv + 2 * kResW);
            // one chunk: execute set P (chunk c), prepare chunk c + 2W into set Q
            // with the length byte Lu, request chunk c + 3W's into Ll
            auto iter = [&](int32_t c, PSet& P, PSet& Q, int32_t& Lu, int32_t& Ll) __attribute__((always_inline)) {
                RS_MARK(0);
                RS_COUNT(10, 1);
                const int32_t t0 = P.t, c0 = P.clen;
                const u32x4 a0 = P.a, b0 = P.b;
                const int32_t cnt = min(64, nseq - 64 * c);
                bool act = (int32_t)lane < cnt;
                ResSeq q;
                res_parse(s, t0, iend, act, c0 >= 255, a0, b0, q);
                // ---- place: the output-position chain
                const int32_t olen = act ? q.lit + q.ml : 0;
                const int32_t oincl = wave_incl_sum(olen);
                RS_MARK(1);
                const uint32_t op0 = c == 0 ? 0u : slot_wait(OPS + ((c - 1) & 3), (uint32_t)c, kResStop);
                RS_MARK(2);
                int32_t o = 0;
                if (op0 == kResStop) {
                    act = false;
                    if (lane == 0) slot_put(OPS + (c & 3), (uint32_t)(c + 1), kResStop);
                } else {
                    o = (int32_t)op0 + oincl - olen;
                    const uint64_t cut = __ballot(act && o + olen > kResLim);
                    if (cut != 0) {   // past the LDS output: the finisher resumes at the first such sequence
                        const int e = __builtin_ctzll(cut);
                        if ((int)lane == e) {
                            meta[b].ip = t0;
                            meta[b].op = o;
                            opg_s = o;
                        }
                        act = act && (int)lane < e;
                        if (lane == 0) slot_put(OPS + (c & 3), (uint32_t)(c + 1), kResStop);
                    } else if (lane == 0) {
                        slot_put(OPS + (c & 3), (uint32_t)(c + 1), op0 + (uint32_t)__builtin_amdgcn_readlane(oincl, 63));
                    }
                }
                // ---- literals (independent of everything: written, then their bits set)
                const bool hl = act && q.lit > 0;
                const bool llong = hl && q.litg && q.lit > kResLong;
                if (hl && !llong) {
                    if (!q.litg) {   // bytes lp .. lp + lit - 1 of the 32 at hand (lp is 1 or 2)
                        const uint32_t sh = (uint32_t)q.lp;
                        const u32x4 x0{__builtin_amdgcn_alignbyte(a0.y, a0.x, sh), __builtin_amdgcn_alignbyte(a0.z, a0.y, sh),
                                       __builtin_amdgcn_alignbyte(a0.w, a0.z, sh), __builtin_amdgcn_alignbyte(b0.x, a0.w, sh)};
                        lds_put_ar(obase + (uint32_t)o, x0, q.lit);
                        if (q.lit > 16) {
                            const u32x4 x1{__builtin_amdgcn_alignbyte(b0.y, b0.x, sh), __builtin_amdgcn_alignbyte(b0.z, b0.y, sh),
                                           __builtin_amdgcn_alignbyte(b0.w, b0.z, sh), __builtin_amdgcn_alignbyte(0u, b0.w, sh)};
                            lds_put_ar(obase + (uint32_t)o + 16u, x1, q.lit - 16);
                        }
                    } else {
                        // good long literals end >= 32 bytes before the block end (lz4.c:2016-2027)
                        for (int32_t i = 0; i < q.lit; i += 16)
                            lds_put_ar(obase + (uint32_t)(o + i), ld16(s + min(t0 + q.lp + i, iend - 16)), q.lit - i);
                    }
                    bits_fill(B, o, q.lit);
                }
                for (uint64_t lw = __ballot(llong); lw != 0; lw &= lw - 1) {   // long literals: the whole wave
                    const int e = __builtin_ctzll(lw);
                    const int32_t oe = __builtin_amdgcn_readlane(o, e), le = __builtin_amdgcn_readlane(q.lit, e);
                    const uint8_t* se = s + __builtin_amdgcn_readlane(t0 + q.lp, e);
                    const int32_t lim = iend - 16 - __builtin_amdgcn_readlane(t0 + q.lp, e);
                    for (int32_t x = 16 * (int32_t)lane; x < le; x += 16 * 64)
                        lds_put_ar(obase + (uint32_t)(oe + x), ld16(se + min(x, lim)), le - x);
                    bits_fill_wave(B, oe, le, lane);
                }
                RS_MARK(3);
                // ---- matches: each copies once every source byte is written
                const int32_t m = o + q.lit, off = q.off, ml = q.ml, s0 = m - off;
                const bool per = off < 16;   // period pattern
                int32_t dn = 0;               // match bytes written
                bool pend = act, lng = false;
                for (int32_t it = 0; __any(pend); ++it) {
                    RS_COUNT(11, 1);
                    if (it == kResSpin) break;   // (bounded: see slot_wait)
                    if (pend && !lng) {
                        const int32_t sp = per ? s0 : s0 + dn;
                        const int32_t L = per ? off : min(min(32, ml - dn), off);
                        // the source's bits, then its bytes: one round trip
                        SrcRead rd;
                        src_read(bbase + 4u * (uint32_t)(sp >> 5), obase + ((uint32_t)sp & ~7u), rd);
                        if (bits_in(rd.bits, sp & 31, L)) {
                            const uint32_t q8 = (uint32_t)sp & 7u;
                            const u32x4 v0 = funnel16(rd.w0, rd.w1, rd.w2, q8);
                            if (per) {   // period pattern of the first off bytes
                                const u32x4 pat = period_pattern(v0, (uint32_t)off);
                                const int32_t stp = 16 - 16 % off;
                                const int32_t w = ml <= kResLong ? ml : 64;   // the rest on the whole wave
                                for (int32_t i = 0; i < w; i += stp) lds_put_ar(obase + (uint32_t)(m + i), pat, w - i);
                                bits_fill(B, m, w);
                                dn = w;
                                lng = true;   // any rest: on the whole wave
                            } else {
                                lds_put_ar(obase + (uint32_t)(m + dn), v0, L);
                                if (L > 16) lds_put_ar(obase + (uint32_t)(m + dn + 16), funnel16(rd.w2, rd.w3, rd.w4, q8), L - 16);
                                bits_set(B, m + dn, L);
                                dn += L;
                            }
                            pend = dn < ml;
                            lng = pend && (lng || ml - dn > kResLong);
                        }
                    }
                    // long copies: one step (up to 1 KiB) each, on the whole wave, once
                    // every piece's source is written.  A copy with offset off may read
                    // eff = off * j bytes back for any j with eff <= dn + off: the
                    // match's bytes repeat with period off.
                    for (uint64_t lg = __ballot(pend && lng); lg != 0; lg &= lg - 1) {
                        const int e = __builtin_ctzll(lg);
                        const int32_t me = __builtin_amdgcn_readlane(m, e), oe = __builtin_amdgcn_readlane(off, e);
                        const int32_t mle = __builtin_amdgcn_readlane(ml, e), de = __builtin_amdgcn_readlane(dn, e);
                        const int32_t eff = oe >= 1024 ? oe : oe * ((de + oe) / oe);
                        const int32_t W = min(eff & ~15, 1024);
                        const int32_t rem = mle - de;
                        const int32_t x = 16 * (int32_t)lane;
                        const bool pc = x < W && x < rem;
                        const int32_t qd = me + de + x, qs = qd - eff;
                        SrcRead rs;
                        const int32_t qq = pc ? qs : 0;
                        src_read(bbase + 4u * (uint32_t)(qq >> 5), obase + ((uint32_t)qq & ~7u), rs);
                        const bool rdy = !pc || bits_in(rs.bits, qq & 31, 16);
                        if (__ballot(!rdy) == 0) {
                            if (pc) lds_put_ar(obase + (uint32_t)qd, funnel16(rs.w0, rs.w1, rs.w2, (uint32_t)qq & 7u), rem - x);
                            const int32_t wl = min(W, rem);
                            bits_fill_wave(B, me + de, wl, lane);
                            if ((int)lane == e) {
                                dn = de + wl;
                                pend = dn < ml;
                            }
                        }
                    }
                }
                RS_MARK(5);
                // ---- the chunk two ahead: its input positions and bytes.  Issued
                // after the match loop, so that no load is in flight while it
                // runs (a wait for any register a pending load targets would
                // wait for it and every older load)
                prepare(c + 2 * kResW, Lu, Q.t, Q.clen, Q.a, Q.b);
                Ll = lens_at(c + 3 * kResW);
                RS_MARK(4);
            };
            for (int32_t c = (int32_t)wv; c < nch; c += 3 * kResW) {
                iter(c, S0, S2, L2, L0);
                if (c + kResW >= nch) break;
                iter(c + kResW, S1, S0, L0, L1);
                if (c + 2 * kResW >= nch) break;
                iter(c + 2 * kResW, S2, S1, L1, L2);
            }
        }
        RS_MARK(0);
        __syncthreads();   // every chunk of the block written
        RS_MARK(6);
        const int32_t og = nseq > 0 ? __builtin_amdgcn_readfirstlane(opg_s) : 0;
        for (int32_t x = 16 * (int32_t)tid; x < og; x += 16 * kResT) {
            const u32x4 v = lds_ld16(OUT + x);
            res_gput(d + x, v, og - x);
        }
        for (int32_t k = 4 * (int32_t)tid; k < (og + 31) >> 5; k += 4 * kResT) lds_st16((lds_u8*)(bitw + k), u32x4{0, 0, 0, 0});
        if (tid < 8) slots[tid] = 0;
        if (tid == 0) nxt_s = (int64_t)atomicAdd(&ctr[2], 1ull);
        __syncthreads();
        RS_MARK(7);
    }
    RS_FLUSH();
}

}  // namespace lz4m

using namespace lz4m;

#ifdef LZ4M_RES_PROF
extern "C" int lz4m_res_prof(unsigned long long* out, int reset) {
    hipError_t e = hipMemcpyFromSymbol(out, HIP_SYMBOL(lz4m::g_res_prof), sizeof(unsigned long long) * 16);
    if (e == hipSuccess && reset) {
        unsigned long long z[16] = {0};
        e = hipMemcpyToSymbol(HIP_SYMBOL(lz4m::g_res_prof), z, sizeof(z));
    }
    return (int)e;
}
#endif

extern "C" int lz4m_resident_exec_launch(const uint8_t* d_src, const int64_t* d_src_off, const int32_t* d_src_len,
                                         uint8_t* d_dst, const int64_t* d_dst_off, int64_t n, void* d_work,
                                         size_t work_bytes, hipStream_t stream) {
    const size_t fixed = lz4m_rows_fixed_bytes(n);
    if (work_bytes < fixed) return LZ4M_ROWS_ENOSPACE;
    unsigned long long* ctr = static_cast<unsigned long long*>(d_work);
    RowMeta* meta = reinterpret_cast<RowMeta*>(static_cast<uint8_t*>(d_work) + kRowsMeta);
    const uint8_t* lens = static_cast<const uint8_t*>(d_work) + fixed;
    int dev = 0, cus = 0, k = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&k, reinterpret_cast<const void*>(res_exec_kernel), kResT, 0);
    if (cus <= 0) cus = 256;
    const int64_t slots = (int64_t)cus * (k > 0 ? k : 1);
    const int64_t grid = n < slots ? n : slots;
    hipLaunchKernelGGL(res_exec_kernel, dim3((uint32_t)grid), dim3(kResT), 0, stream, d_src, d_src_off, d_src_len,
                       d_dst, d_dst_off, meta, lens, n, ctr);
    return (int)hipGetLastError();
}
