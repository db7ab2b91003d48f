// Prototype (dev only, not part of the library): a cooperative LZ4 block
// decoder, one wavefront per block, to price DESIGN.md section 8's next step
// against the lane-per-block decoder.  It decodes the "simple" prefix of each
// valid block -- sequences with literal <= 12 bytes and at most one extra
// match-length byte, inside the reference fast loop's margins -- and reports
// how far it got (ip, op); the exact lane decoder would finish the rest.
//
// Per round (up to 64 sequences):
//   1. the wave stages 1 KiB of input at ip in LDS (16 B per lane);
//   2. every lane parses a speculative sequence at position pos + lane, and a
//      readlane walk follows the chain of sequence starts from pos;
//   3. sequence k is re-parsed in lane k; a wave prefix sum gives output
//      positions; literals are written (exact byte counts);
//   4. matches are copied in passes: a match is ready once its source ends
//      before the first pending match's start (all earlier output is final).
// Sequences with literals > 12 bytes run one at a time on the whole wave.
//
// Measured (tools/probe_coop.py, 262 144 silesia-like blocks, MI355X): the
// decoded prefix is bit-exact and covers 91.6 % of the output (text 99.9 %),
// at 52 / 80 / 100 GB/s with 16 / 32 / 64 resident waves per CU, against
// 351 GB/s for the lane decoder: ~44 us per 64-sequence round, i.e. the
// round is a chain of memory round trips (input staging, the literal fence,
// one fence per readiness pass).  Blocks are assigned statically: an
// atomic work queue in this loop nest compiled to a kernel that hung.
// Round statistics (summed into the `queue` words 0-3; 65 536 blocks):
// silesia-like 175 rounds per block (49 of them single long-literal steps),
// 4.6 readiness passes per round, 49 sequences per parallel round; text 310
// rounds (113 single steps), 2.0 passes per round.
#include "../../python-lz4_amd/csrc/lz4m_common.h"

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace lz4m {
namespace {

constexpr int kIn = 1024;

__device__ __forceinline__ void put_exact_g(uint8_t* p, u32x4 v, uint32_t k) {
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

__device__ __forceinline__ int32_t incl_sum(int32_t v) {
    v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xF, 0xF, false);
    v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xF, 0xF, false);
    v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xF, 0xF, false);
    v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xF, 0xF, false);
    v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xA, 0xF, false);
    v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xC, 0xF, false);
    return v;
}


// whole-wave exact copies (one sequence at a time, for literals > 12 bytes or
// matches past the simple path)
__device__ __forceinline__ void wave_copy_lit(uint8_t* d, const uint8_t* s, int32_t len, uint32_t lane) {
    for (int32_t base = 0; base < len; base += 1024) {
        const int32_t pos = base + 16 * (int32_t)lane;
        if (pos < len) put_exact_g(d + pos, ld16(s + pos), (uint32_t)(len - pos));
    }
}

__device__ __forceinline__ void wave_copy_match(uint8_t* d, int32_t off, int32_t len, uint32_t lane) {
    if (off >= 16) {
        const int32_t w = (off < 1024 ? off : 1024) & ~15;
        for (int32_t base = 0; base < len; base += w) {
            const int32_t pos = base + 16 * (int32_t)lane;
            if (pos < base + w && pos < len) put_exact_g(d + pos, ld16(d + pos - off), (uint32_t)(len - pos));
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
        }
        return;
    }
    const u32x4 pat = period_pattern(ld16(d - off), (uint32_t)off);
    const int32_t step = 16 - (16 % off);
    for (int32_t pos = step * (int32_t)lane; pos < len; pos += step * 64) put_exact_g(d + pos, pat, (uint32_t)(len - pos));
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
}

__device__ __forceinline__ int32_t rdl(int32_t v, int l) { return __builtin_amdgcn_readlane(v, l); }

__global__ __launch_bounds__(256) void coop_kernel(const uint8_t* __restrict__ src, const int64_t* __restrict__ soff,
                                                   const int32_t* __restrict__ slen, uint8_t* dst,
                                                   const int64_t* __restrict__ doff, const int32_t* __restrict__ dcap,
                                                   int32_t* __restrict__ prog, int64_t n,
                                                   unsigned long long* queue) {
    __shared__ __attribute__((aligned(16))) uint8_t ins[4][kIn + 64];
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    lds_u8* IN = (lds_u8*)ins[wv];
    const int64_t waves = (int64_t)gridDim.x * 4;
    for (int64_t b = (int64_t)blockIdx.x * 4 + wv; b < n; b += waves) {
        const uint8_t* s = src + soff[b];
        uint8_t* d = dst + doff[b];
        const int32_t iend = slen[b], oend = dcap[b];
        int32_t ip = 0, op = 0, why = 0, rounds = 0, npass = 0, nsingle = 0, nseqs = 0;
        bool go = oend >= 64 && iend > 0;
        while (go) {
            if (++rounds > 8192) {   // debug cap
                why = 1;
                break;
            }
            // 1. input window [ib, ib + 1 KiB)
            const int32_t ib = ip & ~15;
            {
                const int32_t x = ib + 16 * (int32_t)lane;
                const u32x4 v = x + 16 <= iend ? ld16(s + x) : ld16_guarded(s + x, iend - x);
                lds_st16(IN + 16 * lane, v);
            }
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
            // 2. speculative parse + walk
            int32_t myseq = 0;
            int nseq = 0;
            bool stop = false;
            int32_t pos = ip - ib;
            int guard = 0;
            while (nseq < 64 && pos + 80 <= kIn && ++guard < 128) {
                const u32x4 w = lds_ld16(IN + pos + (int32_t)lane);
                const uint32_t tok = w.x & 0xFFu, lit = tok >> 4, mlc = tok & 15u;
                bool simple = lit <= 12;
                int32_t adv = 3 + (int32_t)lit;
                if (mlc == 15) {
                    simple = simple && byte_of(w, (int)(3 + (lit < 12 ? lit : 12))) != 255u;
                    adv += 1;
                }
                const int32_t nxt = (int32_t)lane + adv;
                const uint64_t smask = __ballot(simple);
                int32_t sidx = 0;
                while (sidx < 64 && nseq < 64) {
                    if (!((smask >> sidx) & 1ull)) {
                        stop = true;
                        break;
                    }
                    if ((int)lane == nseq) myseq = pos + sidx;
                    ++nseq;
                    sidx = rdl(nxt, sidx);
                }
                pos += sidx;
                if (stop) break;
            }
            if (nseq == 0) {
                ++nsingle;
                // one long sequence, whole wave (uniform values)
                int32_t q = ip + 1;
                const uint32_t tok = s[ip];
                int32_t lit = (int32_t)(tok >> 4), ml = (int32_t)(tok & 15u);
                bool okk = true;
                if (lit == 15) {
                    uint32_t x = 255;
                    while (x == 255 && q < iend - 15) {
                        x = s[q++];
                        lit += (int32_t)x;
                    }
                    okk = x != 255;
                }
                okk = okk && q + lit <= iend - 32 && op + lit <= oend - 32;
                if (!okk) break;
                wave_copy_lit(d + op, s + q, lit, lane);
                q += lit;
                const int32_t off = (int32_t)s[q] | ((int32_t)s[q + 1] << 8);
                q += 2;
                if (ml == 15) {
                    uint32_t x = 255;
                    while (x == 255 && q < iend - 4) {
                        x = s[q++];
                        ml += (int32_t)x;
                    }
                    if (x == 255) break;
                }
                ml += 4;
                __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
                if (off < 1 || off > op + lit || op + lit + ml >= oend - 64) break;
                wave_copy_match(d + op + lit, off, ml, lane);
                op += lit + ml;
                ip = q;
                continue;
            }
            // 3. sequence k in lane k
            const bool act = (int)lane < nseq;
            const u32x4 w = lds_ld16(IN + (act ? myseq : 0));
            const uint32_t tok = w.x & 0xFFu, mlc = tok & 15u;
            const int32_t lit = (int32_t)(tok >> 4) & 15;
            const int32_t off = (int32_t)(window_dword(w, (uint32_t)(1 + (lit < 12 ? lit : 12))) & 0xFFFFu);
            int32_t ml = (int32_t)mlc + 4, adv = 3 + lit;
            if (mlc == 15) {
                ml = 19 + (int32_t)byte_of(w, 3 + (lit < 12 ? lit : 12));
                adv += 1;
            }
            const int32_t len = act ? lit + ml : 0;
            const int32_t inc = incl_sum(len);
            const int32_t o = op + inc - len;
            const int32_t sabs = ib + myseq;
            const bool ok = act && lit <= 12 && sabs + 1 <= iend - 17 && sabs + adv <= iend - 5 &&
                            o + len < oend - 64 && off >= 1 && off <= o + lit;
            const uint64_t actm = __ballot(act), bad = actm & ~__ballot(ok);
            const int use = bad ? __builtin_ctzll(bad) : nseq;
            if (use == 0) break;
            const bool u = (int)lane < use;
            if (u && lit > 0) put_exact_g(d + o, window_shift1(w), (uint32_t)lit);
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
            // 4. matches in readiness passes
            const int32_t m = o + lit;
            const int32_t src_hi = m - off + (off < ml ? off : ml);
            uint64_t pend = __ballot(u);
            int passes = 0;
            while (pend) {
                if (++passes > 70) {
                    why = 2;
                    break;
                }
                const int32_t E = rdl(m, __builtin_ctzll(pend));
                const bool ready = ((pend >> lane) & 1ull) && src_hi <= E;
                if (ready) {
                    if (off >= 16) {
                        for (int32_t i = 0; i < ml; i += 16) put_exact_g(d + m + i, ld16(d + m - off + i), (uint32_t)(ml - i));
                    } else {
                        const u32x4 pat = period_pattern(ld16(d + m - off), (uint32_t)off);
                        const int32_t step = 16 - (16 % off);
                        for (int32_t i = 0; i < ml; i += step) put_exact_g(d + m + i, pat, (uint32_t)(ml - i));
                    }
                }
                __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
                pend &= ~__ballot(ready);
            }
            npass += passes;
            nseqs += use;
            op = rdl(o + len, use - 1);
            ip = ib + rdl(myseq + adv, use - 1);
            if (why) break;
            if (use < nseq) break;   // a sequence outside the fast margins: hand off
        }
        if (lane == 0) {
            atomicAdd(queue, (unsigned long long)rounds);
            atomicAdd(queue + 1, (unsigned long long)npass);
            atomicAdd(queue + 2, (unsigned long long)nsingle);
            atomicAdd(queue + 3, (unsigned long long)nseqs);
            prog[2 * b] = why ? -why : ip;
            prog[2 * b + 1] = op;
        }
    }
}

}  // namespace
}  // namespace lz4m

extern "C" int coop_decode(const uint8_t* src, const int64_t* soff, const int32_t* slen, uint8_t* dst,
                           const int64_t* doff, const int32_t* dcap, int32_t* prog, int64_t n, void* queue,
                           int grid, void* stream) {
    hipLaunchKernelGGL(lz4m::coop_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, src, soff, slen, dst, doff,
                       dcap, prog, n, (unsigned long long*)queue);
    return (int)hipGetLastError();
}
