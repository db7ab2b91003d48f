/*
 * lz4m_xxh32_host.c -- streaming XXH32 on a HOST core (plain C99, no HIP).
 *
 * The frame content checksum (lz4frame.c:1041-1042, :1170-1176) is one XXH32
 * stream over all uncompressed bytes: four accumulators, each a serial
 * multiply-rotate recurrence with no associative combine, so
 * the GPU cannot split it (one wavefront runs it at 1.7 GB/s).  It runs here,
 * on a host core, beside the device work: the XXH32 specification
 * (xxhash.c:263-286 primes/round/avalanche, :290-348 tail, :437-554 the
 * streaming state; state layout xxhash.h:264-274, total length mod 2^32).
 *
 * Built with -fno-tree-vectorize: gcc turns the four accumulators into
 * SSE2 lanes with an emulated 32-bit multiply (1.9 GB/s instead of ~14).
 * Kept in its own C file so that it builds without the HIP toolchain: the
 * host sanitizer build (oracle/Makefile `asan`) compiles it with
 * -fsanitize=address,undefined next to the CPU restatement.
 */
#include "../../include/lz4m.h"

#include <string.h>

#define P1 0x9E3779B1u
#define P2 0x85EBCA77u
#define P3 0xC2B2AE3Du
#define P4 0x27D4EB2Fu
#define P5 0x165667B1u

static inline uint32_t rotl32(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }
static inline uint32_t rd32(const uint8_t* p) {
    uint32_t v;
    memcpy(&v, p, 4);
    return v;
}
static inline uint32_t xround(uint32_t acc, uint32_t in) { return rotl32(acc + in * P2, 13) * P1; }

/* 16-byte stripes [p, p + len & ~15) into the four accumulators */
static const uint8_t* stripes(uint32_t* v, const uint8_t* p, size_t len) {
    uint32_t a = v[0], b = v[1], c = v[2], d = v[3];
    const uint8_t* end = p + (len & ~(size_t)15);
    for (; p < end; p += 16) {
        a = xround(a, rd32(p));
        b = xround(b, rd32(p + 4));
        c = xround(c, rd32(p + 8));
        d = xround(d, rd32(p + 12));
    }
    v[0] = a;
    v[1] = b;
    v[2] = c;
    v[3] = d;
    return p;
}

void lz4m_xxh32_host_reset(lz4m_xxh32_state* st, uint32_t seed) {
    memset(st, 0, sizeof *st);
    st->v[0] = seed + P1 + P2;
    st->v[1] = seed + P2;
    st->v[2] = seed;
    st->v[3] = seed - P1;
}

void lz4m_xxh32_host_update(lz4m_xxh32_state* st, const void* input, size_t len) {
    if (len == 0 || input == NULL) return;
    const uint8_t* p = (const uint8_t*)input;
    st->total_len_32 += (uint32_t)len;
    st->large_len |= (uint32_t)((len >= 16) | (st->total_len_32 >= 16));
    uint8_t* mem = (uint8_t*)st->mem32;
    if (st->memsize + len < 16) { /* not a whole stripe yet: buffer it */
        memcpy(mem + st->memsize, p, len);
        st->memsize += (uint32_t)len;
        return;
    }
    if (st->memsize) { /* complete the buffered stripe */
        const size_t fill = 16 - st->memsize;
        memcpy(mem + st->memsize, p, fill);
        stripes(st->v, mem, 16);
        p += fill;
        len -= fill;
        st->memsize = 0;
    }
    const uint8_t* q = stripes(st->v, p, len);
    const size_t rest = len - (size_t)(q - p);
    if (rest) {
        memcpy(mem, q, rest);
        st->memsize = (uint32_t)rest;
    }
}

uint32_t lz4m_xxh32_host_digest(const lz4m_xxh32_state* st) {
    uint32_t h = st->large_len ? rotl32(st->v[0], 1) + rotl32(st->v[1], 7) + rotl32(st->v[2], 12) + rotl32(st->v[3], 18)
                               : st->v[2] /* the seed */ + P5;
    h += st->total_len_32;
    const uint8_t* p = (const uint8_t*)st->mem32;
    size_t n = st->memsize;
    for (; n >= 4; n -= 4, p += 4) h = rotl32(h + rd32(p) * P3, 17) * P4;
    for (; n > 0; --n, ++p) h = rotl32(h + (uint32_t)(*p) * P5, 11) * P1;
    h ^= h >> 15;
    h *= P2;
    h ^= h >> 13;
    h *= P3;
    h ^= h >> 16;
    return h;
}

uint32_t lz4m_xxh32_host(const void* input, size_t len, uint32_t seed) {
    lz4m_xxh32_state st;
    lz4m_xxh32_host_reset(&st, seed);
    lz4m_xxh32_host_update(&st, input, len);
    return lz4m_xxh32_host_digest(&st);
}
