/*
 * oracle/asan_check.c -- host sanitizer run (TEST INFRASTRUCTURE ONLY).
 *
 * SURVEY.md section 5 "Race detection/sanitizers": the CPU code of this
 * repository -- the restatement in lz4_oracle.c and the package's own host
 * XXH32 (python-lz4_amd/csrc/lz4m_xxh32_host.c) -- is built with
 * -fsanitize=address,undefined (oracle/Makefile `asan`) and driven here over
 * the inputs the reference's safety contract is about (lz4.h:197-200: never
 * read or write outside the given buffers): every buffer is its own exact-size
 * heap allocation, so any access one byte outside is reported.
 *
 *   - compress: sizes 0..70 000 (ragged, both table layouts, accelerations),
 *     limitedOutput with capacity = compressed size - 1 and tiny capacities;
 *   - decompress: the valid blocks with exact / short / zero capacity,
 *     truncations, random byte mutations and pure garbage (lz4.c:1936-2339);
 *   - dict= compress (lz4.c:1541-1581) and usingDict decode, linked streams;
 *   - XXH32: one-shot vs the streaming state fed in random chunks, and the
 *     package's host XXH32 against the restatement.
 * Exit status 0 = no finding and every round trip exact.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../include/lz4m.h"

int orc_compress_bound(int n);
int orc_compress(const uint8_t* src, int n, uint8_t* dst, int cap, int variant, int accel);
int orc_compress_dict(const uint8_t* win, int64_t d_len, int n, uint8_t* dst, int cap, int accel);
int orc_compress_linked(const uint8_t* src, int64_t n, int bsize, int accel, uint8_t* dst, int64_t dst_stride,
                        int32_t* out_len);
int orc_decompress_safe(const uint8_t* src, uint8_t* dst, int src_size, int cap);
int orc_decompress_dict(const uint8_t* src, uint8_t* dst, int src_size, int cap, const uint8_t* dict,
                        size_t dict_len);
uint32_t orc_xxh32(const void* input, size_t len, uint32_t seed);
size_t orc_xxh32_state_size(void);
void orc_xxh32_reset(void* s, uint32_t seed);
void orc_xxh32_update(void* s, const void* input, size_t len);
uint32_t orc_xxh32_digest(const void* s);

static uint64_t g_rng = 0x9E3779B97F4A7C15ull;
static uint32_t rnd(void) {
    g_rng ^= g_rng << 13;
    g_rng ^= g_rng >> 7;
    g_rng ^= g_rng << 17;
    return (uint32_t)(g_rng >> 11);
}

static int g_fail = 0;
#define CHECK(c, ...)                          \
    do {                                       \
        if (!(c)) {                            \
            fprintf(stderr, "FAIL: " __VA_ARGS__); \
            fputc('\n', stderr);               \
            g_fail = 1;                        \
        }                                      \
    } while (0)

/* exact-size copy: ASan sees the block's true end */
static uint8_t* dup_exact(const uint8_t* p, size_t n) {
    uint8_t* q = (uint8_t*)malloc(n ? n : 1);
    if (n) memcpy(q, p, n);
    return q;
}

/* compressible test data: words, short repeats, runs, noise */
static void fill(uint8_t* p, int n, int kind) {
    static const char* words[] = {"lz4 ", "block ", "frame ", "the ", "decoder ", "HBM ", "wave ", "of ", "\n"};
    int i = 0;
    while (i < n) {
        const int what = kind == 0 ? (int)(rnd() % 4) : kind - 1;
        if (what == 0) {
            const char* w = words[rnd() % 9];
            for (int j = 0; w[j] && i < n; ++j) p[i++] = (uint8_t)w[j];
        } else if (what == 1 && i > 8) {
            const int off = 1 + (int)(rnd() % (i < 300 ? i : 300)), len = 4 + (int)(rnd() % 40);
            for (int j = 0; j < len && i < n; ++j, ++i) p[i] = p[i - off];
        } else if (what == 2) {
            const uint8_t b = (uint8_t)rnd();
            for (int j = 0, len = 1 + (int)(rnd() % 300); j < len && i < n; ++j) p[i++] = b;
        } else {
            p[i++] = (uint8_t)rnd();
        }
    }
}

static void roundtrip(const uint8_t* data, int n, int variant, int accel) {
    uint8_t* src = dup_exact(data, (size_t)n);
    const int bound = orc_compress_bound(n);
    uint8_t* c = (uint8_t*)malloc((size_t)bound);
    const int clen = orc_compress(src, n, c, bound, variant, accel);
    CHECK(clen > 0, "compress n=%d variant=%d", n, variant);
    uint8_t* cx = dup_exact(c, (size_t)clen);
    /* limitedOutput: one byte short fails cleanly, a tiny capacity too */
    if (clen > 1) {
        uint8_t* s = (uint8_t*)malloc((size_t)clen - 1);
        CHECK(orc_compress(src, n, s, clen - 1, variant, accel) == 0, "limited n=%d", n);
        free(s);
    }
    {
        const int tiny = (int)(rnd() % 16) + 1;
        uint8_t* s = (uint8_t*)malloc((size_t)tiny);
        (void)orc_compress(src, n, s, tiny, variant, accel);
        free(s);
    }
    /* decode with the exact capacity, a short capacity and no capacity */
    uint8_t* out = (uint8_t*)malloc(n ? (size_t)n : 1);
    const int r = orc_decompress_safe(cx, out, clen, n);
    CHECK(r == n && (n == 0 || memcmp(out, src, (size_t)n) == 0), "roundtrip n=%d r=%d", n, r);
    if (n > 0) {
        const int cap = (int)(rnd() % (uint32_t)n);
        uint8_t* o2 = (uint8_t*)malloc(cap ? (size_t)cap : 1);
        CHECK(orc_decompress_safe(cx, o2, clen, cap) < 0, "short capacity n=%d cap=%d", n, cap);
        free(o2);
    }
    /* truncations and mutations: any status, no out-of-bounds access */
    for (int t = 0; t < 6 && clen > 0; ++t) {
        const int cut = (int)(rnd() % (uint32_t)clen);
        uint8_t* tr = dup_exact(cx, (size_t)cut);
        (void)orc_decompress_safe(tr, out, cut, n);
        free(tr);
    }
    for (int t = 0; t < 10 && clen > 0; ++t) {
        uint8_t* m = dup_exact(cx, (size_t)clen);
        for (int f = 0, nf = 1 + (int)(rnd() % 4); f < nf; ++f) m[rnd() % (uint32_t)clen] = (uint8_t)rnd();
        (void)orc_decompress_safe(m, out, clen, n);
        free(m);
    }
    free(out);
    free(cx);
    free(c);
    free(src);
}

static void garbage(void) {
    for (int t = 0; t < 2000; ++t) {
        const int n = (int)(rnd() % 200), cap = (int)(rnd() % 400);
        uint8_t* g = (uint8_t*)malloc(n ? (size_t)n : 1);
        for (int i = 0; i < n; ++i) g[i] = (uint8_t)rnd();
        uint8_t* o = (uint8_t*)malloc(cap ? (size_t)cap : 1);
        (void)orc_decompress_safe(g, o, n, cap);
        free(o);
        free(g);
    }
}

static void dict_cases(const uint8_t* data, int total) {
    static const int dlens[] = {0, 5, 8, 100, 20000, 65536, 100000};
    for (size_t k = 0; k < sizeof dlens / sizeof dlens[0]; ++k) {
        const int dl = dlens[k] < total / 2 ? dlens[k] : total / 2;
        const int n = 1 + (int)(rnd() % 65536);
        if (dl + n > total) continue;
        /* LZ4_loadDict keeps nothing of a dictionary below 8 B (lz4.c:1564-1566) */
        const int dt = dl < 8 ? 0 : dl > 65536 ? 65536 : dl;
        /* window = last dt bytes of the dictionary followed by the source */
        uint8_t* win = dup_exact(data + (dl - dt), (size_t)(dt + n));
        const int bound = orc_compress_bound(n);
        uint8_t* c = (uint8_t*)malloc((size_t)bound);
        const int clen = orc_compress_dict(win, dl, n, c, bound, 1 + (int)(rnd() % 3));
        CHECK(clen > 0, "dict compress dl=%d n=%d", dl, n);
        uint8_t* dict = dup_exact(data, (size_t)dl);
        uint8_t* cx = dup_exact(c, (size_t)clen);
        uint8_t* out = (uint8_t*)malloc((size_t)n);
        const int r = orc_decompress_dict(cx, out, clen, n, dl ? dict : NULL, (size_t)dl);
        CHECK(r == n && memcmp(out, data + dl, (size_t)n) == 0, "dict roundtrip dl=%d n=%d r=%d", dl, n, r);
        free(out);
        free(cx);
        free(dict);
        free(c);
        free(win);
    }
}

static void linked_cases(const uint8_t* data, int total) {
    const int bsize = 65536;
    const int n = total < 5 * bsize + 1234 ? total : 5 * bsize + 1234;
    const int nb = (n + bsize - 1) / bsize;
    uint8_t* src = dup_exact(data, (size_t)n);
    uint8_t* dst = (uint8_t*)malloc((size_t)nb * bsize);
    int32_t* lens = (int32_t*)malloc(sizeof(int32_t) * (size_t)nb);
    CHECK(orc_compress_linked(src, n, bsize, 1, dst, bsize, lens) == nb, "linked block count");
    /* decode block k with the previous 64 KiB of output as its dictionary */
    uint8_t* out = (uint8_t*)malloc((size_t)n);
    for (int k = 0; k < nb; ++k) {
        const int pos = k * bsize, len = n - pos < bsize ? n - pos : bsize;
        if (lens[k] == 0) {
            memcpy(out + pos, src + pos, (size_t)len);
            continue;
        }
        uint8_t* cx = dup_exact(dst + (size_t)k * bsize, (size_t)lens[k]);
        const int dl = pos < 65536 ? pos : 65536;
        const int r = orc_decompress_dict(cx, out + pos, lens[k], len, dl ? out + pos - dl : NULL, (size_t)dl);
        CHECK(r == len, "linked block %d r=%d", k, r);
        free(cx);
    }
    CHECK(memcmp(out, src, (size_t)n) == 0, "linked roundtrip");
    free(out);
    free(lens);
    free(dst);
    free(src);
}

static void xxh_cases(const uint8_t* data, int total) {
    void* st = malloc(orc_xxh32_state_size());
    for (int t = 0; t < 300; ++t) {
        const int n = (int)(rnd() % (t < 200 ? 100u : (uint32_t)total));
        const uint32_t seed = t & 1 ? rnd() : 0;
        uint8_t* p = dup_exact(data + (rnd() % (uint32_t)(total - n + 1)), (size_t)n);
        const uint32_t h = orc_xxh32(p, (size_t)n, seed);
        lz4m_xxh32_state hs;
        lz4m_xxh32_host_reset(&hs, seed);
        orc_xxh32_reset(st, seed);
        for (int i = 0; i < n;) {
            const int c = (int)(rnd() % 40u) + (rnd() & 1 ? 0 : (int)(rnd() % 5000u));
            const int k = c < n - i ? c : n - i;
            uint8_t* chunk = dup_exact(p + i, (size_t)k);
            lz4m_xxh32_host_update(&hs, chunk, (size_t)k);
            orc_xxh32_update(st, chunk, (size_t)k);
            free(chunk);
            i += k;
        }
        CHECK(orc_xxh32_digest(st) == h, "orc streaming xxh32 n=%d", n);
        CHECK(lz4m_xxh32_host_digest(&hs) == h, "host streaming xxh32 n=%d", n);
        CHECK(lz4m_xxh32_host(p, (size_t)n, seed) == h, "host one-shot xxh32 n=%d", n);
        free(p);
    }
    free(st);
}

int main(void) {
    const int total = 400000;
    uint8_t* data = (uint8_t*)malloc((size_t)total);
    fill(data, total, 0);
    static const int sizes[] = {0, 1, 4, 5, 12, 13, 14, 15, 16, 17, 31, 32, 63, 64, 100, 255, 256, 1000, 4096,
                                65535, 65536, 65547, 65548, 70000};
    for (size_t i = 0; i < sizeof sizes / sizeof sizes[0]; ++i)
        for (int variant = sizes[i] < 65547 ? 0 : 1; variant < 2; ++variant) roundtrip(data + (rnd() % 1000), sizes[i], variant, 1);
    for (int t = 0; t < 150; ++t) {
        const int n = (int)(rnd() % 70001u);
        uint8_t* p = (uint8_t*)malloc(n ? (size_t)n : 1);
        fill(p, n, (int)(rnd() % 5));
        /* byU16 / hash4 only below 65 547 B (lz4.c:1353-1354) */
        roundtrip(p, n, n < 65547 ? (int)(rnd() & 1) : 1, t % 7 == 0 ? 1 + (int)(rnd() % 70000u) : 1);
        free(p);
    }
    garbage();
    dict_cases(data, total);
    linked_cases(data, total);
    xxh_cases(data, total);
    free(data);
    printf("asan_check: %s\n", g_fail ? "FAILED" : "ok");
    return g_fail;
}
