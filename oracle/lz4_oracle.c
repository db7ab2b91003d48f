/*
 * oracle/lz4_oracle.c -- CPU restatement of the reference LZ4 block codec and
 * XXH32 for the batched hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the shipped package links, loads or
 * calls this file; only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may use it, and only as the checker.
 *
 * It is written from the format semantics of the vendored lz4 v1.9.4
 * (/root/reference/lz4libs), not copied: each function cites the reference
 * lines whose behaviour it restates.  Parity of this restatement is pinned by
 * tests/test_oracle.py against (a) the reference compiled from source into
 * oracle/_ref/ (oracle/Makefile) and (b) the golden vectors committed in
 * tests/golden/ (generated from oracle/_ref by tests/golden/make_golden.py).
 *
 * Decoder behaviour is that of the x86_64 build of the reference
 * (LZ4_FAST_DEC_LOOP=1, lz4.c:457-470): the fast phase and the safe phase
 * differ in which malformed inputs they reject and at which input position,
 * so both phases are restated.
 */
#include <stdint.h>
#include <stddef.h>
#include <string.h>

#define ORC_MINMATCH      4      /* lz4.c:240 */
#define ORC_LASTLITERALS  5      /* lz4.c:243 */
#define ORC_MFLIMIT       12     /* lz4.c:244 */
#define ORC_MIN_LENGTH    13     /* lz4.c:247 */
#define ORC_LIMIT_64K     (65536 + ORC_MFLIMIT - 1)   /* lz4.c:689 */
#define ORC_MAX_INPUT     0x7E000000                  /* lz4.h:211 */
#define ORC_DIST_MAX      65535                       /* lz4.h:632 */
#define ORC_ACCEL_MAX     65537                       /* lz4.c:53 */

enum { ORC_TABLE_U16_HASH4 = 0, ORC_TABLE_U32_HASH5 = 1 };

static uint16_t orc_rd16(const uint8_t* p) { return (uint16_t)(p[0] | (p[1] << 8)); }
static uint32_t orc_rd32(const uint8_t* p) { uint32_t v; memcpy(&v, p, 4); return v; }
static uint64_t orc_rd64(const uint8_t* p) { uint64_t v; memcpy(&v, p, 8); return v; }

int orc_compress_bound(int n)     /* lz4.h:212 */
{
    if ((unsigned)n > (unsigned)ORC_MAX_INPUT) return 0;
    return n + n / 255 + 16;
}

/* Hash of the bytes at p for the two table layouts (lz4.c:756-780):
 * byU16 tables hash 4 bytes into 13 bits, byU32 tables hash 5 bytes into
 * 12 bits (LZ4_MEMORY_USAGE 14, lz4.h:150-170). */
static uint32_t orc_hash(const uint8_t* p, int variant)
{
    if (variant == ORC_TABLE_U16_HASH4)
        return (orc_rd32(p) * 2654435761u) >> (32 - 13);
    return (uint32_t)(((orc_rd64(p) << 24) * 889523592379ull) >> (64 - 12));
}

/* Forward match length, capped at `limit` (lz4.c:658-682). */
static unsigned orc_count(const uint8_t* a, const uint8_t* b, const uint8_t* limit)
{
    const uint8_t* const start = a;
    while (a < limit && *a == *b) { a++; b++; }
    return (unsigned)(a - start);
}

static uint8_t* orc_put_len(uint8_t* op, unsigned len)
{
    while (len >= 255) { *op++ = 255; len -= 255; }
    *op++ = (uint8_t)len;
    return op;
}

/*
 * Greedy single-pass compressor with a fresh, zeroed hash table.
 * Restates LZ4_compress_generic_validated (lz4.c:910-1302) for the modes the
 * hot path uses:
 *   variant U16_HASH4  = LZ4_compress_default on inputs < 65547 B
 *                        (byU16, noDict, noDictIssue; lz4.c:1352-1354) and the
 *                        frame's independent blocks (lz4.c:1378-1406);
 *   variant U32_HASH5  = lz4.block.compress (_block.c:93-121 ->
 *                        LZ4_compress_fast_continue on a reset stream,
 *                        byU32 + withPrefix64k with dictSize 0, lz4.c:1632-1675)
 *                        and LZ4_compress_default on inputs >= 65547 B.
 * `cap` < bound selects limitedOutput: returns 0 when the block does not fit
 * (lz4.c:1085-1087, 1158-1181, 1269-1279).
 */
int orc_compress(const uint8_t* src, int n, uint8_t* dst, int cap, int variant, int accel)
{
    static const int kSkipTrigger = 6;                     /* lz4.c:690 */
    uint32_t table[8192];
    const uint8_t* const iend = src + n;
    const uint8_t* const mflimit1 = iend - ORC_MFLIMIT + 1;  /* lz4.c:942 */
    const uint8_t* const matchlimit = iend - ORC_LASTLITERALS;
    const uint8_t* anchor = src;
    const uint8_t* ip = src;
    uint8_t* op = dst;
    uint8_t* const olimit = dst + cap;
    const int limited = cap < orc_compress_bound(n);
    uint32_t fwd_h;

    if ((unsigned)n > (unsigned)ORC_MAX_INPUT) return 0;           /* lz4.c:1324 */
    if (accel < 1) accel = 1;                                      /* lz4.c:1350-1351 */
    if (accel > ORC_ACCEL_MAX) accel = ORC_ACCEL_MAX;
    if (n == 0) {                                                  /* lz4.c:1325-1336 */
        if (limited && cap <= 0) return 0;
        dst[0] = 0;
        return 1;
    }
    if (variant == ORC_TABLE_U16_HASH4 && n >= ORC_LIMIT_64K) return 0;   /* lz4.c:963 */
    memset(table, 0, sizeof(table));
    if (n < ORC_MIN_LENGTH) goto last_literals;                    /* lz4.c:981 */

    table[orc_hash(ip, variant)] = 0;                              /* lz4.c:984 */
    ip++;
    fwd_h = orc_hash(ip, variant);

    for (;;) {
        const uint8_t* match;
        uint8_t* token;

        {   /* search with skip acceleration (lz4.c:1016-1075) */
            const uint8_t* fwd = ip;
            int step = 1;
            int attempts = accel << kSkipTrigger;
            for (;;) {
                const uint32_t h = fwd_h;
                const uint32_t cur = (uint32_t)(fwd - src);
                const uint32_t cand = table[h];
                ip = fwd;
                fwd += step;
                step = attempts++ >> kSkipTrigger;
                if (fwd > mflimit1) goto last_literals;
                match = src + cand;
                fwd_h = orc_hash(fwd, variant);
                table[h] = cur;
                if (variant == ORC_TABLE_U32_HASH5 && cand + ORC_DIST_MAX < cur)
                    continue;                                      /* lz4.c:1064-1067 */
                if (orc_rd32(match) == orc_rd32(ip)) break;        /* lz4.c:1070 */
            }
        }

        /* backward catch-up (lz4.c:1080) */
        while (ip > anchor && match > src && ip[-1] == match[-1]) { ip--; match--; }

        {   /* literal run (lz4.c:1083-1107) */
            const unsigned lit = (unsigned)(ip - anchor);
            token = op++;
            if (limited && op + lit + (2 + 1 + ORC_LASTLITERALS) + lit / 255 > olimit) return 0;
            if (lit >= 15) { *token = 15 << 4; op = orc_put_len(op, lit - 15); }
            else *token = (uint8_t)(lit << 4);
            memcpy(op, anchor, lit);
            op += lit;
        }

next_match:
        /* offset + match length (lz4.c:1125-1197) */
        {
            const unsigned off = (unsigned)(ip - match);
            unsigned mcode;
            op[0] = (uint8_t)off; op[1] = (uint8_t)(off >> 8); op += 2;
            mcode = orc_count(ip + ORC_MINMATCH, match + ORC_MINMATCH, matchlimit);
            ip += mcode + ORC_MINMATCH;
            if (limited && op + (1 + ORC_LASTLITERALS) + (mcode + 240) / 255 > olimit) return 0;
            if (mcode >= 15) { *token += 15; op = orc_put_len(op, mcode - 15); }
            else *token += (uint8_t)mcode;
        }
        anchor = ip;
        if (ip >= mflimit1) break;                                 /* lz4.c:1204 */

        table[orc_hash(ip - 2, variant)] = (uint32_t)(ip - 2 - src);   /* lz4.c:1207 */

        {   /* immediate re-match at ip, no catch-up (lz4.c:1218-1258) */
            const uint32_t h = orc_hash(ip, variant);
            const uint32_t cur = (uint32_t)(ip - src);
            const uint32_t cand = table[h];
            match = src + cand;
            table[h] = cur;
            if ((variant == ORC_TABLE_U16_HASH4 || cand + ORC_DIST_MAX >= cur)
                && orc_rd32(match) == orc_rd32(ip)) {
                token = op++;
                *token = 0;
                goto next_match;
            }
        }
        fwd_h = orc_hash(++ip, variant);                           /* lz4.c:1262 */
    }

last_literals:
    {   /* lz4.c:1266-1293 */
        const size_t run = (size_t)(iend - anchor);
        if (limited && op + run + 1 + (run + 255 - 15) / 255 > olimit) return 0;
        if (run >= 15) { *op++ = 15 << 4; op = orc_put_len(op, (unsigned)(run - 15)); }
        else *op++ = (uint8_t)(run << 4);
        memcpy(op, anchor, run);
        op += run;
    }
    return (int)(op - dst);
}

int orc_compress_default(const uint8_t* src, uint8_t* dst, int n, int cap)
{   /* lz4.c:1346-1367, 1435-1438 */
    return orc_compress(src, n, dst, cap,
                        n < ORC_LIMIT_64K ? ORC_TABLE_U16_HASH4 : ORC_TABLE_U32_HASH5, 1);
}

int orc_compress_block_api(const uint8_t* src, uint8_t* dst, int n, int cap, int accel)
{   /* _block.c:93-121 (non-HC, no dict) */
    return orc_compress(src, n, dst, cap, ORC_TABLE_U32_HASH5, accel);
}

/*
 * Greedy byU32 compressor of one block that has HISTORY: the streaming modes
 * of LZ4_compress_fast_continue (lz4.c:1632-1708) restated over one
 * contiguous window w[0 .. hist+n): history w[0 .. hist), block w[hist ..).
 * The caller owns the 4096-entry table (carried across calls).
 *
 * A table entry is an index; window byte p has index ibase + p, so the block
 * starts at index ibase + hist (the stream's currentOffset, lz4.c:925-926).
 * Candidates with index < low_idx are outside the valid area (dictSmall,
 * lz4.c:1061, 1247); candidates further than 65535 back are too far
 * (lz4.c:1062-1065).  Backward catch-up (lz4.c:1080) stops at window byte
 * low_src for matches inside the block and low_dict for matches in the
 * history (extDict sets lowLimit per candidate, lz4.c:1036-1053; prefix mode
 * fixes it at source - dictSize, lz4.c:966).  A match that runs off the end
 * of the history continues into the block (lz4.c:1141-1153), which the
 * contiguous window gives for free.
 *
 * The three python-lz4 callers:
 *   lz4.block.compress(dict=D), |D| >= 8   (_block.c:101-104 -> LZ4_loadDict,
 *     lz4.c:1541-1581, then usingExtDict): window = last min(|D|,64K) bytes
 *     of D + block, ibase = 65536 - hist, low_idx = ibase, low_src = hist,
 *     low_dict = 0;
 *   lz4.block.compress(dict=D), |D| < 8    (LZ4_loadDict keeps no dictionary,
 *     prefix mode with dictSmall): hist = 0, ibase = low_idx = 65536;
 *   linked frame blocks (lz4frame.c:865-871, prefix mode over the frame):
 *     window = frame start, hist = block offset, ibase = low_* = 0.
 */
int orc_compress_window(const uint8_t* w, int64_t hist, int n, uint8_t* dst, int cap, int accel,
                        uint32_t* table, uint32_t ibase, uint32_t low_idx, int64_t low_src,
                        int64_t low_dict)
{
    static const int kSkipTrigger = 6;
    const uint8_t* const src = w + hist;
    const uint8_t* const iend = src + n;
    const uint8_t* const mflimit1 = iend - ORC_MFLIMIT + 1;
    const uint8_t* const matchlimit = iend - ORC_LASTLITERALS;
    const uint8_t* anchor = src;
    const uint8_t* ip = src;
    uint8_t* op = dst;
    uint8_t* const olimit = dst + cap;
    const int limited = cap < orc_compress_bound(n);
    const uint32_t start_idx = ibase + (uint32_t)hist;
    uint32_t fwd_h;

    if ((unsigned)n > (unsigned)ORC_MAX_INPUT) return 0;
    if (accel < 1) accel = 1;
    if (accel > ORC_ACCEL_MAX) accel = ORC_ACCEL_MAX;
    if (n == 0) {
        if (limited && cap <= 0) return 0;
        dst[0] = 0;
        return 1;
    }
    if (n < ORC_MIN_LENGTH) goto last_literals;

    table[orc_hash(ip, ORC_TABLE_U32_HASH5)] = start_idx;          /* lz4.c:984 */
    ip++;
    fwd_h = orc_hash(ip, ORC_TABLE_U32_HASH5);

    for (;;) {
        const uint8_t* match;
        uint8_t* token;
        {
            const uint8_t* fwd = ip;
            int step = 1;
            int attempts = accel << kSkipTrigger;
            for (;;) {
                const uint32_t h = fwd_h;
                const uint32_t cur = ibase + (uint32_t)(fwd - w);
                const uint32_t cand = table[h];
                ip = fwd;
                fwd += step;
                step = attempts++ >> kSkipTrigger;
                if (fwd > mflimit1) goto last_literals;
                fwd_h = orc_hash(fwd, ORC_TABLE_U32_HASH5);
                table[h] = cur;
                if (cand < low_idx) continue;                      /* lz4.c:1061 */
                if (cand + ORC_DIST_MAX < cur) continue;           /* lz4.c:1062-1065 */
                match = w + (int64_t)(cand - ibase);
                if (orc_rd32(match) == orc_rd32(ip)) break;
            }
        }
        {   /* catch-up with the lowLimit of the match's segment */
            const uint8_t* const low = w + (match < src ? low_dict : low_src);
            while (ip > anchor && match > low && ip[-1] == match[-1]) { ip--; match--; }
        }
        {
            const unsigned lit = (unsigned)(ip - anchor);
            token = op++;
            if (limited && op + lit + (2 + 1 + ORC_LASTLITERALS) + lit / 255 > olimit) return 0;
            if (lit >= 15) { *token = 15 << 4; op = orc_put_len(op, lit - 15); }
            else *token = (uint8_t)(lit << 4);
            memcpy(op, anchor, lit);
            op += lit;
        }
next_match:
        {
            const unsigned off = (unsigned)(ip - match);
            unsigned mcode;
            op[0] = (uint8_t)off; op[1] = (uint8_t)(off >> 8); op += 2;
            mcode = orc_count(ip + ORC_MINMATCH, match + ORC_MINMATCH, matchlimit);
            ip += mcode + ORC_MINMATCH;
            if (limited && op + (1 + ORC_LASTLITERALS) + (mcode + 240) / 255 > olimit) return 0;
            if (mcode >= 15) { *token += 15; op = orc_put_len(op, mcode - 15); }
            else *token += (uint8_t)mcode;
        }
        anchor = ip;
        if (ip >= mflimit1) break;
        table[orc_hash(ip - 2, ORC_TABLE_U32_HASH5)] = ibase + (uint32_t)(ip - 2 - w);
        {
            const uint32_t h = orc_hash(ip, ORC_TABLE_U32_HASH5);
            const uint32_t cur = ibase + (uint32_t)(ip - w);
            const uint32_t cand = table[h];
            table[h] = cur;
            if (cand >= low_idx && cand + ORC_DIST_MAX >= cur) {
                match = w + (int64_t)(cand - ibase);
                if (orc_rd32(match) == orc_rd32(ip)) {
                    token = op++;
                    *token = 0;
                    goto next_match;
                }
            }
        }
        fwd_h = orc_hash(++ip, ORC_TABLE_U32_HASH5);
    }
last_literals:
    {
        const size_t run = (size_t)(iend - anchor);
        if (limited && op + run + 1 + (run + 255 - 15) / 255 > olimit) return 0;
        if (run >= 15) { *op++ = 15 << 4; op = orc_put_len(op, (unsigned)(run - 15)); }
        else *op++ = (uint8_t)(run << 4);
        memcpy(op, anchor, run);
        op += run;
    }
    (void)start_idx;
    return (int)(op - dst);
}

int orc_compress_dict_mode(const uint8_t* win, int64_t d_len, int n, uint8_t* dst, int cap, int accel, int prefix);

/* lz4.block.compress(source, dict=D) for a non-HC mode (_block.c:93-107):
 * LZ4_resetStream, LZ4_loadDict (lz4.c:1541-1581: last 64 KiB of D, every
 * third position hashed, indexes ending at 64 KiB), LZ4_compress_fast_continue.
 * `win` holds the last min(d_len, 65536) bytes of D followed by the source. */
int orc_compress_dict(const uint8_t* win, int64_t d_len, int n, uint8_t* dst, int cap, int accel)
{
    return orc_compress_dict_mode(win, d_len, n, dst, cap, accel, 0);
}

/* The same call when D's memory ends exactly where the source begins
 * (prefix = 1): LZ4_compress_fast_continue sees dictEnd == source and takes
 * prefix mode (lz4.c:1671-1676, withPrefix64k) instead of usingExtDict, so
 * backward catch-up of EVERY match may reach back to the dictionary's first
 * byte (lowLimit = source - dictSize, lz4.c:967) -- with extDict a match
 * inside the source stops at the source start (lz4.c:1052-1053).  Valid-area
 * (dictSmall: prefixIdxLimit = startIndex - dictSize, lz4.c:937/1061) and
 * distance rules are the same in both modes. */
int orc_compress_dict_mode(const uint8_t* win, int64_t d_len, int n, uint8_t* dst, int cap, int accel, int prefix)
{
    uint32_t table[4096];
    memset(table, 0, sizeof(table));
    if (d_len < 8)                                                 /* lz4.c:1564-1566 */
        return orc_compress_window(win, 0, n, dst, cap, accel, table, 65536, 65536, 0, 0);
    {
        const int64_t dt = d_len > 65536 ? 65536 : d_len;
        const uint32_t ibase = (uint32_t)(65536 - dt);
        int64_t p;
        for (p = 0; p <= dt - 8; p += 3)                           /* lz4.c:1575-1578 */
            table[orc_hash(win + p, ORC_TABLE_U32_HASH5)] = ibase + (uint32_t)p;
        return orc_compress_window(win, dt, n, dst, cap, accel, table, ibase, ibase, prefix ? 0 : dt, 0);
    }
}

/* The blocks of one linked frame (LZ4F_compressFrame with blockLinked,
 * lz4frame.c:865-871 + 960-1001): one stream, LZ4_compress_fast_continue per
 * block straight from the contiguous source, dstCapacity = blockSize - 1
 * (lz4frame.c:835).  out_len[k] = compressed size, 0 = stored raw.  The
 * 2 GB index renormalisation (LZ4_renormDictT, lz4.c:1612-1630) is restated
 * as a window shift; it never changes a parse. */
int orc_compress_linked(const uint8_t* src, int64_t n, int bsize, int accel, uint8_t* dst,
                        int64_t dst_stride, int32_t* out_len)
{
    uint32_t table[4096];
    const uint8_t* w = src;
    int64_t pos = 0, k = 0;
    uint32_t start = 0;
    memset(table, 0, sizeof(table));
    for (; pos < n; pos += bsize, ++k) {
        const int len = (int)(n - pos < bsize ? n - pos : bsize);
        if ((uint64_t)start + (uint64_t)len > 0x80000000ull) {
            const uint32_t delta = start - 65536;
            int i;
            for (i = 0; i < 4096; i++) table[i] = table[i] < delta ? 0 : table[i] - delta;
            w += delta;
            start = 65536;
        }
        out_len[k] = orc_compress_window(w, (int64_t)(src + pos - w), len, dst + k * dst_stride, len - 1,
                                         accel, table, 0, 0, 0, 0);
        start += (uint32_t)len;
    }
    return (int)k;
}

/* read_variable_length (lz4.c:1903-1928).  Returns 0 on success. */
static int orc_read_len(const uint8_t** ipp, const uint8_t* ilimit, int initial_check, size_t* out)
{
    const uint8_t* ip = *ipp;
    size_t len = 0;
    unsigned s;
    if (initial_check && ip >= ilimit) return -1;
    do {
        s = *ip++;
        len += s;
        if (ip > ilimit) { *ipp = ip; return -1; }
    } while (s == 255);
    *ipp = ip;
    *out = len;
    return 0;
}

/* Overlapping LZ77 copy with the reference semantics: dst[i] = dst[i - off];
 * a zero offset produces zero bytes (lz4.c:478-485, 2300-2307). */
static void orc_match_copy(uint8_t* op, size_t off, size_t len)
{
    size_t i;
    if (off == 0) { memset(op, 0, len); return; }
    for (i = 0; i < len; i++) op[i] = op[(ptrdiff_t)i - (ptrdiff_t)off];
}


/*
 * LZ4_decompress_safe (lz4.c:2344-2350 -> LZ4_decompress_generic 1936-2339,
 * decode_full_block).  Returns the decoded size, or -(ip - src) - 1 where ip
 * is the input position at which the input was rejected (lz4.c:2336-2337).
 *
 * dict/dict_len restate the usingExtDict variant that
 * LZ4_decompress_safe_usingDict (lz4.c:2612-2625) selects for a dictionary
 * held in a separate buffer (the `dict=` argument of lz4.block.decompress,
 * _block.c:357-359); dict_len 0 is the plain noDict path.
 *
 * The reference runs a "fast" sequence loop while at least 64 bytes of
 * output room remain (lz4.c:1990-2109) and leaves it for good the first time
 * a sequence needs the careful path (its `goto safe_literal_copy` /
 * `goto safe_match_copy`); the sticky `fast` flag below is that transition.
 */
int orc_decompress_dict(const uint8_t* src, uint8_t* dst, int src_size, int cap,
                        const uint8_t* dict, size_t dict_len)
{
    const uint8_t* ip = src;
    const uint8_t* const iend = src + src_size;
    uint8_t* op = dst;
    uint8_t* const oend = dst + cap;
    const int check_window = dict_len < 65536;                   /* lz4.c:1961 */
    const uint8_t* const dict_end = dict ? dict + dict_len : NULL;
    int fast;
    unsigned tok;
    size_t lit, ml, off, add;

    if (src == NULL || cap < 0) return -1;                       /* lz4.c:1950 */
    if (cap == 0) return (src_size == 1 && src[0] == 0) ? 0 : -1;  /* lz4.c:1978-1982 */
    if (src_size == 0) return -1;                                /* lz4.c:1983 */

    /* offset reaches before the dictionary / destination start */
#define OOW(o)    (check_window && (o) > (size_t)(op - dst) + dict_len)
#define INPFX(o)  ((o) <= (size_t)(op - dst))

    fast = (oend - op) >= 64;
    for (;;) {
        tok = *ip++;
        lit = tok >> 4;

        if (fast) {                                              /* lz4.c:1996-2109 */
            if (lit == 15) {
                if (orc_read_len(&ip, iend - 15, 1, &add)) goto fail;
                lit += add;
                if (op + lit > oend - 32 || ip + lit > iend - 32) { fast = 0; goto literal_tail; }
            } else if (ip > iend - 17) {
                fast = 0; goto literal_tail;
            }
            memcpy(op, ip, lit); ip += lit; op += lit;
            off = orc_rd16(ip); ip += 2;
            ml = tok & 15;
            if (ml == 15) {
                if (orc_read_len(&ip, iend - ORC_LASTLITERALS + 1, 0, &add)) goto fail;
                ml += add + ORC_MINMATCH;
                if (OOW(off)) goto fail;
                if (op + ml >= oend - 64) { fast = 0; goto match_tail; }
            } else {
                ml += ORC_MINMATCH;
                if (op + ml >= oend - 64) { fast = 0; goto match_tail; }
                if (off >= 8 && INPFX(off)) { orc_match_copy(op, off, ml); op += ml; continue; }
            }
            if (OOW(off)) goto fail;
            if (!INPFX(off)) {                                   /* match starts in the dictionary */
                if (op + ml > oend - ORC_LASTLITERALS) goto fail;
                goto dict_copy;
            }
            orc_match_copy(op, off, ml); op += ml;
            continue;
        }

        /* safe phase (lz4.c:2114-2329) */
        if (lit != 15 && ip < iend - 16 && op <= oend - 32) {   /* two-stage shortcut, lz4.c:2128-2158 */
            memcpy(op, ip, lit); op += lit; ip += lit;
            ml = tok & 15;
            off = orc_rd16(ip); ip += 2;
            if (ml != 15 && off >= 8 && INPFX(off)) {
                orc_match_copy(op, off, ml + ORC_MINMATCH);
                op += ml + ORC_MINMATCH;
                continue;
            }
            goto match_length;
        }
        if (lit == 15) {
            if (orc_read_len(&ip, iend - 15, 1, &add)) goto fail;
            lit += add;
        }
literal_tail:                                                    /* lz4.c:2172-2229 */
        if (op + lit > oend - ORC_MFLIMIT || ip + lit > iend - (2 + 1 + ORC_LASTLITERALS)) {
            if (ip + lit != iend || op + lit > oend) goto fail;  /* must be the last literals */
            memmove(op, ip, lit); ip += lit; op += lit;
            break;
        }
        memcpy(op, ip, lit); ip += lit; op += lit;
        off = orc_rd16(ip); ip += 2;
        ml = tok & 15;
match_length:                                                    /* lz4.c:2238-2245 */
        if (ml == 15) {
            if (orc_read_len(&ip, iend - ORC_LASTLITERALS + 1, 0, &add)) goto fail;
            ml += add;
        }
        ml += ORC_MINMATCH;
match_tail:                                                      /* lz4.c:2248-2328 */
        if (OOW(off)) goto fail;
        if (!INPFX(off)) {
            if (op + ml > oend - ORC_LASTLITERALS) goto fail;
            goto dict_copy;
        }
        if (op + ml > oend - ORC_LASTLITERALS) goto fail;        /* lz4.c:2315-2317 */
        orc_match_copy(op, off, ml); op += ml;
        continue;

dict_copy:                                                       /* lz4.c:2252-2277 */
        {
            const size_t in_dict = off - (size_t)(op - dst);
            if (ml <= in_dict) {
                memmove(op, dict_end - in_dict, ml); op += ml;
            } else {
                memcpy(op, dict_end - in_dict, in_dict); op += in_dict;
                orc_match_copy(op, (size_t)(op - dst), ml - in_dict);
                op += ml - in_dict;
            }
        }
    }
#undef OOW
#undef INPFX
    return (int)(op - dst);
fail:
    return (int)(-(ip - src)) - 1;
}

int orc_decompress_safe(const uint8_t* src, uint8_t* dst, int src_size, int cap)
{
    return orc_decompress_dict(src, dst, src_size, cap, NULL, 0);
}

/* ---------------- XXH32 (xxhash.c:263-554) ---------------- */
#define P1 2654435761u
#define P2 2246822519u
#define P3 3266489917u
#define P4 668265263u
#define P5 374761393u
static uint32_t orc_rotl(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }
static uint32_t orc_round(uint32_t acc, uint32_t in) { return orc_rotl(acc + in * P2, 13) * P1; }

/* tail + avalanche (xxhash.c:278-348) */
static uint32_t orc_xxh_finish(uint32_t h, const uint8_t* p, size_t len)
{
    while (len >= 4) { h = orc_rotl(h + orc_rd32(p) * P3, 17) * P4; p += 4; len -= 4; }
    while (len > 0) { h = orc_rotl(h + (*p++) * P5, 11) * P1; len--; }
    h ^= h >> 15; h *= P2; h ^= h >> 13; h *= P3; h ^= h >> 16;
    return h;
}

uint32_t orc_xxh32(const void* input, size_t len, uint32_t seed)   /* xxhash.c:351-416 */
{
    const uint8_t* p = (const uint8_t*)input;
    uint32_t h;
    if (len >= 16) {
        const uint8_t* const limit = p + len - 15;
        uint32_t v1 = seed + P1 + P2, v2 = seed + P2, v3 = seed, v4 = seed - P1;
        do {
            v1 = orc_round(v1, orc_rd32(p)); v2 = orc_round(v2, orc_rd32(p + 4));
            v3 = orc_round(v3, orc_rd32(p + 8)); v4 = orc_round(v4, orc_rd32(p + 12));
            p += 16;
        } while (p < limit);
        h = orc_rotl(v1, 1) + orc_rotl(v2, 7) + orc_rotl(v3, 12) + orc_rotl(v4, 18);
    } else {
        h = seed + P5;
    }
    h += (uint32_t)len;
    return orc_xxh_finish(h, p, len & 15);
}

/* streaming state (xxhash.h:264-274, xxhash.c:437-554) */
typedef struct { uint32_t total, large, v[4], mem[4], memsize; } orc_xxh32_state;

void orc_xxh32_reset(orc_xxh32_state* s, uint32_t seed)
{
    memset(s, 0, sizeof(*s));
    s->v[0] = seed + P1 + P2; s->v[1] = seed + P2; s->v[2] = seed; s->v[3] = seed - P1;
}

void orc_xxh32_update(orc_xxh32_state* s, const void* input, size_t len)
{
    const uint8_t* p = (const uint8_t*)input;
    const uint8_t* const end = p + len;
    s->total += (uint32_t)len;
    s->large |= (len >= 16) | (s->total >= 16);
    if (s->memsize + len < 16) {
        memcpy((uint8_t*)s->mem + s->memsize, p, len);
        s->memsize += (uint32_t)len;
        return;
    }
    if (s->memsize) {
        const size_t fill = 16 - s->memsize;
        memcpy((uint8_t*)s->mem + s->memsize, p, fill);
        for (int i = 0; i < 4; i++) s->v[i] = orc_round(s->v[i], s->mem[i]);
        p += fill;
        s->memsize = 0;
    }
    while (p + 16 <= end) {
        for (int i = 0; i < 4; i++) s->v[i] = orc_round(s->v[i], orc_rd32(p + 4 * i));
        p += 16;
    }
    if (p < end) { memcpy(s->mem, p, (size_t)(end - p)); s->memsize = (uint32_t)(end - p); }
}

uint32_t orc_xxh32_digest(const orc_xxh32_state* s)
{
    uint32_t h = s->large ? orc_rotl(s->v[0], 1) + orc_rotl(s->v[1], 7) + orc_rotl(s->v[2], 12) + orc_rotl(s->v[3], 18)
                          : s->v[2] + P5;
    h += s->total;
    return orc_xxh_finish(h, (const uint8_t*)s->mem, s->memsize);
}

size_t orc_xxh32_state_size(void) { return sizeof(orc_xxh32_state); }

/* Batch helpers used by the tests and by bench.py's cpu_baseline leg:
 * n blocks at byte offsets, one call, so the per-call FFI cost stays out. */
int orc_compress_batch(const uint8_t* src, const int64_t* src_off, const int32_t* src_len,
                       uint8_t* dst, const int64_t* dst_off, int32_t dst_cap,
                       int32_t* out_len, int64_t n, int variant, int accel)
{
    for (int64_t i = 0; i < n; i++)
        out_len[i] = orc_compress(src + src_off[i], src_len[i], dst + dst_off[i], dst_cap, variant, accel);
    return 0;
}

int orc_decompress_batch(const uint8_t* src, const int64_t* src_off, const int32_t* src_len,
                         uint8_t* dst, const int64_t* dst_off, const int32_t* dst_cap,
                         int32_t* status, int64_t n)
{
    for (int64_t i = 0; i < n; i++)
        status[i] = orc_decompress_safe(src + src_off[i], dst + dst_off[i], src_len[i], dst_cap[i]);
    return 0;
}
