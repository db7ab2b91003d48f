// lz4m_host.hip -- single-buffer, host-pointer entry points with the lz4.h
// contracts, for a C caller that replaces the
// reference's per-call lz4libs functions one for one (e.g. a rebuilt
// lz4/block/_block.c).  Each call copies its input to the device, runs the
// batched kernel on a batch of one, and copies the result back; device
// buffers are cached per thread and grow as needed.  These are convenience
// wrappers: throughput comes from the batched entry points, a single
// 64 KiB block is latency-bound on one lane.
#include "../../include/lz4m.h"

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

namespace {

constexpr int kMaxInput = 0x7E000000;   // LZ4_MAX_INPUT_SIZE, lz4.h:211
constexpr size_t kMeta = 256;           // per-call record (offsets, sizes, result, decoder scratch)

// Per-thread device buffer, pinned host staging buffer and stream, for the
// device that is current when the call is made.  A call is then one
// host-to-device copy of [input | record], the launch, one device-to-host
// copy of [record | output] and one synchronisation.
struct Scratch {
    int dev = -1;
    uint8_t* buf = nullptr;
    uint8_t* host = nullptr;
    size_t cap = 0;
    hipStream_t stream = nullptr;
    void release() {
        if (buf) (void)hipFree(buf);
        if (host) (void)hipHostFree(host);
        if (stream) (void)hipStreamDestroy(stream);
        buf = host = nullptr;
        stream = nullptr;
        cap = 0;
    }
    ~Scratch() { release(); }
    bool get(size_t bytes) {
        int d = 0;
        if (hipGetDevice(&d) != hipSuccess) return false;
        if (d != dev) {
            release();
            dev = d;
        }
        if (stream == nullptr && hipStreamCreateWithFlags(&stream, hipStreamNonBlocking) != hipSuccess) return false;
        if (bytes > cap) {
            if (buf) (void)hipFree(buf);
            if (host) (void)hipHostFree(host);
            buf = host = nullptr;
            cap = 0;
            const size_t want = bytes + bytes / 4 + 4096;
            if (hipMalloc(reinterpret_cast<void**>(&buf), want) != hipSuccess) return false;
            if (hipHostMalloc(reinterpret_cast<void**>(&host), want, hipHostMallocDefault) != hipSuccess) return false;
            cap = want;
        }
        return true;
    }
};

thread_local Scratch t_scratch;

inline size_t up(size_t x) { return (x + 255) & ~(size_t)255; }

struct CMeta {
    int64_t src_off, dst_off;
    int32_t src_len, dst_cap, result, pad;
    uint64_t work[8];   // decoder scratch (lz4m_decompress_workspace_bytes)
};
static_assert(sizeof(CMeta) <= kMeta, "record size");

// One block through a batched entry point.  Layout (device and pinned host
// alike): [input, up(len)] [record, kMeta] [output, cap]; copies in the first
// two parts, runs `launch` on the record, copies back the last two.  Returns
// the record's result (-1 if a HIP call failed; `fail` is returned then).
template <typename Launch>
int32_t one_block(const char* src, int32_t len, char* dst, int32_t cap, int32_t fail, Launch launch) {
    const size_t in = up((size_t)len + 16);
    if (!t_scratch.get(in + kMeta + (size_t)cap + 16)) return fail;
    uint8_t* h = t_scratch.host;
    uint8_t* d = t_scratch.buf;
    if (len) memcpy(h, src, (size_t)len);
    CMeta m{};
    m.src_off = 0;
    m.dst_off = (int64_t)(in + kMeta);
    m.src_len = len;
    m.dst_cap = cap;
    m.result = fail;
    memcpy(h + in, &m, sizeof m);
    hipStream_t s = t_scratch.stream;
    if (hipMemcpyAsync(d, h, in + kMeta, hipMemcpyHostToDevice, s) != hipSuccess) return fail;
    CMeta* dm = reinterpret_cast<CMeta*>(d + in);
    if (launch(d, dm, s) != 0) return fail;
    // the output comes back in full (its size is known only on the device)
    if (hipMemcpyAsync(h + in, d + in, kMeta + (size_t)cap, hipMemcpyDeviceToHost, s) != hipSuccess) return fail;
    if (hipStreamSynchronize(s) != hipSuccess) return fail;
    memcpy(&m, h + in, sizeof m);
    if (m.result > 0 && m.result <= cap) memcpy(dst, h + in + kMeta, (size_t)m.result);
    return m.result;
}

// one-block compress through the batched compressors; returns the compressed size or 0
int compress_one(const char* src, char* dst, int srcSize, int dstCapacity, int table, int acceleration) {
    if (srcSize < 0 || srcSize > kMaxInput || dstCapacity < 0 || (srcSize > 0 && !src) || (dstCapacity > 0 && !dst))
        return 0;
    const int32_t r = one_block(src, srcSize, dst, dstCapacity, 0, [&](uint8_t* d, CMeta* dm, hipStream_t s) {
        return lz4m_compress_batch(d, &dm->src_off, &dm->src_len, d, &dm->dst_off, &dm->dst_cap, &dm->result, 1,
                                   table, acceleration, reinterpret_cast<lz4m_stream_t>(s));
    });
    return r > 0 ? r : 0;
}

}  // namespace

extern "C" int lz4m_decompress_safe(const char* src, char* dst, int compressedSize, int dstCapacity) {
    if (compressedSize < 0 || dstCapacity < 0) return -1;
    if ((compressedSize > 0 && !src) || (dstCapacity > 0 && !dst)) return -1;
    return one_block(src, compressedSize, dst, dstCapacity, -1, [&](uint8_t* d, CMeta* dm, hipStream_t s) {
        return lz4m_decompress_batch_ws(d, &dm->src_off, &dm->src_len, d, &dm->dst_off, &dm->dst_cap, &dm->result, 1,
                                        dm->work, sizeof dm->work, reinterpret_cast<lz4m_stream_t>(s));
    });
}

extern "C" int lz4m_compress_default(const char* src, char* dst, int srcSize, int dstCapacity) {
    return compress_one(src, dst, srcSize, dstCapacity, LZ4M_TABLE_AUTO, 1);
}

extern "C" int lz4m_compress_block_api(const char* src, char* dst, int srcSize, int dstCapacity, int acceleration) {
    return compress_one(src, dst, srcSize, dstCapacity, LZ4M_TABLE_U32_HASH5, acceleration);
}

extern "C" uint32_t lz4m_xxh32(const void* input, size_t length, uint32_t seed) {
    if (length > 0 && !input) return 0;
    if (!t_scratch.get(up(length + 16) + 256)) return 0;
    uint8_t* d = t_scratch.buf;
    uint32_t* d_out = reinterpret_cast<uint32_t*>(d + up(length + 16));
    hipStream_t s = t_scratch.stream;
    if (length && hipMemcpyAsync(d, input, length, hipMemcpyHostToDevice, s) != hipSuccess) return 0;
    if (lz4m_xxh32_long(d, (int64_t)length, seed, d_out, reinterpret_cast<lz4m_stream_t>(s)) != 0) return 0;
    uint32_t h = 0;
    if (hipMemcpyAsync(&h, d_out, sizeof h, hipMemcpyDeviceToHost, s) != hipSuccess) return 0;
    if (hipStreamSynchronize(s) != hipSuccess) return 0;
    return h;
}
// ---------------------------------------------------------------- host XXH32
// The frame content checksum (lz4frame.c:1041-1042, :1170-1176) is one XXH32
// stream over all uncompressed bytes: four accumulators, each a serial
// multiply-rotate recurrence with no associative combine, so
// the GPU cannot split it (one wavefront runs it at 1.7 GB/s).  It runs here,
// on a host core, beside the device work: the XXH32 specification
// (xxhash.c:263-286 primes/round/avalanche, :290-348 tail, :437-554 the
// streaming state; state layout xxhash.h:264-274, total length mod 2^32).
namespace {
constexpr uint32_t kP1 = 0x9E3779B1u, kP2 = 0x85EBCA77u, kP3 = 0xC2B2AE3Du, kP4 = 0x27D4EB2Fu, kP5 = 0x165667B1u;
inline uint32_t rotl32(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }
inline uint32_t rd32(const uint8_t* p) {
    uint32_t v;
    memcpy(&v, p, 4);
    return v;
}
inline uint32_t xround(uint32_t acc, uint32_t in) { return rotl32(acc + in * kP2, 13) * kP1; }
// 16-byte stripes [p, p + len & ~15) into the four accumulators
inline const uint8_t* stripes(uint32_t* v, const uint8_t* p, size_t len) {
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
}  // namespace

extern "C" void lz4m_xxh32_host_reset(lz4m_xxh32_state* st, uint32_t seed) {
    memset(st, 0, sizeof *st);
    st->v[0] = seed + kP1 + kP2;
    st->v[1] = seed + kP2;
    st->v[2] = seed;
    st->v[3] = seed - kP1;
}

extern "C" void lz4m_xxh32_host_update(lz4m_xxh32_state* st, const void* input, size_t len) {
    if (len == 0 || input == nullptr) return;
    const uint8_t* p = static_cast<const uint8_t*>(input);
    st->total_len_32 += (uint32_t)len;
    st->large_len |= (uint32_t)((len >= 16) | (st->total_len_32 >= 16));
    uint8_t* mem = reinterpret_cast<uint8_t*>(st->mem32);
    if (st->memsize + len < 16) {   // not a whole stripe yet: buffer it
        memcpy(mem + st->memsize, p, len);
        st->memsize += (uint32_t)len;
        return;
    }
    if (st->memsize) {   // complete the buffered stripe
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

extern "C" uint32_t lz4m_xxh32_host_digest(const lz4m_xxh32_state* st) {
    uint32_t h = st->large_len ? rotl32(st->v[0], 1) + rotl32(st->v[1], 7) + rotl32(st->v[2], 12) + rotl32(st->v[3], 18)
                               : st->v[2] /* the seed */ + kP5;
    h += st->total_len_32;
    const uint8_t* p = reinterpret_cast<const uint8_t*>(st->mem32);
    size_t n = st->memsize;
    for (; n >= 4; n -= 4, p += 4) h = rotl32(h + rd32(p) * kP3, 17) * kP4;
    for (; n > 0; --n, ++p) h = rotl32(h + (*p) * kP5, 11) * kP1;
    h ^= h >> 15;
    h *= kP2;
    h ^= h >> 13;
    h *= kP3;
    h ^= h >> 16;
    return h;
}

extern "C" uint32_t lz4m_xxh32_host(const void* input, size_t len, uint32_t seed) {
    lz4m_xxh32_state st;
    lz4m_xxh32_host_reset(&st, seed);
    lz4m_xxh32_host_update(&st, input, len);
    return lz4m_xxh32_host_digest(&st);
}
