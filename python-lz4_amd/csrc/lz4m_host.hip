// lz4m_host.hip -- single-buffer, host-pointer entry points with the lz4.h
// contracts, for a C caller that replaces the
// reference's per-call lz4libs functions one for one (e.g. a rebuilt
// lz4/block/_block.c).  A block of up to 64 KiB is one launch of a lone-block
// kernel on mapped pinned memory (one_block_mapped: the kernel reads the
// caller's bytes and the call record from the thread's pinned staging buffer,
// stages the block in LDS, writes the result back itself and releases a done
// flag that the host polls).  Larger inputs copy to
// the device, run the batched kernel on a batch of one and copy the result
// back; device buffers are cached per thread and grow as needed.  Throughput
// comes from the batched entry points.
#include "../../include/lz4m.h"

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

namespace {

constexpr int kMaxInput = 0x7E000000;   // LZ4_MAX_INPUT_SIZE, lz4.h:211
constexpr size_t kMeta = 256;           // per-call record (offsets, sizes, result, decoder scratch)
constexpr int kSoloLimit = 65536 + 11;  // LZ4_64Klimit (lz4.c:689): lz4m_compress_solo's range
constexpr int kSoloDecIn = 66 * 1024 - 64;   // lz4m_decompress_solo's input range

// Per-thread device buffer, pinned host staging buffer and stream, for the
// device that is current when the call is made.  A call is then one
// host-to-device copy of [input | record], the launch, one device-to-host
// copy of [record | output] and one synchronisation.
struct Scratch {
    int dev = -1;
    uint8_t* buf = nullptr;
    uint8_t* host = nullptr;
    uint8_t* host_dev = nullptr;   // the device's address of `host` (mapped pinned memory)
    size_t cap = 0;
    hipStream_t stream = nullptr;
    void release() {
        if (buf) (void)hipFree(buf);
        if (host) (void)hipHostFree(host);
        if (stream) (void)hipStreamDestroy(stream);
        buf = host = host_dev = nullptr;
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
            buf = host = host_dev = nullptr;
            cap = 0;
            const size_t want = bytes + bytes / 4 + 4096;
            if (hipMalloc(reinterpret_cast<void**>(&buf), want) != hipSuccess) return false;
            if (hipHostMalloc(reinterpret_cast<void**>(&host), want, hipHostMallocDefault) != hipSuccess) return false;
            if (hipHostGetDevicePointer(reinterpret_cast<void**>(&host_dev), host, 0) != hipSuccess) return false;
            cap = want;
        }
        return true;
    }
};

thread_local Scratch t_scratch;
thread_local const uint8_t* t_out = nullptr;   // the last call's output in the pinned buffer (the _staged calls)

inline size_t up(size_t x) { return (x + 255) & ~(size_t)255; }

struct CMeta {
    int64_t src_off, dst_off;
    int32_t src_len, dst_cap, result, done;   // done: set by a lone-block kernel when its output is in host memory
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
    t_out = h + in + kMeta;
    if (dst && m.result > 0 && m.result <= cap) memcpy(dst, h + in + kMeta, (size_t)m.result);
    return m.result;
}

// One block through a lone-block kernel (lz4m_compress_solo /
// lz4m_decompress_solo) that reads its input and record straight from the
// mapped pinned staging buffer and writes its result and output back into it:
// no copies on the stream, one launch and one synchronisation per call (the
// copies of one_block cost ~10 us each in launch gaps at 64 KiB).  Layout of
// the pinned buffer as in one_block; the device buffer holds the output.
template <typename Launch>
int32_t one_block_mapped(const char* src, int32_t len, char* dst, int32_t cap, int32_t fail, Launch launch) {
    const size_t in = up((size_t)len + 16);
    if (!t_scratch.get(in + kMeta + (size_t)cap + 16)) return fail;
    uint8_t* h = t_scratch.host;
    uint8_t* hd = t_scratch.host_dev;
    if (len) memcpy(h, src, (size_t)len);
    CMeta m{};
    m.src_off = 0;
    m.dst_off = 0;   // output at the device buffer's start
    m.src_len = len;
    m.dst_cap = cap;
    m.result = fail;
    memcpy(h + in, &m, sizeof m);
    hipStream_t s = t_scratch.stream;
    CMeta* hm = reinterpret_cast<CMeta*>(h + in);
    if (launch(hd, reinterpret_cast<CMeta*>(hd + in), t_scratch.buf, hd + in + kMeta, s) != 0) return fail;
    // the kernel's last act is a system-scope release of `done` after its
    // output: poll it (the completion signal and the waiting thread's wake-up
    // cost ~10 us more); every 256 polls check the stream, so a failed launch
    // ends the wait
    for (uint32_t i = 1; __atomic_load_n(&hm->done, __ATOMIC_ACQUIRE) == 0; ++i) {
        if ((i & 255) == 0) {
            const hipError_t q = hipStreamQuery(s);
            if (q == hipSuccess && __atomic_load_n(&hm->done, __ATOMIC_ACQUIRE) == 0) return fail;   // ended without the flag
            if (q != hipSuccess && q != hipErrorNotReady) return fail;
        }
        __builtin_ia32_pause();
    }
    memcpy(&m, h + in, sizeof m);
    t_out = h + in + kMeta;
    if (dst && m.result > 0 && m.result <= cap) memcpy(dst, h + in + kMeta, (size_t)m.result);
    return m.result;
}

// one-block compress through the batched compressors; returns the compressed size or 0
// dst == nullptr: the output stays in the pinned buffer (t_out), for the _staged calls
int compress_one(const char* src, char* dst, int srcSize, int dstCapacity, int table, int acceleration) {
    if (srcSize < 0 || srcSize > kMaxInput || dstCapacity < 0 || (srcSize > 0 && !src)) return 0;
    // blocks below 65547 bytes: the LDS-staged lone-block kernel (the
    // skip-ahead search then waits on no memory round trip), no copies
    if (srcSize < kSoloLimit) {
        const int32_t r = one_block_mapped(
            src, srcSize, dst, dstCapacity, 0, [&](uint8_t* hd, CMeta* hm, uint8_t* d, uint8_t* hout, hipStream_t s) {
                return lz4m_compress_solo(hd, srcSize, d, dstCapacity, &hm->result, table, acceleration, hout,
                                          &hm->done, reinterpret_cast<lz4m_stream_t>(s));
            });
        return r > 0 ? r : 0;
    }
    const int32_t r = one_block(src, srcSize, dst, dstCapacity, 0, [&](uint8_t* d, CMeta* dm, hipStream_t s) {
        return lz4m_compress_batch(d, &dm->src_off, &dm->src_len, d, &dm->dst_off, &dm->dst_cap, &dm->result, 1,
                                   table, acceleration, reinterpret_cast<lz4m_stream_t>(s));
    });
    return r > 0 ? r : 0;
}

// dst == nullptr: the output stays in the pinned buffer (t_out), for the _staged calls
int decompress_one(const char* src, char* dst, int compressedSize, int dstCapacity) {
    // inputs up to 66 KiB - 64 (any 64 KiB block): the LDS-staged lone-block
    // decoder, no copies
    if (compressedSize <= kSoloDecIn)
        return one_block_mapped(src, compressedSize, dst, dstCapacity, -1,
                                [&](uint8_t* hd, CMeta* hm, uint8_t* d, uint8_t* hout, hipStream_t s) {
                                    return lz4m_decompress_solo(hd, &hm->src_off, &hm->src_len, d, &hm->dst_off,
                                                                &hm->dst_cap, &hm->result, compressedSize, hout,
                                                                &hm->done, reinterpret_cast<lz4m_stream_t>(s));
                                });
    return one_block(src, compressedSize, dst, dstCapacity, -1, [&](uint8_t* d, CMeta* dm, hipStream_t s) {
        return lz4m_decompress_batch_ws(d, &dm->src_off, &dm->src_len, d, &dm->dst_off, &dm->dst_cap, &dm->result, 1,
                                        dm->work, sizeof dm->work, reinterpret_cast<lz4m_stream_t>(s));
    });
}

}  // namespace

extern "C" int lz4m_decompress_safe(const char* src, char* dst, int compressedSize, int dstCapacity) {
    if (compressedSize < 0 || dstCapacity < 0) return -1;
    if ((compressedSize > 0 && !src) || (dstCapacity > 0 && !dst)) return -1;
    return decompress_one(src, dst, compressedSize, dstCapacity);
}

extern "C" int lz4m_decompress_safe_staged(const char* src, int compressedSize, int dstCapacity, const char** out) {
    if (compressedSize < 0 || dstCapacity < 0 || !out || (compressedSize > 0 && !src)) return -1;
    const int r = decompress_one(src, nullptr, compressedSize, dstCapacity);
    *out = reinterpret_cast<const char*>(t_out);
    return r;
}

extern "C" int lz4m_compress_default(const char* src, char* dst, int srcSize, int dstCapacity) {
    if (dstCapacity > 0 && !dst) return 0;
    return compress_one(src, dst, srcSize, dstCapacity, LZ4M_TABLE_AUTO, 1);
}

extern "C" int lz4m_compress_block_api(const char* src, char* dst, int srcSize, int dstCapacity, int acceleration) {
    if (dstCapacity > 0 && !dst) return 0;
    return compress_one(src, dst, srcSize, dstCapacity, LZ4M_TABLE_U32_HASH5, acceleration);
}

extern "C" int lz4m_compress_block_api_staged(const char* src, int srcSize, int dstCapacity, int acceleration,
                                              int header, const char** out) {
    if (!out || (header != 0 && header != 4)) return 0;
    const int r = compress_one(src, nullptr, srcSize, dstCapacity, LZ4M_TABLE_U32_HASH5, acceleration);
    if (r > 0 && header) {   // the LE32 size just before the output, in the call record's slack (kMeta)
        uint8_t* p = const_cast<uint8_t*>(t_out) - 4;
        for (int k = 0; k < 4; ++k) p[k] = (uint8_t)((uint32_t)srcSize >> (8 * k));
    }
    *out = reinterpret_cast<const char*>(t_out) - header;
    return r;
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
