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

struct Scratch {
    uint8_t* buf = nullptr;
    size_t cap = 0;
    hipStream_t stream = nullptr;
    ~Scratch() {
        if (buf) (void)hipFree(buf);
        if (stream) (void)hipStreamDestroy(stream);
    }
    // `bytes` of device memory (>= 256 B aligned pieces carved by the caller)
    uint8_t* get(size_t bytes) {
        if (stream == nullptr && hipStreamCreateWithFlags(&stream, hipStreamNonBlocking) != hipSuccess) return nullptr;
        if (bytes > cap) {
            if (buf) (void)hipFree(buf);
            buf = nullptr;
            cap = 0;
            const size_t want = bytes + bytes / 4 + 4096;
            if (hipMalloc(reinterpret_cast<void**>(&buf), want) != hipSuccess) return nullptr;
            cap = want;
        }
        return buf;
    }
};

thread_local Scratch t_scratch;

inline size_t up(size_t x) { return (x + 255) & ~(size_t)255; }

// one-block compress through lz4m_compress_batch; returns the compressed size or 0
int compress_one(const char* src, char* dst, int srcSize, int dstCapacity, int table, int acceleration) {
    if (srcSize < 0 || srcSize > kMaxInput || dstCapacity < 0 || (srcSize > 0 && !src) || (dstCapacity > 0 && !dst))
        return 0;
    const size_t need = up((size_t)srcSize + 16) + up((size_t)dstCapacity + 16) + 256;
    uint8_t* d = t_scratch.get(need);
    if (!d) return 0;
    uint8_t* d_src = d;
    uint8_t* d_dst = d + up((size_t)srcSize + 16);
    uint8_t* d_meta = d_dst + up((size_t)dstCapacity + 16);
    struct Meta {
        int64_t src_off, dst_off;
        int32_t src_len, dst_cap, out_len, pad;
    } m{0, 0, srcSize, dstCapacity, 0, 0};
    hipStream_t s = t_scratch.stream;
    if (srcSize && hipMemcpyAsync(d_src, src, (size_t)srcSize, hipMemcpyHostToDevice, s) != hipSuccess) return 0;
    if (hipMemcpyAsync(d_meta, &m, sizeof m, hipMemcpyHostToDevice, s) != hipSuccess) return 0;
    Meta* dm = reinterpret_cast<Meta*>(d_meta);
    if (lz4m_compress_batch(d_src, &dm->src_off, &dm->src_len, d_dst, &dm->dst_off, &dm->dst_cap, &dm->out_len, 1,
                            table, acceleration, reinterpret_cast<lz4m_stream_t>(s)) != 0)
        return 0;
    if (hipMemcpyAsync(&m, d_meta, sizeof m, hipMemcpyDeviceToHost, s) != hipSuccess) return 0;
    if (hipStreamSynchronize(s) != hipSuccess) return 0;
    if (m.out_len > 0 && hipMemcpy(dst, d_dst, (size_t)m.out_len, hipMemcpyDeviceToHost) != hipSuccess) return 0;
    return m.out_len;
}

}  // namespace

extern "C" int lz4m_decompress_safe(const char* src, char* dst, int compressedSize, int dstCapacity) {
    if (compressedSize < 0 || dstCapacity < 0) return -1;
    if ((compressedSize > 0 && !src) || (dstCapacity > 0 && !dst)) return -1;
    const size_t need = up((size_t)compressedSize + 16) + up((size_t)dstCapacity + 16) + 256;
    uint8_t* d = t_scratch.get(need);
    if (!d) return -1;
    uint8_t* d_src = d;
    uint8_t* d_dst = d + up((size_t)compressedSize + 16);
    uint8_t* d_meta = d_dst + up((size_t)dstCapacity + 16);
    struct Meta {
        int64_t src_off, dst_off;
        int32_t src_len, dst_cap, status, pad;
        uint64_t work[8];
    } m{0, 0, compressedSize, dstCapacity, -1, 0, {0, 0, 0, 0, 0, 0, 0, 0}};
    hipStream_t s = t_scratch.stream;
    if (compressedSize && hipMemcpyAsync(d_src, src, (size_t)compressedSize, hipMemcpyHostToDevice, s) != hipSuccess)
        return -1;
    if (hipMemcpyAsync(d_meta, &m, sizeof m, hipMemcpyHostToDevice, s) != hipSuccess) return -1;
    Meta* dm = reinterpret_cast<Meta*>(d_meta);
    if (lz4m_decompress_batch_ws(d_src, &dm->src_off, &dm->src_len, d_dst, &dm->dst_off, &dm->dst_cap, &dm->status, 1,
                                 dm->work, sizeof m.work, reinterpret_cast<lz4m_stream_t>(s)) != 0)
        return -1;
    if (hipMemcpyAsync(&m, d_meta, sizeof m, hipMemcpyDeviceToHost, s) != hipSuccess) return -1;
    if (hipStreamSynchronize(s) != hipSuccess) return -1;
    if (m.status > 0 && hipMemcpy(dst, d_dst, (size_t)m.status, hipMemcpyDeviceToHost) != hipSuccess) return -1;
    return m.status;
}

extern "C" int lz4m_compress_default(const char* src, char* dst, int srcSize, int dstCapacity) {
    return compress_one(src, dst, srcSize, dstCapacity, LZ4M_TABLE_AUTO, 1);
}

extern "C" int lz4m_compress_block_api(const char* src, char* dst, int srcSize, int dstCapacity, int acceleration) {
    return compress_one(src, dst, srcSize, dstCapacity, LZ4M_TABLE_U32_HASH5, acceleration);
}

extern "C" uint32_t lz4m_xxh32(const void* input, size_t length, uint32_t seed) {
    if (length > 0 && !input) return 0;
    uint8_t* d = t_scratch.get(up(length + 16) + 256);
    if (!d) return 0;
    uint32_t* d_out = reinterpret_cast<uint32_t*>(d + up(length + 16));
    hipStream_t s = t_scratch.stream;
    if (length && hipMemcpyAsync(d, input, length, hipMemcpyHostToDevice, s) != hipSuccess) return 0;
    if (lz4m_xxh32_long(d, (int64_t)length, seed, d_out, reinterpret_cast<lz4m_stream_t>(s)) != 0) return 0;
    uint32_t h = 0;
    if (hipMemcpyAsync(&h, d_out, sizeof h, hipMemcpyDeviceToHost, s) != hipSuccess) return 0;
    if (hipStreamSynchronize(s) != hipSuccess) return 0;
    return h;
}
