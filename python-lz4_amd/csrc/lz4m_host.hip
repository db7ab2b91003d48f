// lz4m_host.hip -- single-buffer, host-pointer entry points with the lz4.h
// contracts, for a C caller that replaces the
// reference's per-call lz4libs functions one for one (e.g. a rebuilt
// lz4/block/_block.c).  A block of up to 64 KiB is a request to the thread's
// persistent worker kernel (one_block_worker: a mailbox in coherent mapped
// memory), or with the worker off one launch of a lone-block kernel on mapped
// pinned memory (one_block_mapped).  Either reads the caller's bytes and the
// call record from a pinned staging buffer, stages the block in LDS, writes
// the result back itself and releases a done flag that the host polls
// (DESIGN.md section 3.3b).  Larger inputs copy to
// the device, run the batched kernel on a batch of one and copy the result
// back; device buffers are cached per thread and grow as needed.  Throughput
// comes from the batched entry points.
#include "../../include/lz4m.h"
#include "lz4m_worker.h"

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <atomic>
#include <chrono>

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

typedef lz4m::CallMeta CMeta;   // the call record (lz4m_worker.h), shared with the single-call workers
static_assert(sizeof(CMeta) <= kMeta && kMeta == lz4m::kCallMeta, "record size");

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
    const auto t0 = std::chrono::steady_clock::now();
    for (uint32_t i = 1; __atomic_load_n(&hm->done, __ATOMIC_ACQUIRE) == 0; ++i) {
        if ((i & 255) == 0) {
            const hipError_t q = hipStreamQuery(s);
            if (q == hipSuccess && __atomic_load_n(&hm->done, __ATOMIC_ACQUIRE) == 0) return fail;   // ended without the flag
            if (q != hipSuccess && q != hipErrorNotReady) return fail;
            // a lone block takes well under a millisecond: a kernel that has
            // not finished in 30 s is queued behind something that does not
            // end, and the call fails instead of waiting without bound
            if ((i & 0xFFFF) == 0 && std::chrono::steady_clock::now() - t0 > std::chrono::seconds(30)) return fail;
        }
        __builtin_ia32_pause();
    }
    memcpy(&m, h + in, sizeof m);
    t_out = h + in + kMeta;
    if (dst && m.result > 0 && m.result <= cap) memcpy(dst, h + in + kMeta, (size_t)m.result);
    return m.result;
}

// ---------------------------------------------------- single-call workers
// A lone call served by a persistent one-workgroup kernel that polls a
// mailbox in mapped pinned memory (lz4m_worker.h): while calls keep coming,
// none of them pays a kernel launch.  One worker per kind (decompress /
// compress) and host thread; it exits by itself after kIdle of no requests,
// after kLife in total (so a stream it shares a hardware queue with waits at
// most that long, whatever the call rate), on the host's quit, or when the
// thread ends.  A call whose worker has exited starts it again; calls outside
// its buffers take the launch-per-call path.
constexpr size_t kWorkIn = 66 * 1024;         // input region: the lone-block kernels' ranges
constexpr size_t kWorkOut = 1 << 20;          // output region: capacities up to 1 MiB
constexpr size_t kWorkMb = 128;               // two mailboxes
constexpr uint64_t kIdle = 200000;            // 2 ms of the 100 MHz real-time clock
constexpr uint64_t kLife = 200000;            // 2 ms: a launch's whole lifetime (r05f: 5 ms held a shared queue 5 ms)
constexpr int32_t kSoloStageFail = LZ4M_SOLO_STAGE_FAIL;   // lone-block compress: a staging wait gave up (lz4m_compress.hip)

std::atomic<int> g_worker_mode{-1};           // -1: from LZ4M_WORKER at first use
// every call the worker path took and then handed to the launch path: a
// worker that neither served nor exited within 1 s, a stream error, more than
// three restarts in one call, a failed (re)start, a lone-block staging wait
// that gave up.  Each one but the last also turns the worker path off for the
// process.  Tests assert it stays 0 (tests/conftest.py).
std::atomic<int> g_worker_failures{0};
void worker_failed(bool turn_off) {
    g_worker_failures.fetch_add(1, std::memory_order_relaxed);
    if (turn_off) g_worker_mode.store(0, std::memory_order_relaxed);
}
bool worker_enabled() {
    int m = g_worker_mode.load(std::memory_order_relaxed);
    if (m < 0) {
        const char* e = getenv("LZ4M_WORKER");
        m = (e != nullptr && e[0] == '0') ? 0 : 1;
        g_worker_mode.store(m, std::memory_order_relaxed);
    }
    return m != 0;
}

struct Workers {
    int dev = -1;
    uint8_t* host = nullptr;       // [mailbox 0 | mailbox 1] then the data regions (coherent)
    uint8_t* host_dev = nullptr;
    uint8_t* data = nullptr;       // = host + kWorkMb: per kind [input kWorkIn] [record kMeta] [output kWorkOut]
    uint8_t* data_dev = nullptr;
    uint8_t* dbuf = nullptr;       // device output buffers, one per kind
    hipStream_t stream[2] = {nullptr, nullptr};
    bool launched[2] = {false, false};
    uint32_t seq[2] = {0, 0};
    lz4m::Mailbox* mb(int k) { return reinterpret_cast<lz4m::Mailbox*>(host + 64 * k); }
    static constexpr size_t kRegion = kWorkIn + kMeta + kWorkOut + 256;
    size_t region(int k) const { return (size_t)k * kRegion; }
    uint8_t* base(int k) { return data + region(k); }
    bool idle(int k) { return hipStreamQuery(stream[k]) == hipSuccess; }
    // Tell worker k to quit and wait (<= 2 s) until its stream is idle.
    // Returns false if it is still queued or running: its mailbox keeps
    // quit = 1 and the caller abandons this whole set (abandon()), so a late
    // worker exits without touching a live request.
    bool stop(int k) {
        if (!launched[k]) return true;
        __atomic_store_n(&mb(k)->quit, 1u, __ATOMIC_RELEASE);
        const auto t0 = std::chrono::steady_clock::now();
        hipError_t q;
        while ((q = hipStreamQuery(stream[k])) == hipErrorNotReady &&
               std::chrono::steady_clock::now() - t0 < std::chrono::seconds(2))
            __builtin_ia32_pause();
        if (q == hipErrorNotReady) return false;
        launched[k] = false;
        __atomic_store_n(&mb(k)->quit, 0u, __ATOMIC_RELEASE);
        return true;
    }
    // Drop this set of mailboxes, staging regions, device buffers and streams
    // without freeing them (a worker that did not stop may still read and
    // write them); the next get() allocates a fresh set.
    void abandon() {
        host = host_dev = dbuf = data = data_dev = nullptr;
        stream[0] = stream[1] = nullptr;
        launched[0] = launched[1] = false;
        seq[0] = seq[1] = 0;
        dev = -1;
    }
    // stop both workers; abandon the set if either did not stop
    bool stop_all() {
        const bool a = stop(0), b = stop(1);
        if (!(a && b)) abandon();
        return a && b;
    }
    void release() {
        if (!stop_all()) return;   // abandoned: nothing of it may be freed
        for (int k = 0; k < 2; ++k)
            if (stream[k]) (void)hipStreamDestroy(stream[k]);
        if (dbuf) (void)hipFree(dbuf);
        if (host) (void)hipHostFree(host);
        host = host_dev = dbuf = data = data_dev = nullptr;
        stream[0] = stream[1] = nullptr;
    }
    ~Workers() { release(); }
    bool get() {
        int d = 0;
        if (hipGetDevice(&d) != hipSuccess) return false;
        if (d != dev) {
            release();
            dev = d;
        }
        if (host) return true;
        // coherent (fine-grained): the worker polls the mailboxes and reads
        // each request's bytes while it runs, with no kernel boundary to
        // invalidate a cached copy (request bytes in non-coherent, L2-cached
        // memory measured no faster: DESIGN.md 3.3b)
        if (hipHostMalloc(reinterpret_cast<void**>(&host), kWorkMb + 2 * kRegion,
                          hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess)
            return false;
        memset(host, 0, kWorkMb);
        data = host + kWorkMb;
        if (hipHostGetDevicePointer(reinterpret_cast<void**>(&host_dev), host, 0) != hipSuccess ||
            hipHostGetDevicePointer(reinterpret_cast<void**>(&data_dev), data, 0) != hipSuccess ||
            hipMalloc(reinterpret_cast<void**>(&dbuf), 2 * (kWorkOut + 256)) != hipSuccess) {
            release();
            return false;
        }
        for (int k = 0; k < 2; ++k)
            if (hipStreamCreateWithFlags(&stream[k], hipStreamNonBlocking) != hipSuccess) {
                release();
                return false;
            }
        return true;
    }
    bool start(int k) {
        if (launched[k] && idle(k)) launched[k] = false;   // exited (idle or quit)
        if (launched[k]) return true;
        __atomic_store_n(&mb(k)->quit, 0u, __ATOMIC_RELEASE);
        if (lz4m_worker_launch(k, reinterpret_cast<lz4m::Mailbox*>(host_dev + 64 * k), data_dev + region(k),
                               dbuf + (size_t)k * (kWorkOut + 256), kIdle, kLife, stream[k]) != 0)
            return false;
        launched[k] = true;
        return true;
    }
};
thread_local Workers t_workers;

// One block through the thread's worker of `kind` (0 decompress, 1 compress).
// Returns false (nothing done) when the worker path does not apply.
bool one_block_worker(int kind, const char* src, int32_t len, char* dst, int32_t cap, int32_t fail, int table,
                      int accel, int32_t* result) {
    if (!worker_enabled()) return false;
    const size_t in = up((size_t)len + 16);
    const int32_t out_cap = kind == 1 ? lz4m_compress_bound(len) : cap;
    if (in > kWorkIn || out_cap > (int32_t)kWorkOut || len < 0) return false;
    Workers& W = t_workers;
    if (!W.get()) {
        worker_failed(true);
        return false;
    }
    uint8_t* h = W.base(kind);
    if (len) memcpy(h, src, (size_t)len);
    CMeta m{};
    m.src_off = 0;
    m.dst_off = 0;   // output at the device buffer's start
    m.src_len = len;
    m.dst_cap = cap;
    m.result = fail;
    memcpy(h + in, &m, sizeof m);
    lz4m::Mailbox* M = W.mb(kind);
    M->rec_off = (int32_t)in;
    M->src_len = len;
    M->dst_cap = cap;
    M->table = table;
    M->accel = accel;
    if (!W.start(kind)) {
        worker_failed(true);
        return false;
    }
    if (++W.seq[kind] == 0) W.seq[kind] = 1;
    __atomic_store_n(&M->seq, W.seq[kind], __ATOMIC_RELEASE);
    CMeta* hm = reinterpret_cast<CMeta*>(h + in);
    int restarts = 0;
    const auto t0 = std::chrono::steady_clock::now();
    // every 256 polls: has the worker exited without serving (it went idle or
    // reached its lifetime as the request arrived)?  Then start it again; it
    // serves the request.  A worker that neither serves nor exits within a
    // second is stopped and the worker path is turned off for the process
    // (the launch path then serves every call): a call never waits on it
    // without bound.  Every hand-over to the launch path is counted.
    for (uint32_t i = 1; __atomic_load_n(&hm->done, __ATOMIC_ACQUIRE) == 0; ++i) {
        if ((i & 255) == 0) {
            const hipError_t q = hipStreamQuery(W.stream[kind]);
            if (__atomic_load_n(&hm->done, __ATOMIC_ACQUIRE) != 0) break;
            if (q != hipSuccess && q != hipErrorNotReady) {   // the stream failed: this set is unusable
                worker_failed(true);
                W.abandon();
                return false;
            }
            if (q == hipSuccess) {
                if (++restarts > 3) {
                    worker_failed(true);
                    return false;
                }
                W.launched[kind] = false;
                if (!W.start(kind)) {
                    worker_failed(true);
                    return false;
                }
            } else if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(1)) {
                worker_failed(true);
                W.stop_all();
                return false;
            }
        }
        __builtin_ia32_pause();
    }
    memcpy(&m, h + in, sizeof m);
    if (kind == 1 && m.result == kSoloStageFail) {   // the block never reached LDS: redo it by launch
        worker_failed(false);
        return false;
    }
    t_out = h + in + kMeta;
    if (dst && m.result > 0 && m.result <= cap) memcpy(dst, h + in + kMeta, (size_t)m.result);
    *result = m.result;
    return true;
}

// one-block compress through the batched compressors; returns the compressed size or 0
// dst == nullptr: the output stays in the pinned buffer (t_out), for the _staged calls
int compress_one(const char* src, char* dst, int srcSize, int dstCapacity, int table, int acceleration) {
    if (srcSize < 0 || srcSize > kMaxInput || dstCapacity < 0 || (srcSize > 0 && !src)) return 0;
    // blocks below 65547 bytes: the LDS-staged lone-block kernel (the
    // skip-ahead search then waits on no memory round trip), no copies
    if (srcSize < kSoloLimit) {
        int32_t rw = 0;
        if (one_block_worker(1, src, srcSize, dst, dstCapacity, 0, table, acceleration, &rw)) return rw > 0 ? rw : 0;
        const int32_t r = one_block_mapped(
            src, srcSize, dst, dstCapacity, 0, [&](uint8_t* hd, CMeta* hm, uint8_t* d, uint8_t* hout, hipStream_t s) {
                return lz4m_compress_solo(hd, srcSize, d, dstCapacity, &hm->result, table, acceleration, hout,
                                          &hm->done, reinterpret_cast<lz4m_stream_t>(s));
            });
        if (r != kSoloStageFail) return r > 0 ? r : 0;
        worker_failed(false);   // staging gave up on the launch path too: the batched kernel below
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
    int32_t rw = 0;
    if (compressedSize <= kSoloDecIn && one_block_worker(0, src, compressedSize, dst, dstCapacity, -1, 0, 1, &rw))
        return rw;
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

// diagnostics (tests, probes): out[0..7] = this thread's decompress / compress
// mailbox seq, served, quit, and the launched flags; out[8..11] = per kind the
// requests its last launch served and how that launch ended (1 idle, 2 quit);
// out[12..15] = per kind the poll's two real-time stamps (LZ4M_WORKER_TS
// builds); returns the failure count
extern "C" int lz4m_single_call_worker_state(uint32_t* out) {
    Workers& W = t_workers;
    for (int k = 0; k < 2; ++k) {
        lz4m::Mailbox* M = W.host ? W.mb(k) : nullptr;
        out[3 * k] = M ? __atomic_load_n(&M->seq, __ATOMIC_ACQUIRE) : 0u;
        out[3 * k + 1] = M ? __atomic_load_n(&M->served, __ATOMIC_ACQUIRE) : 0u;
        out[3 * k + 2] = M ? __atomic_load_n(&M->quit, __ATOMIC_ACQUIRE) : 0u;
        out[8 + 2 * k] = M ? __atomic_load_n(&M->pad[0], __ATOMIC_ACQUIRE) : 0u;
        out[9 + 2 * k] = M ? __atomic_load_n(&M->pad[1], __ATOMIC_ACQUIRE) : 0u;
        out[12 + 2 * k] = M ? __atomic_load_n(&M->pad[2], __ATOMIC_ACQUIRE) : 0u;   // LZ4M_WORKER_TS builds
        out[13 + 2 * k] = M ? __atomic_load_n(&M->pad[3], __ATOMIC_ACQUIRE) : 0u;
    }
    out[6] = W.launched[0];
    out[7] = W.launched[1];
    return g_worker_failures.load(std::memory_order_relaxed);
}

extern "C" int lz4m_single_call_worker(int mode) {
    const int prev = worker_enabled() ? 1 : 0;
    if (mode == 0 || mode == 1) {
        g_worker_mode.store(mode, std::memory_order_relaxed);
        if (mode == 0) t_workers.stop_all();   // this thread's workers stop now (other threads' go idle by themselves)
    }
    return prev;
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
