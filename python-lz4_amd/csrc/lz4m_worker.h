// lz4m_worker.h -- internal interface of the single-call workers (not part of
// the C-ABI): the per-call record and the mailbox a persistent one-workgroup
// kernel polls, so that a lone lz4.block.compress / decompress call
// (/root/reference/lz4/block/_block.c:221-237, :355-361) costs no kernel
// launch while calls keep coming.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace lz4m {

// One call's record, in the thread's mapped pinned staging buffer (layout
// [input, up(len)] [record, kCallMeta] [output, cap]).
struct CallMeta {
    int64_t src_off, dst_off;
    int32_t src_len, dst_cap, result, done;   // done: set (system-scope release) when the output is in host memory
    uint64_t work[8];                         // decoder scratch (lz4m_decompress_workspace_bytes)
};
constexpr size_t kCallMeta = 256;
static_assert(sizeof(CallMeta) <= kCallMeta, "record size");

// A worker's mailbox (mapped pinned host memory, one per worker kind and host
// thread).  The host writes the request fields, then `seq` with a release; the
// worker's lane 0 polls `seq` (system-scope acquire), serves the request with
// the lone-block kernel's own body, then stores `served` before it polls again.  It exits on `quit`,
// after `idle` ticks of the 100 MHz real-time clock without a request, or, between requests, once
// it has run `life` ticks: a stream that shares its hardware queue waits at most that long even
// while calls keep coming (the host starts it again on the next call).
struct Mailbox {
    uint32_t seq;       // host: request number (never 0)
    uint32_t quit;      // host: 1 = exit now
    uint32_t served;    // worker: the last request number served
    int32_t accel;      // request (compress): acceleration
    int32_t rec_off;    // request: the record's offset in the staging buffer (rec_off..table: one 16-byte load)
    int32_t src_len;    // request: input bytes (at offset 0)
    int32_t dst_cap;    // request: output capacity
    int32_t table;      // request (compress): LZ4M_TABLE_*
    uint32_t pad[8];    // worker diagnostics: [0] requests served by this launch, [1] exit reason (1 idle, 2 quit, 3 lifetime)
};
static_assert(sizeof(Mailbox) == 64 && offsetof(Mailbox, rec_off) == 16, "mailbox layout");

// LZ4M_WORKER_TS (diagnostic builds only): lane 0 stamps the 100 MHz real-time
// clock at each stage of a lone-block call into the record's work[] words
// (bodies) and the mailbox's pad[2..3] (poll), for tools/probe_wts.py.
#ifdef LZ4M_WORKER_TS
#define LZ4M_WTS(ptr, i)                                                                                  \
    do {                                                                                                  \
        if (threadIdx.x == 0 && (ptr) != nullptr)                                                         \
            __hip_atomic_store((uint32_t*)(ptr) + (i), (uint32_t)__builtin_amdgcn_s_memrealtime(),         \
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);                              \
    } while (0)
#else
#define LZ4M_WTS(ptr, i) \
    do {                 \
    } while (0)
#endif

// the request a worker serves next, broadcast to the workgroup (lane 0 polls);
// 0 = exit.  Fields of the request land in cmd[1..5]; cmd[6] counts the
// requests served.  `last` is the request just served (0: none yet): once every
// thread is past it, lane 0 publishes it as `served` before polling again.
__device__ __forceinline__ uint32_t worker_next(Mailbox* mb, uint32_t& last, uint64_t idle, uint64_t birth, uint64_t life,
                                                uint32_t* cmd) {
    __syncthreads();   // every thread is past the previous request and its reads of cmd
    if (threadIdx.x == 0) {
        if (last != 0) {
            cmd[6] += 1;
            __hip_atomic_store(&mb->pad[0], cmd[6], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(&mb->served, last, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        uint32_t seq = 0, why = 0;
        for (;;) {
            seq = __hip_atomic_load(&mb->seq, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
            if (__hip_atomic_load(&mb->quit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0) {
                why = 2;
                break;
            }
            // lifetime over: exit even with a request pending (the host sees the
            // stream idle and starts a new launch, which serves it)
            if (__builtin_amdgcn_s_memrealtime() - birth > life) {
                why = 3;
                break;
            }
            if (seq != last) {
                LZ4M_WTS(&mb->pad[2], 0);
                break;
            }
            if (__builtin_amdgcn_s_memrealtime() - t0 > idle) {
                why = 1;
                break;
            }
            __builtin_amdgcn_s_sleep(8);
        }
        // the request's bytes and fields were written before seq: every later
        // load of the workgroup (after the barrier) reads this request's
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
        if (why != 0) __hip_atomic_store(&mb->pad[1], why, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        cmd[0] = why != 0 ? 0u : seq;
        // the five request fields in one PCIe round trip (two independent
        // loads after the fence; per-field atomic loads would wait one by one)
        typedef uint32_t u32x4m __attribute__((ext_vector_type(4)));
        const u32x4m f = *reinterpret_cast<const u32x4m*>(&mb->rec_off);   // rec_off, src_len, dst_cap, table
        const uint32_t acc = *reinterpret_cast<const uint32_t*>(&mb->accel);
        cmd[1] = f.x;
        cmd[2] = f.y;
        cmd[3] = f.z;
        cmd[4] = f.w;
        cmd[5] = acc;
        LZ4M_WTS(&mb->pad[3], 0);
    }
    __syncthreads();
    last = cmd[0];
    return last;
}

// a worker's first act: the served count starts at 0, `last` at the mailbox's
// served, `birth` (thread 0's) at the real-time clock
__device__ __forceinline__ uint32_t worker_init(Mailbox* mb, uint32_t* cmd, uint64_t& birth) {
    birth = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0) {
        cmd[6] = mb->served != 0 ? ~0u : 0u;   // the first publication re-stores the served number
        __hip_atomic_store(&mb->pad[1], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    return __hip_atomic_load(&mb->served, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

}  // namespace lz4m

extern "C" {
// launch the persistent worker of `kind` (0 = decompress, 1 = compress) on
// `stream`: mailbox mb, staging buffer hd (device views of mapped pinned
// memory), device output buffer dbuf; idle / lifetime limits in ticks of the
// 100 MHz real-time clock
int lz4m_worker_launch(int kind, lz4m::Mailbox* mb, uint8_t* hd, uint8_t* dbuf, uint64_t idle_ticks,
                       uint64_t life_ticks, hipStream_t stream);
int lz4m_compress_worker_launch(lz4m::Mailbox* mb, uint8_t* hd, uint8_t* dbuf, uint64_t idle_ticks,
                                uint64_t life_ticks, hipStream_t stream);
}
