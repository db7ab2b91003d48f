/*
 * lz4m_host_copy.c -- multi-threaded host memcpy with an optional streaming
 * XXH32 of the source in one more thread (plain C99 + pthreads, no HIP).
 *
 * The drop-in frame calls (lz4.frame.compress / decompress on Python bytes,
 * _frame.c:226-228, :1058-1063) move their data through pinned staging
 * buffers: the caller's bytes into a pinned chunk before each host-to-device
 * copy, each device-to-host chunk into the result bytes object.  One core
 * copies ~8-10 GB/s, so an 8 GiB frame spends seconds in memcpy alone; the
 * copy is split over a few threads, and the frame's content checksum
 * (lz4frame.c:1850, one serial XXH32 stream) is hashed from the same chunk
 * while it is copied, instead of in a second pass over the result.
 */
#include "../../include/lz4m.h"

#include <pthread.h>
#include <string.h>

typedef struct {
    uint8_t* dst;
    const uint8_t* src;
    size_t n;
} CopyJob;

typedef struct {
    lz4m_xxh32_state* st;
    const uint8_t* src;
    size_t n;
} HashJob;

static void* copy_run(void* p) {
    const CopyJob* j = (const CopyJob*)p;
    if (j->n) memcpy(j->dst, j->src, j->n);
    return NULL;
}

static void* hash_run(void* p) {
    const HashJob* j = (const HashJob*)p;
    lz4m_xxh32_host_update(j->st, j->src, j->n);
    return NULL;
}

void lz4m_host_copy(void* dst, const void* src, size_t n, int threads, lz4m_xxh32_state* hash) {
    enum { kMaxThreads = 16 };
    if (threads < 1) threads = 1;
    if (threads > kMaxThreads) threads = kMaxThreads;
    if (n < ((size_t)1 << 22)) threads = 1;   /* below 4 MiB a thread costs more than it copies */
    pthread_t tid[kMaxThreads + 1];
    CopyJob cj[kMaxThreads];
    HashJob hj;
    int started[kMaxThreads + 1];
    const size_t part = ((n / (size_t)threads) + 63) & ~(size_t)63;
    for (int t = 0; t < threads; ++t) {
        const size_t lo = (size_t)t * part < n ? (size_t)t * part : n;
        const size_t hi = lo + part < n ? lo + part : n;
        cj[t].dst = (uint8_t*)dst + lo;
        cj[t].src = (const uint8_t*)src + lo;
        cj[t].n = hi - lo;
        started[t] = 0;
    }
    started[threads] = 0;
    if (hash) {   /* the hash reads the source concurrently with the copies */
        hj.st = hash;
        hj.src = (const uint8_t*)src;
        hj.n = n;
        started[threads] = pthread_create(&tid[threads], NULL, hash_run, &hj) == 0;
        if (!started[threads]) hash_run(&hj);
    }
    for (int t = 1; t < threads; ++t) {
        started[t] = pthread_create(&tid[t], NULL, copy_run, &cj[t]) == 0;
        if (!started[t]) copy_run(&cj[t]);
    }
    copy_run(&cj[0]);
    for (int t = 1; t <= threads; ++t)
        if (started[t]) pthread_join(tid[t], NULL);
}
