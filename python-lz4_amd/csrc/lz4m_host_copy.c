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
 *
 * The threads are a persistent pool (created on first use, again in a forked
 * child): an 8 GiB frame is 128 calls of 64 MiB, and creating 16 threads per
 * call cost ~0.5 ms each time.  Calls from several host threads take turns.
 * (A process that forks while one of its threads is inside a call leaves the
 * child with that call's lock taken: fork between calls.)
 */
#define _POSIX_C_SOURCE 200809L
#include "../../include/lz4m.h"

#include <pthread.h>
#include <string.h>
#include <unistd.h>

enum { kMaxThreads = 16 };

typedef struct {
    uint8_t* dst;
    const uint8_t* src;
    size_t n;
    lz4m_xxh32_state* st; /* not NULL: hash src[0, n) into st instead of copying */
    /* a list copy (lz4m_host_copy_many) when dsts != NULL: items [i0, i1) */
    void* const* dsts;
    const void* const* srcs;
    const size_t* lens;
    size_t i0, i1;
} Job;

static void run_job(const Job* j) {
    if (j->dsts != NULL) {
        for (size_t i = j->i0; i < j->i1; ++i)
            if (j->lens[i]) memcpy(j->dsts[i], j->srcs[i], j->lens[i]);
    } else if (j->st != NULL) {
        lz4m_xxh32_host_update(j->st, j->src, j->n);
    } else if (j->n) {
        memcpy(j->dst, j->src, j->n);
    }
}

/* worker w (0 .. kMaxThreads - 1) runs jobs[w] of each generation it sees
 * with active[w] set */
static struct {
    pthread_mutex_t mu;
    pthread_cond_t go, done;
    pthread_mutex_t call; /* one call at a time */
    unsigned long gen;
    unsigned long base;   /* gen when the workers were started: a worker that starts late must not skip the first post */
    int pending;
    int started;          /* workers running */
    pid_t pid;            /* the process that started them */
    Job jobs[kMaxThreads];
    int active[kMaxThreads];
} P = {PTHREAD_MUTEX_INITIALIZER, PTHREAD_COND_INITIALIZER, PTHREAD_COND_INITIALIZER, PTHREAD_MUTEX_INITIALIZER,
       0, 0, 0, 0, 0, {{0}}, {0}};

static void* worker(void* arg) {
    const int w = (int)(size_t)arg;
    unsigned long seen = 0;
    pthread_mutex_lock(&P.mu);
    seen = P.base;
    for (;;) {
        while (P.gen == seen) pthread_cond_wait(&P.go, &P.mu);
        seen = P.gen;
        if (!P.active[w]) continue;
        const Job j = P.jobs[w];
        pthread_mutex_unlock(&P.mu);
        run_job(&j);
        pthread_mutex_lock(&P.mu);
        if (--P.pending == 0) pthread_cond_signal(&P.done);
    }
    return NULL;
}

/* start the pool (again after a fork: the child has none of the threads);
 * returns the number of workers running.  Called with P.call held. */
static int pool(void) {
    const pid_t me = getpid();
    if (P.started > 0 && P.pid == me) return P.started;
    if (P.started > 0 && P.pid != me) { /* a forked child: fresh synchronisation objects, no workers */
        pthread_mutex_init(&P.mu, NULL);
        pthread_cond_init(&P.go, NULL);
        pthread_cond_init(&P.done, NULL);
        P.gen = 0;
        P.pending = 0;
        P.started = 0;
    }
    P.pid = me;
    pthread_mutex_lock(&P.mu);
    P.base = P.gen;
    pthread_mutex_unlock(&P.mu);
    while (P.started < kMaxThreads) {
        pthread_t t;
        pthread_attr_t a;
        pthread_attr_init(&a);
        pthread_attr_setdetachstate(&a, PTHREAD_CREATE_DETACHED);
        const int ok = pthread_create(&t, &a, worker, (void*)(size_t)P.started) == 0;
        pthread_attr_destroy(&a);
        if (!ok) break;
        ++P.started;
    }
    return P.started;
}

static void run_jobs(const Job* jobs, int njobs);

void lz4m_host_copy(void* dst, const void* src, size_t n, int threads, lz4m_xxh32_state* hash) {
    if (threads < 1) threads = 1;
    if (threads > kMaxThreads) threads = kMaxThreads;
    if (n < ((size_t)1 << 22)) threads = 1; /* below 4 MiB a thread costs more than it copies */
    Job jobs[kMaxThreads + 1];
    /* ceil(n / threads) rounded up to 64 bytes: the parts cover all of n
     * (rounding n / threads down lost up to threads - 1 tail bytes) */
    const size_t part = ((n + (size_t)threads - 1) / (size_t)threads + 63) & ~(size_t)63;
    for (int t = 0; t < threads; ++t) {
        const size_t lo = (size_t)t * part < n ? (size_t)t * part : n;
        const size_t hi = lo + part < n ? lo + part : n;
        jobs[t].dst = (uint8_t*)dst + lo;
        jobs[t].src = (const uint8_t*)src + lo;
        jobs[t].n = hi - lo;
        jobs[t].st = NULL;
        jobs[t].dsts = NULL;
    }
    int njobs = threads; /* jobs[0] runs on the caller */
    if (hash) {          /* the hash reads the source concurrently with the copies */
        jobs[njobs].dst = NULL;
        jobs[njobs].src = (const uint8_t*)src;
        jobs[njobs].n = n;
        jobs[njobs].st = hash;
        jobs[njobs].dsts = NULL;
        ++njobs;
    }
    run_jobs(jobs, njobs);
}

/* jobs[0] on the caller, the others on the pool's workers */
static void run_jobs(const Job* jobs, int njobs) {
    if (njobs == 1) {
        run_job(&jobs[0]);
        return;
    }
    pthread_mutex_lock(&P.call);
    const int workers = pool();
    pthread_mutex_lock(&P.mu);
    int posted = 0;
    for (int w = 0; w < kMaxThreads; ++w) P.active[w] = 0;
    for (int k = 1; k < njobs && posted < workers; ++k, ++posted) {
        P.jobs[posted] = jobs[k];
        P.active[posted] = 1;
    }
    P.pending = posted;
    ++P.gen;
    pthread_cond_broadcast(&P.go);
    pthread_mutex_unlock(&P.mu);
    run_job(&jobs[0]);
    for (int k = 1 + posted; k < njobs; ++k) run_job(&jobs[k]); /* no worker for it (thread creation failed) */
    pthread_mutex_lock(&P.mu);
    while (P.pending > 0) pthread_cond_wait(&P.done, &P.mu);
    pthread_mutex_unlock(&P.mu);
    pthread_mutex_unlock(&P.call);
}

void lz4m_host_copy_many(void* const* dst, const void* const* src, const size_t* n, size_t count, int threads) {
    if (count == 0) return;
    size_t total = 0;
    for (size_t i = 0; i < count; ++i) total += n[i];
    if (threads < 1) threads = 1;
    if (threads > kMaxThreads) threads = kMaxThreads;
    if (total < ((size_t)1 << 22)) threads = 1; /* below 4 MiB a thread costs more than it copies */
    if ((size_t)threads > count) threads = (int)count;
    Job jobs[kMaxThreads];
    /* contiguous item ranges of about total / threads bytes each */
    size_t i = 0, acc = 0;
    for (int t = 0; t < threads; ++t) {
        const size_t goal = total / (size_t)threads * (size_t)(t + 1);
        const size_t i0 = i;
        while (i < count && (acc < goal || t == threads - 1)) acc += n[i++];
        jobs[t].dst = NULL;
        jobs[t].src = NULL;
        jobs[t].n = 0;
        jobs[t].st = NULL;
        jobs[t].dsts = dst;
        jobs[t].srcs = src;
        jobs[t].lens = n;
        jobs[t].i0 = i0;
        jobs[t].i1 = i;
    }
    run_jobs(jobs, threads);
}
