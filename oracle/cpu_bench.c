/*
 * oracle/cpu_bench.c -- host-core throughput harness for bench.py's
 * cpu_baseline leg (TEST/BENCH INFRASTRUCTURE ONLY, never part of the
 * shipped package).
 *
 * Built twice by oracle/Makefile:
 *   oracle/_ref/libref_bench.so   linked with the reference lz4libs compiled
 *                                 from /root/reference (cpu_baseline.kind
 *                                 "reference");
 *   oracle/build/liboracle_bench.so linked with the restatement in
 *                                 lz4_oracle.c ("port"), used when the
 *                                 reference build is absent.
 * One contiguous slice of blocks per pthread; returns wall seconds.
 */
#include <pthread.h>
#include <stdint.h>
#include <stddef.h>
#include <time.h>

#ifdef CPU_BENCH_REF
int LZ4_compress_default(const char* src, char* dst, int srcSize, int dstCapacity);
int LZ4_decompress_safe(const char* src, char* dst, int compressedSize, int dstCapacity);
unsigned int XXH32(const void* input, size_t length, unsigned int seed);
#define DO_COMPRESS(s, d, n, c)   LZ4_compress_default((const char*)(s), (char*)(d), (n), (c))
#define DO_DECOMPRESS(s, d, n, c) LZ4_decompress_safe((const char*)(s), (char*)(d), (n), (c))
#define DO_XXH32(p, n)            XXH32((p), (n), 0)
#else
int orc_compress_default(const uint8_t* src, uint8_t* dst, int n, int cap);
int orc_decompress_safe(const uint8_t* src, uint8_t* dst, int src_size, int cap);
uint32_t orc_xxh32(const void* input, size_t len, uint32_t seed);
#define DO_COMPRESS(s, d, n, c)   orc_compress_default((s), (d), (n), (c))
#define DO_DECOMPRESS(s, d, n, c) orc_decompress_safe((s), (d), (n), (c))
#define DO_XXH32(p, n)            orc_xxh32((p), (n), 0)
#endif

typedef struct {
    int op;                       /* 0 compress, 1 decompress, 2 xxh32 */
    const uint8_t* src; const int64_t* src_off; const int32_t* src_len;
    uint8_t* dst; const int64_t* dst_off; const int32_t* dst_cap;
    int32_t* out; int64_t lo, hi; int reps;
} job_t;

static void* worker(void* arg)
{
    job_t* j = (job_t*)arg;
    for (int r = 0; r < j->reps; r++) {
        for (int64_t i = j->lo; i < j->hi; i++) {
            const uint8_t* s = j->src + j->src_off[i];
            if (j->op == 0)
                j->out[i] = DO_COMPRESS(s, j->dst + j->dst_off[i], j->src_len[i], j->dst_cap[i]);
            else if (j->op == 1)
                j->out[i] = DO_DECOMPRESS(s, j->dst + j->dst_off[i], j->src_len[i], j->dst_cap[i]);
            else
                j->out[i] = (int32_t)DO_XXH32(s, (size_t)j->src_len[i]);
        }
    }
    return NULL;
}

double cpu_bench_run(int op, int threads, int reps,
                     const uint8_t* src, const int64_t* src_off, const int32_t* src_len,
                     uint8_t* dst, const int64_t* dst_off, const int32_t* dst_cap,
                     int32_t* out, int64_t n)
{
    pthread_t tid[256];
    job_t jobs[256];
    struct timespec t0, t1;
    if (threads < 1) threads = 1;
    if (threads > 256) threads = 256;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    for (int t = 0; t < threads; t++) {
        jobs[t] = (job_t){op, src, src_off, src_len, dst, dst_off, dst_cap, out,
                          n * t / threads, n * (t + 1) / threads, reps};
        pthread_create(&tid[t], NULL, worker, &jobs[t]);
    }
    for (int t = 0; t < threads; t++) pthread_join(tid[t], NULL);
    clock_gettime(CLOCK_MONOTONIC, &t1);
    return (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
}
