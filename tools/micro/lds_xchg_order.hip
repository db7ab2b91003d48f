// Microbenchmark / probe (dev only): in what order does one ds_wrxchg_rtn_b32
// instruction apply the lanes of a wave that hit the same LDS address?  The
// exact compressor's search step needs, per hash bucket, the serial insert
// order (lane 0 first).  Each lane exchanges its lane id + 1 into bucket
// h(lane) (random groups, seeded); the returned values then form, per
// bucket, a chain.  Counts the instructions whose chains are in increasing
// lane order (every lane got the nearest lower lane of its bucket, or the
// initial 0), and the ones that are not.
//   hipcc --offload-arch=gfx950 -O3 tools/micro/lds_xchg_order.hip -o tools/micro/lds_xchg_order.bin
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

template <bool HALF>
__global__ __launch_bounds__(256) void k(uint32_t seed, int buckets, unsigned long long* res) {
    __shared__ uint32_t tab[4][256];
    const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
    unsigned long long good = 0, bad = 0;
    for (int it = 0; it < 256; ++it) {
        for (int i = (int)lane; i < 256; i += 64) tab[w][i] = 0;
        __builtin_amdgcn_s_waitcnt(0xc07f);
        uint32_t x = (seed + 7919u * (uint32_t)it + 104729u * (blockIdx.x * 4u + w)) * 2654435761u ^ (lane * 40503u);
        x ^= x >> 13;
        x *= 0x5bd1e995u;
        x ^= x >> 15;
        const uint32_t h = x % (uint32_t)buckets;
        uint32_t prev = 0;
        if (HALF) {   // 16-bit entries: a masked OR with return on the enclosing dword
            uint16_t* t16 = (uint16_t*)&tab[w][0];
            const uint32_t a = (uint32_t)(uintptr_t)(t16 + h) & ~3u, sh = (h & 1u) * 16u;
            uint32_t old = 0;
            asm volatile("ds_mskor_rtn_b32 %0, %1, %2, %3\n s_waitcnt lgkmcnt(0)" : "=v"(old) : "v"(a), "v"(0xFFFFu << sh), "v"((lane + 1u) << sh) : "memory");
            prev = (old >> sh) & 0xFFFFu;
        } else {
            uint32_t* p = &tab[w][h];
            asm volatile("ds_wrxchg_rtn_b32 %0, %1, %2\n s_waitcnt lgkmcnt(0)" : "=v"(prev) : "v"((uint32_t)(uintptr_t)p), "v"(lane + 1u) : "memory");
        }
        // expected: the nearest lower lane with the same bucket (+1), else 0
        uint32_t exp = 0;
        for (int l = 0; l < 64; ++l) {   // uniform trip count: every lane active in the shuffle
            const uint32_t hl = __shfl(h, l);
            if (l < (int)lane && hl == h) exp = (uint32_t)l + 1u;
        }
        const bool ok = prev == exp;
        const uint64_t m = __ballot(!ok);
        if (lane == 0) {
            if (m) ++bad;
            else ++good;
        }
    }
    if (lane == 0) {
        atomicAdd(&res[0], good);
        atomicAdd(&res[1], bad);
    }
}

int main() {
    unsigned long long* d;
    hipMalloc(&d, 16);
    for (int half = 0; half < 2; ++half)
        for (int buckets : {1, 2, 4, 8, 16, 32, 64, 256}) {
            hipMemset(d, 0, 16);
            if (half) k<true><<<2048, 256>>>(12345u + (uint32_t)buckets, buckets, d);
            else k<false><<<2048, 256>>>(12345u + (uint32_t)buckets, buckets, d);
            unsigned long long h[2];
            hipMemcpy(h, d, 16, hipMemcpyDeviceToHost);
            printf("%s buckets %3d: in lane order %llu, not %llu\n", half ? "mskor_rtn b16" : "wrxchg_rtn b32", buckets, h[0], h[1]);
        }
    hipFree(d);
    return 0;
}
