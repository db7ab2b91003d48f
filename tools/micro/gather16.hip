// Microbenchmark (dev only): random 16-byte reads from a large buffer --
// plain hipMalloc vs uncached vs fine-grained allocations.  Each lane reads
// R random 16-B pieces inside its own 64 KiB region (like a decoder lane
// reading match sources from its own block's output) and XORs them.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int ILP>
__global__ __launch_bounds__(256) void k(const uint8_t* __restrict__ buf, int64_t nreg, int reads, uint32_t* out) {
    const int64_t g = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const uint8_t* base = buf + (g % nreg) * 65536;
    uint32_t x = (uint32_t)g * 2654435761u, acc = 0;
    for (int r = 0; r < reads; r += ILP) {
        u32x4 v[ILP];
#pragma unroll
        for (int i = 0; i < ILP; ++i) {
            x = x * 1664525u + 1013904223u;
            __builtin_memcpy(&v[i], base + ((x >> 8) & 0xFFF0u), 16);
        }
#pragma unroll
        for (int i = 0; i < ILP; ++i) acc ^= v[i].x ^ v[i].w;
    }
    if (acc == 0x12345678u) out[0] = acc;
}

template <int ILP> void run(const char* name, uint8_t* d, int64_t nreg, uint32_t* o) {
    const int reads = 256;
    const int grid = 256 * 8;   // 8 WG/CU x 256 CUs
    hipEvent_t a, b; (void)hipEventCreate(&a); (void)hipEventCreate(&b);
    hipLaunchKernelGGL(k<ILP>, dim3(grid), dim3(256), 0, 0, d, nreg, reads, o);
    (void)hipEventRecord(a);
    hipLaunchKernelGGL(k<ILP>, dim3(grid), dim3(256), 0, 0, d, nreg, reads, o);
    (void)hipEventRecord(b); (void)hipEventSynchronize(b);
    float ms; (void)hipEventElapsedTime(&ms, a, b);
    const double n = (double)grid * 256 * reads;
    printf("%-12s ILP %d: %.3f G reads/s  (%.1f GB/s useful 16B, %.1f GB/s if 128B lines)\n", name, ILP,
           n / ms / 1e6, n * 16 / ms / 1e6, n * 128 / ms / 1e6);
}
int main() {
    const int64_t nreg = 262144;   // 16 GiB
    const size_t sz = (size_t)nreg * 65536;
    uint32_t* o; (void)hipMalloc(&o, 64);
    uint8_t* d;
    (void)hipMalloc(&d, sz); (void)hipMemset(d, 1, sz);
    run<1>("plain", d, nreg, o); run<4>("plain", d, nreg, o);
    (void)hipFree(d);
    if (hipExtMallocWithFlags((void**)&d, sz, hipDeviceMallocUncached) == hipSuccess) {
        (void)hipMemset(d, 1, sz);
        run<1>("uncached", d, nreg, o); run<4>("uncached", d, nreg, o);
        (void)hipFree(d);
    } else printf("uncached alloc failed\n");
    if (hipExtMallocWithFlags((void**)&d, sz, hipDeviceMallocFinegrained) == hipSuccess) {
        (void)hipMemset(d, 1, sz);
        run<1>("finegrained", d, nreg, o); run<4>("finegrained", d, nreg, o);
        (void)hipFree(d);
    } else printf("finegrained alloc failed\n");
    return 0;
}
