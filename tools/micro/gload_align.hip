// Microbenchmark (dev only): cost of 16-byte global loads (global_load_dwordx4)
// by byte alignment on gfx950 -- the row executor reads its inputs and far
// match sources 16 bytes at arbitrary offsets.  Every lane of 16 waves per CU
// issues ITER loads at  base + stride * lane + MIS  (+ a rotating offset that
// keeps the working set in L2, or spreads it over a 1 GiB buffer for HBM);
// the loads are independent (8 in flight per lane).  Prints ns per
// wave-instruction for each alignment.  Build: hipcc --offload-arch=gfx950 -O3
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
constexpr int ITER = 2048;

__global__ __launch_bounds__(256) void k(const uint8_t* __restrict__ buf, uint64_t span, uint32_t stride,
                                         uint32_t mis, uint32_t* out) {
    const uint32_t lane = threadIdx.x & 63, w = blockIdx.x * 4 + (threadIdx.x >> 6);
    uint32_t acc = 0;
    const uint64_t wbase = ((uint64_t)w * 4096u) % span;
    for (int it = 0; it < ITER; it += 8) {
        u32x4 v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const uint64_t a = (wbase + (uint64_t)(it + u) * 8192u + (uint64_t)stride * lane) % span + mis;
            __builtin_memcpy(&v[u], buf + a, 16);
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) acc += v[u].x ^ v[u].w;
    }
    if (acc == 0x12345678u) out[0] = acc;
}

int main() {
    const uint64_t spans[2] = {2ull << 20, 1ull << 30};   // L2-resident (per XCD), HBM
    uint8_t* buf;
    uint32_t* out;
    hipMalloc(&buf, (1ull << 30) + 4096);
    hipMalloc(&out, 64);
    hipMemset(buf, 1, (1ull << 30) + 4096);
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    const int grid = cus * 4;   // 16 waves per CU
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const uint32_t strides[2] = {16, 128};   // consecutive 16-byte pieces / one line per lane
    for (uint64_t span : spans)
        for (uint32_t stride : strides)
            for (uint32_t mis : {0u, 1u, 4u, 8u, 15u, 120u}) {
                hipLaunchKernelGGL(k, dim3(grid), dim3(256), 0, 0, buf, span, stride, mis, out);
                hipEventRecord(a);
                for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k, dim3(grid), dim3(256), 0, 0, buf, span, stride, mis, out);
                hipEventRecord(b);
                hipEventSynchronize(b);
                float ms = 0;
                hipEventElapsedTime(&ms, a, b);
                const double insts = 5.0 * grid * 4 * ITER;   // wave-instructions
                printf("span %5llu MiB stride %3u mis %3u: %.3f ms, %.2f ns per wave-load chip-wide, %.1f GB/s requested\n",
                       (unsigned long long)(span >> 20), stride, mis, ms / 5, ms * 1e6 / insts,
                       insts * 64 * 16 / (ms * 1e-3) / 1e9);
            }
    return 0;
}
