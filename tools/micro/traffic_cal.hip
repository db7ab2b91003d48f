// Calibration of the rocprofv3 HBM traffic counters (dev only, not part of
// the library): kernels whose HBM bytes are known, in the access shapes the
// decoder uses, so that FETCH_SIZE / WRITE_SIZE / TCC_EA0_{RD,WR}REQ_* can be
// converted to bytes (tools/pmc_cal.sh, tools/pmc_cal_report.py).
//
//   copy16       coalesced streaming copy, 16 B per lane: reads N, writes N
//   lane_write   every lane writes its own 64 KiB region 16 B at a time
//                (the lane-per-block finisher's output shape): writes N
//   row_write    16-lane rows, each row writes its own 64 KiB region 256 B
//                per instruction (the row decoder's flush shape): writes N
//   lane_read    every lane reads its own 64 KiB region, 8 x 16 B = one
//                128-B line per iteration (no line is fetched twice): reads N
//   rand_read    every lane reads R random 16-B pieces of its own 64 KiB
//                region (the far match sources' shape); bytes NOT known --
//                reported as lines touched for comparison only
//
// Buffers are 4 GiB (16x the 256 MiB Infinity Cache) and written once before
// the timed kernels, so every read misses the on-die caches.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
constexpr int64_t kRegion = 65536;

__global__ __launch_bounds__(256) void fill(u32x4* p, int64_t n16) {
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += (int64_t)gridDim.x * 256)
        p[i] = u32x4{(uint32_t)i, (uint32_t)(i >> 7), 0x9E3779B9u ^ (uint32_t)i, 7u};
}

__global__ __launch_bounds__(256) void copy16(const u32x4* __restrict__ a, u32x4* __restrict__ b, int64_t n16) {
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += (int64_t)gridDim.x * 256) b[i] = a[i];
}

// lane g owns region g (lanes of a wave write 64 different regions)
__global__ __launch_bounds__(64) void lane_write(uint8_t* __restrict__ b, int64_t regions) {
    const int64_t g = (int64_t)blockIdx.x * 64 + threadIdx.x;
    if (g >= regions) return;
    u32x4* p = reinterpret_cast<u32x4*>(b + g * kRegion);
    for (int i = 0; i < (int)(kRegion / 16); ++i) p[i] = u32x4{(uint32_t)g, (uint32_t)i, 1u, 2u};
}

// row r (16 lanes) owns region r; one instruction writes 256 contiguous bytes
__global__ __launch_bounds__(64) void row_write(uint8_t* __restrict__ b, int64_t regions) {
    const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 4);
    const int j = threadIdx.x & 15;
    if (r >= regions) return;
    u32x4* p = reinterpret_cast<u32x4*>(b + r * kRegion);
    for (int i = j; i < (int)(kRegion / 16); i += 16) p[i] = u32x4{(uint32_t)r, (uint32_t)i, 3u, 4u};
}

__global__ __launch_bounds__(64) void lane_read(const uint8_t* __restrict__ b, int64_t regions, uint32_t* out) {
    const int64_t g = (int64_t)blockIdx.x * 64 + threadIdx.x;
    if (g >= regions) return;
    const u32x4* p = reinterpret_cast<const u32x4*>(b + g * kRegion);
    uint32_t acc = 0;
    for (int i = 0; i < (int)(kRegion / 16); i += 8) {
        u32x4 v[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = p[i + k];
#pragma unroll
        for (int k = 0; k < 8; ++k) acc ^= v[k].x ^ v[k].w;
    }
    if (acc == 0x12345678u) out[0] = acc;
}

__global__ __launch_bounds__(64) void rand_read(const uint8_t* __restrict__ b, int64_t regions, int reads,
                                                uint32_t* out) {
    const int64_t g = (int64_t)blockIdx.x * 64 + threadIdx.x;
    if (g >= regions) return;
    const uint8_t* base = b + g * kRegion;
    uint32_t x = (uint32_t)g * 2654435761u, acc = 0;
    for (int r = 0; r < reads; r += 4) {
        u32x4 v[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            x = x * 1664525u + 1013904223u;
            __builtin_memcpy(&v[k], base + ((x >> 8) & 0xFFF0u), 16);
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) acc ^= v[k].x ^ v[k].w;
    }
    if (acc == 0x12345678u) out[0] = acc;
}

#define CK(x)                                                                 \
    do {                                                                      \
        hipError_t e_ = (x);                                                  \
        if (e_ != hipSuccess) {                                               \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));           \
            exit(1);                                                          \
        }                                                                     \
    } while (0)

int main() {
    const int64_t N = 4ll << 30;             // bytes per buffer
    const int64_t regions = N / kRegion;     // 65 536 regions of 64 KiB
    const int reads = 512;
    uint8_t *a, *b;
    uint32_t* o;
    CK(hipMalloc(&a, N));
    CK(hipMalloc(&b, N));
    CK(hipMalloc(&o, 64));
    hipLaunchKernelGGL(fill, dim3(8192), dim3(256), 0, 0, (u32x4*)a, N / 16);
    hipLaunchKernelGGL(fill, dim3(8192), dim3(256), 0, 0, (u32x4*)b, N / 16);
    CK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    float ms;
    // one launch each, in this order (tools/pmc_cal_report.py keys on the names)
    CK(hipEventRecord(e0));
    hipLaunchKernelGGL(copy16, dim3(8192), dim3(256), 0, 0, (const u32x4*)a, (u32x4*)b, N / 16);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    CK(hipEventElapsedTime(&ms, e0, e1));
    printf("{\"kernel\": \"copy16\", \"read\": %lld, \"write\": %lld, \"ms\": %.3f}\n", (long long)N, (long long)N, ms);
    CK(hipEventRecord(e0));
    hipLaunchKernelGGL(lane_write, dim3((uint32_t)(regions / 64)), dim3(64), 0, 0, a, regions);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    CK(hipEventElapsedTime(&ms, e0, e1));
    printf("{\"kernel\": \"lane_write\", \"read\": 0, \"write\": %lld, \"ms\": %.3f}\n", (long long)N, ms);
    CK(hipEventRecord(e0));
    hipLaunchKernelGGL(row_write, dim3((uint32_t)(regions / 4)), dim3(64), 0, 0, b, regions);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    CK(hipEventElapsedTime(&ms, e0, e1));
    printf("{\"kernel\": \"row_write\", \"read\": 0, \"write\": %lld, \"ms\": %.3f}\n", (long long)N, ms);
    CK(hipEventRecord(e0));
    hipLaunchKernelGGL(lane_read, dim3((uint32_t)(regions / 64)), dim3(64), 0, 0, a, regions, o);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    CK(hipEventElapsedTime(&ms, e0, e1));
    printf("{\"kernel\": \"lane_read\", \"read\": %lld, \"write\": 0, \"ms\": %.3f}\n", (long long)N, ms);
    CK(hipEventRecord(e0));
    hipLaunchKernelGGL(rand_read, dim3((uint32_t)(regions / 64)), dim3(64), 0, 0, b, regions, reads, o);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    CK(hipEventElapsedTime(&ms, e0, e1));
    printf("{\"kernel\": \"rand_read\", \"read\": null, \"pieces\": %lld, \"write\": 0, \"ms\": %.3f}\n",
           (long long)regions * reads, ms);
    CK(hipFree(a));
    CK(hipFree(b));
    CK(hipFree(o));
    return 0;
}
