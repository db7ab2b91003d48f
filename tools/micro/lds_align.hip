// Microbenchmark (dev only): cost of LDS accesses by width and byte
// alignment on gfx950 -- the row decoder puts and reads 16-byte windows at
// arbitrary byte offsets of its history buffers.  Every lane of 16 waves per
// CU issues ITER accesses of one kind at address 32 * lane + MIS (+ a rotating
// 512-byte offset); the kernel time per wave-instruction is printed.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) uint8_t lds_u8;
constexpr int ITER = 4096;

template <int OP, int W>
__global__ __launch_bounds__(64) void k(uint32_t mis, uint32_t* out) {
    __shared__ __attribute__((aligned(16))) uint8_t buf[8192];
    const uint32_t lane = threadIdx.x;
    lds_u8* b = (lds_u8*)buf;
    for (int i = lane; i < 2048; i += 64) reinterpret_cast<uint32_t*>(buf)[i] = i * 2654435761u;
    __syncthreads();
    uint32_t acc = 0;
    u32x4 v = u32x4{lane, lane * 3, lane * 5, lane * 7};
    for (int it = 0; it < ITER; ++it) {
        const uint32_t a = 32u * lane + mis + ((uint32_t)(it & 7) << 9);
        asm volatile("" ::: "memory");   // one access per iteration (no hoisting or pairing)
        if (OP == 0) {   // read
            if (W == 16) {
                u32x4 x;
                __builtin_memcpy(&x, (const uint8_t*)(b + a), 16);
                acc += x.x ^ x.w;
            } else if (W == 8) {
                u32x2 x;
                __builtin_memcpy(&x, (const uint8_t*)(b + a), 8);
                acc += x.x ^ x.y;
            } else {
                uint32_t x;
                __builtin_memcpy(&x, (const uint8_t*)(b + a), 4);
                acc += x;
            }
        } else if (OP == 2) {   // masked OR of one aligned dword (ds_mskor_b32)
            const uint32_t aa = (uint32_t)(uintptr_t)(b + (a & ~3u));
            asm volatile("ds_mskor_b32 %0, %1, %2" ::"v"(aa), "v"(0x00FFFF00u), "v"(v.x & 0x00FFFF00u) : "memory");
            v.x += (uint32_t)it;
        } else {         // write
            v.x += (uint32_t)it;
            if (W == 16) {
                __builtin_memcpy((uint8_t*)(b + a), &v, 16);
            } else if (W == 8) {
                __builtin_memcpy((uint8_t*)(b + a), &v, 8);
            } else if (W == 4) {
                __builtin_memcpy((uint8_t*)(b + a), &v, 4);
            } else if (W == 2) {
                const uint16_t h = (uint16_t)v.x;
                __builtin_memcpy((uint8_t*)(b + a), &h, 2);
            } else {
                *(b + a) = (uint8_t)v.x;
            }
            __builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0): keep the stores in order with the loop
        }
    }
    __syncthreads();
    acc += reinterpret_cast<uint32_t*>(buf)[lane];
    if (acc == 0x12345678u) out[0] = acc;
}

template <int OP, int W>
void run(const char* name, uint32_t* o) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const int grid = 256 * 16;
    for (uint32_t mis : {0u, 1u, 2u, 4u, 8u}) {
        hipLaunchKernelGGL((k<OP, W>), dim3(grid), dim3(64), 0, 0, mis, o);
        hipEventRecord(e0);
        hipLaunchKernelGGL((k<OP, W>), dim3(grid), dim3(64), 0, 0, mis, o);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        // per CU: 16 waves x ITER wave-instructions; cycles at ~2.1 GHz
        const double per = ms * 1e-3 * 2.1e9 / (16.0 * ITER);
        printf("{\"op\": \"%s\", \"misalign\": %u, \"ms\": %.3f, \"cu_cycles_per_wave_instr\": %.2f}\n", name, mis, ms,
               per);
    }
}

int main() {
    uint32_t* o;
    hipMalloc(&o, 64);
    run<0, 16>("ds_read_b128", o);
    run<0, 8>("ds_read_b64", o);
    run<0, 4>("ds_read_b32", o);
    run<1, 16>("ds_write_b128", o);
    run<1, 8>("ds_write_b64", o);
    run<1, 4>("ds_write_b32", o);
    run<1, 2>("ds_write_b16", o);
    run<1, 1>("ds_write_b8", o);
    run<2, 4>("ds_mskor_b32", o);
    hipFree(o);
    return 0;
}
