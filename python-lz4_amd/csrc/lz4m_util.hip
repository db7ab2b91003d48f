// lz4m_util.hip -- compaction and frame-assembly kernels (gfx950).
//
// Variable-length block outputs are compacted by an exclusive prefix scan of
// their sizes (3 launches: per-tile sums, scan of tile sums, per-tile scan)
// followed by a wave-per-item gather.  Frame emission writes the
// LZ4F_makeBlock records (lz4frame.c:825-850) for independent blocks at the
// scanned offsets.
#include "lz4m_common.h"
#include "../../include/lz4m.h"
#include "lz4m_xxh32_dev.h"

namespace lz4m {

constexpr int kScanThreads = 256;
constexpr int kScanPerThread = 8;
constexpr int kScanTile = kScanThreads * kScanPerThread;   // 2048 items per tile

// inclusive scan of one int64 per lane across the 256-thread workgroup
__device__ __forceinline__ int64_t wg_inclusive_scan(int64_t v, int64_t* lds) {
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const int64_t o = __shfl_up(v, d);
        if ((int)lane >= d) v += o;
    }
    if (lane == 63) lds[wave] = v;
    __syncthreads();
    int64_t pre = 0;
    for (uint32_t w = 0; w < wave; ++w) pre += lds[w];
    __syncthreads();
    return v + pre;
}

__global__ __launch_bounds__(kScanThreads) void scan_tile_sums(const int32_t* __restrict__ len, int64_t add,
                                                               int64_t* __restrict__ tile_sum, int64_t n) {
    __shared__ int64_t lds[4];
    const int64_t base = (int64_t)blockIdx.x * kScanTile + (int64_t)threadIdx.x * kScanPerThread;
    int64_t s = 0;
#pragma unroll
    for (int k = 0; k < kScanPerThread; ++k)
        if (base + k < n) s += (int64_t)len[base + k] + add;
    const int64_t inc = wg_inclusive_scan(s, lds);
    if (threadIdx.x == kScanThreads - 1) tile_sum[blockIdx.x] = inc;
}

// exclusive scan of the tile sums in place (one workgroup, serial over tiles
// of 256)
__global__ __launch_bounds__(kScanThreads) void scan_tiles(int64_t* __restrict__ tile_sum, int64_t ntiles,
                                                           int64_t base) {
    __shared__ int64_t lds[4];
    __shared__ int64_t carry_s;
    if (threadIdx.x == 0) carry_s = base;
    __syncthreads();
    for (int64_t t0 = 0; t0 < ntiles; t0 += kScanThreads) {
        const int64_t t = t0 + threadIdx.x;
        const int64_t v = t < ntiles ? tile_sum[t] : 0;
        const int64_t inc = wg_inclusive_scan(v, lds);
        const int64_t carry = carry_s;
        if (t < ntiles) tile_sum[t] = carry + inc - v;
        __syncthreads();
        if (threadIdx.x == kScanThreads - 1) carry_s = carry + inc;
        __syncthreads();
    }
}

__global__ __launch_bounds__(kScanThreads) void scan_apply(const int32_t* __restrict__ len, int64_t add,
                                                           const int64_t* __restrict__ tile_pre,
                                                           int64_t* __restrict__ out, int64_t n) {
    __shared__ int64_t lds[4];
    const int64_t base = (int64_t)blockIdx.x * kScanTile + (int64_t)threadIdx.x * kScanPerThread;
    int64_t v[kScanPerThread];
    int64_t s = 0;
#pragma unroll
    for (int k = 0; k < kScanPerThread; ++k) {
        v[k] = base + k < n ? (int64_t)len[base + k] + add : 0;
        s += v[k];
    }
    const int64_t inc = wg_inclusive_scan(s, lds);
    int64_t run = tile_pre[blockIdx.x] + inc - s;
#pragma unroll
    for (int k = 0; k < kScanPerThread; ++k) {
        if (base + k < n) out[base + k] = run;
        run += v[k];
        if (base + k == n - 1) out[n] = run;
    }
}

__global__ void scan_store_base(int64_t* out, int64_t base) { out[0] = base; }

__global__ __launch_bounds__(256) void gather_kernel(const uint8_t* __restrict__ src,
                                                     const int64_t* __restrict__ src_off,
                                                     const int32_t* __restrict__ len, uint8_t* __restrict__ out,
                                                     const int64_t* __restrict__ out_off, int64_t n) {
    const int64_t item = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const uint32_t lane = threadIdx.x & 63;
    if (item >= n) return;
    const uint8_t* s = src + src_off[item];
    uint8_t* d = out + out_off[item];
    const int64_t L = len[item];
    for (int64_t pos = 16 * (int64_t)lane; pos < L; pos += 16 * kWave) {
        if (L - pos >= 16) {
            st16(d + pos, ld16(s + pos));
        } else {
            for (int64_t k = pos; k < L; ++k) d[k] = s[k];
        }
    }
}

// ------------------------------------------------------------------ frames
__device__ __forceinline__ bool stored_raw(int32_t raw_len, int32_t cmp_len) {
    return cmp_len <= 0 || cmp_len >= raw_len;   // lz4frame.c:838
}

__global__ void frame_sizes_kernel(const int32_t* __restrict__ raw_len, const int32_t* __restrict__ cmp_len,
                                   int block_checksum, int32_t* __restrict__ rec_len, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int32_t payload = stored_raw(raw_len[i], cmp_len[i]) ? raw_len[i] : cmp_len[i];
    rec_len[i] = 4 + payload + (block_checksum ? 4 : 0);
}

// wave per block: header + payload
__global__ __launch_bounds__(256) void frame_emit_kernel(const uint8_t* __restrict__ raw,
                                                         const int64_t* __restrict__ raw_off,
                                                         const int32_t* __restrict__ raw_len,
                                                         const uint8_t* __restrict__ cmp,
                                                         const int64_t* __restrict__ cmp_off,
                                                         const int32_t* __restrict__ cmp_len,
                                                         uint8_t* __restrict__ frame,
                                                         const int64_t* __restrict__ frame_off, int64_t n) {
    const int64_t item = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const uint32_t lane = threadIdx.x & 63;
    if (item >= n) return;
    const bool raw_blk = stored_raw(raw_len[item], cmp_len[item]);
    const int64_t L = raw_blk ? raw_len[item] : cmp_len[item];
    const uint8_t* s = raw_blk ? raw + raw_off[item] : cmp + cmp_off[item];
    uint8_t* d = frame + frame_off[item];
    if (lane == 0) {
        const uint32_t hdr = (uint32_t)L | (raw_blk ? 0x80000000u : 0u);   // lz4frame.c:839-842
        d[0] = (uint8_t)hdr;
        d[1] = (uint8_t)(hdr >> 8);
        d[2] = (uint8_t)(hdr >> 16);
        d[3] = (uint8_t)(hdr >> 24);
    }
    d += 4;
    for (int64_t pos = 16 * (int64_t)lane; pos < L; pos += 16 * kWave) {
        if (L - pos >= 16) {
            st16(d + pos, ld16(s + pos));
        } else {
            for (int64_t k = pos; k < L; ++k) d[k] = s[k];
        }
    }
}

// quad per block (xxh32_quad_acc): block checksum = XXH32 of the payload
// (lz4frame.c:844-847), read back from the frame buffer after
// frame_emit_kernel; 16 blocks per 64-lane workgroup.
__global__ __launch_bounds__(64) void frame_block_crc_kernel(uint8_t* __restrict__ frame,
                                                             const int64_t* __restrict__ frame_off,
                                                             const int32_t* __restrict__ raw_len,
                                                             const int32_t* __restrict__ cmp_len, int64_t n) {
    const uint32_t l = threadIdx.x, a = l & 3u;
    const int64_t i = (int64_t)blockIdx.x * 16 + (l >> 2);
    const bool live = i < n;
    const int64_t L = live ? (stored_raw(raw_len[i], cmp_len[i]) ? raw_len[i] : cmp_len[i]) : 0;
    uint8_t* d = frame + (live ? frame_off[i] + 4 : 0);
    const uint32_t n16 = (uint32_t)(L >> 4);
    const uint32_t steps = wave_max_u32(n16);
    const uint64_t has = __ballot(n16 > 0);
    const uint8_t* dv = n16 > 0 ? d : (has ? (const uint8_t*)readlane64((int64_t)(uintptr_t)d, __builtin_ctzll(has)) : d);
    const uint32_t v = xxh32_quad_acc(dv, n16, steps, 0, a);
    const uint32_t c = xxh32_quad_finish(v, d, L, 0);
    if (live && a == 0) {
        d[L] = (uint8_t)c;
        d[L + 1] = (uint8_t)(c >> 8);
        d[L + 2] = (uint8_t)(c >> 16);
        d[L + 3] = (uint8_t)(c >> 24);
    }
}


// LZ4F_decompress's walk over the block records of a frame already in HBM
// (lz4frame.c:1643-1701 block headers, 1926-1965 endmark and content
// checksum).  Serial by construction -- each record's position depends on
// the previous one's size -- so one lane walks it: one dependent HBM read per
// record (~1-2 us; 2 048 records of an 8 GiB, 4 MiB-block frame take a few
// ms).  result = {records, state, end, content-checksum position}; state 0 =
// complete frame, 1 = incomplete, 2 = block size above the maximum, 3 =
// content checksum missing, 4 = more than max_rec records.
__global__ void frame_scan_kernel(const uint8_t* __restrict__ frame, int64_t n, int64_t pos, int crc,
                                  int content_checksum, int32_t max_block, int64_t max_rec,
                                  int64_t* __restrict__ rec_pos, int32_t* __restrict__ rec_len,
                                  uint8_t* __restrict__ rec_raw, int64_t* __restrict__ result) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    int64_t k = 0, state = 0, end = 0, cpos = -1;
    while (true) {
        if (n - pos < 4) {
            state = 1;
            break;
        }
        const uint32_t hdr = ld32(frame + pos);
        pos += 4;
        if (hdr == 0) {   // endmark
            if (content_checksum) {
                if (n - pos < 4) {
                    state = 3;
                    break;
                }
                cpos = pos;
                end = pos + 4;
            } else {
                end = pos;
            }
            break;
        }
        const int64_t size = hdr & 0x7FFFFFFFu;
        if (size > max_block) {
            state = 2;
            break;
        }
        if (n - pos < size + crc) {
            state = 1;
            break;
        }
        if (k == max_rec) {
            state = 4;
            break;
        }
        rec_pos[k] = pos;
        rec_len[k] = (int32_t)size;
        rec_raw[k] = (uint8_t)(hdr >> 31);
        ++k;
        pos += size + crc;
    }
    result[0] = k;
    result[1] = state;
    result[2] = end;
    result[3] = cpos;
}

}  // namespace lz4m

using namespace lz4m;

extern "C" int64_t lz4m_scan_scratch_entries(int64_t n) { return n <= 0 ? 1 : (n + kScanTile - 1) / kScanTile; }

extern "C" int lz4m_exclusive_scan(const int32_t* d_len, int64_t add, int64_t base, int64_t* d_out,
                                   int64_t* d_scratch, int64_t n, lz4m_stream_t stream) {
    if (n < 0 || !d_out) return LZ4M_EINVAL;
    hipStream_t s = (hipStream_t)stream;
    const int64_t ntiles = lz4m_scan_scratch_entries(n);
    if (n == 0) {
        hipLaunchKernelGGL(scan_store_base, dim3(1), dim3(1), 0, s, d_out, base);
        return (int)hipGetLastError();
    }
    hipLaunchKernelGGL(scan_tile_sums, dim3((uint32_t)ntiles), dim3(kScanThreads), 0, s, d_len, add, d_scratch, n);
    hipLaunchKernelGGL(scan_tiles, dim3(1), dim3(kScanThreads), 0, s, d_scratch, ntiles, base);
    hipLaunchKernelGGL(scan_apply, dim3((uint32_t)ntiles), dim3(kScanThreads), 0, s, d_len, add, d_scratch, d_out, n);
    return (int)hipGetLastError();
}

extern "C" int lz4m_gather(const uint8_t* d_src, const int64_t* d_src_off, const int32_t* d_len, uint8_t* d_out,
                           const int64_t* d_out_off, int64_t n, lz4m_stream_t stream) {
    if (n < 0) return LZ4M_EINVAL;
    if (n == 0) return 0;
    hipLaunchKernelGGL(gather_kernel, dim3((uint32_t)((n + 3) / 4)), dim3(256), 0, (hipStream_t)stream, d_src,
                       d_src_off, d_len, d_out, d_out_off, n);
    return (int)hipGetLastError();
}

extern "C" int lz4m_frame_block_sizes(const int32_t* d_raw_len, const int32_t* d_cmp_len, int block_checksum,
                                      int32_t* d_rec_len, int64_t n, lz4m_stream_t stream) {
    if (n < 0) return LZ4M_EINVAL;
    if (n == 0) return 0;
    hipLaunchKernelGGL(frame_sizes_kernel, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                       d_raw_len, d_cmp_len, block_checksum, d_rec_len, n);
    return (int)hipGetLastError();
}

extern "C" int lz4m_frame_emit(const uint8_t* d_raw, const int64_t* d_raw_off, const int32_t* d_raw_len,
                               const uint8_t* d_cmp, const int64_t* d_cmp_off, const int32_t* d_cmp_len,
                               uint8_t* d_frame, const int64_t* d_frame_off, int block_checksum, int64_t n,
                               lz4m_stream_t stream) {
    if (n < 0) return LZ4M_EINVAL;
    if (n == 0) return 0;
    hipStream_t s = (hipStream_t)stream;
    hipLaunchKernelGGL(frame_emit_kernel, dim3((uint32_t)((n + 3) / 4)), dim3(256), 0, s, d_raw, d_raw_off,
                       d_raw_len, d_cmp, d_cmp_off, d_cmp_len, d_frame, d_frame_off, n);
    if (block_checksum)
        hipLaunchKernelGGL(frame_block_crc_kernel, dim3((uint32_t)((n + 15) / 16)), dim3(64), 0, s, d_frame,
                           d_frame_off, d_raw_len, d_cmp_len, n);
    return (int)hipGetLastError();
}

extern "C" int lz4m_frame_scan(const uint8_t* d_frame, int64_t frame_len, int64_t pos, int block_checksum,
                               int content_checksum, int32_t max_block, int64_t max_rec, int64_t* d_rec_pos,
                               int32_t* d_rec_len, uint8_t* d_rec_raw, int64_t* d_result, lz4m_stream_t stream) {
    if (frame_len < 0 || pos < 0 || max_block < 0 || max_rec < 0 || !d_result) return LZ4M_EINVAL;
    hipLaunchKernelGGL(frame_scan_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, d_frame, frame_len, pos,
                       block_checksum ? 4 : 0, content_checksum, max_block, max_rec, d_rec_pos, d_rec_len, d_rec_raw,
                       d_result);
    return (int)hipGetLastError();
}

extern "C" int lz4m_version_number(void) { return 10904; }
extern "C" const char* lz4m_version_string(void) { return "1.9.4"; }
