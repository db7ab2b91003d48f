// lz4m_rows.h -- internal interface of the large-batch decoder (lz4m_rows.hip),
// used by the dispatch in lz4m_decompress.hip.  Not part of the C-ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace lz4m {

// One record per block, written by rows_parse_kernel: where its recorded
// sequence lengths live, how many good sequences it has, and the reference
// decoder's state (input / output position) at the first sequence that is
// not good -- where the exact finisher resumes.
struct RowMeta {
    int64_t loff;
    int32_t nseq, ip, op, pad0;
    int64_t pad1;
};
static_assert(sizeof(RowMeta) == 32, "RowMeta layout");

// scratch layout: 64 bytes of counters, one RowMeta per block, then the
// length bytes
constexpr size_t kRowsMeta = 64;

}  // namespace lz4m

#define LZ4M_ROWS_ENOSPACE 0x10001

extern "C" {
// scratch needed before the length bytes: 64 bytes of counters + one RowMeta per block
size_t lz4m_rows_fixed_bytes(int64_t n);
// persistent grid sizes for the two kernels on the current device
int lz4m_rows_grids(int64_t n, int* parse_grid, int* exec_grid);
// parse + row execution; the finisher is launched by the caller afterwards
int lz4m_rows_launch(const uint8_t* d_src, const int64_t* d_src_off, const int32_t* d_src_len, uint8_t* d_dst,
                     const int64_t* d_dst_off, const int32_t* d_dst_cap, int64_t n, void* d_work, size_t work_bytes,
                     int parse_grid, int exec_grid, hipStream_t stream);
}
