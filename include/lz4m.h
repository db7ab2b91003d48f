/*
 * include/lz4m.h -- C-ABI of the MI355X-native batched LZ4 block codec.
 *
 * Drop-in boundary for the python-lz4 hot path: the
 * reference's CPython extensions (lz4/block/_block.c, lz4/frame/_frame.c)
 * call into lz4libs/lz4.c and lz4libs/xxhash.c once per block; these entry
 * points replace those calls with stream-ordered, batched HIP launches over
 * device-resident blocks.  Plain pointers and sizes only: every pointer named
 * d_* is a device (HBM) pointer, `stream` is a hipStream_t.  No batched entry
 * point synchronises or touches host memory except the speculative mode of
 * lz4m_compress_linked_batch (one stream synchronisation per pass); only
 * lz4m_decompress_batch allocates (64 bytes, stream-ordered), so every other
 * call can be captured into a hipGraph.
 *
 * Return value of every launcher: 0 on success, otherwise a hipError_t value
 * (launch failure) or LZ4M_EINVAL (bad argument).
 *
 * Per-block results follow the reference's own conventions:
 *   - decompress status = decoded size, or -(input position)-1 at the point
 *     where the input was rejected (lz4.c:2336-2337), bit-identical to
 *     LZ4_decompress_safe / LZ4_decompress_safe_usingDict;
 *   - compress length   = compressed size, or 0 when it does not fit in the
 *     block's capacity (lz4.h:180-186, limitedOutput).
 */
#ifndef LZ4M_H
#define LZ4M_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct ihipStream_t* lz4m_stream_t;   /* == hipStream_t */

#define LZ4M_EINVAL 0x10000
/* The device failed the LDS lane-order self-test (lz4m_selftest_lds_order):
 * the compressors' search steps rely on one instruction's same-address LDS
 * atomics being applied in lane order (gfx950 does), and refuse to run. */
#define LZ4M_EDEVICE 0x10001

/* Match-finder table layouts:
 *   U16_HASH4: LZ4_compress_default on blocks < 65547 B (lz4.c:1353-1354),
 *              frame independent blocks (lz4.c:1399-1406);
 *   U32_HASH5: lz4.block.compress (_block.c:109 -> LZ4_compress_fast_continue,
 *              lz4.c:1671-1675) and LZ4_compress_default on >= 65547 B. */
#define LZ4M_TABLE_U16_HASH4 0
#define LZ4M_TABLE_U32_HASH5 1
/* pick what LZ4_compress_default would pick for each block's size */
#define LZ4M_TABLE_AUTO      2
/* parallel-parse compressor (lz4m_pcompress.hip): a valid block near the
 * ratio of LZ4_compress_default (greedy, full insertion, catch-up), NOT
 * byte-identical to it; blocks up to 64 KiB (larger ones get size 0);
 * `acceleration` is ignored.  For bulk compression (BASELINE config 3).
 * PARALLEL uses a 12-bit hash table (+1.5 % size on the silesia-like mix,
 * 1.7x the speed), PARALLEL_HQ the reference's 13 bits (-0.02 % size). */
#define LZ4M_PARSE_PARALLEL  3
#define LZ4M_PARSE_PARALLEL_HQ 5
/* the same parse for blocks of any size (32 KiB LDS table of u32 positions,
 * offsets limited to 65535 like LZ4_DISTANCE_MAX); e.g. 4 MiB frame blocks */
#define LZ4M_PARSE_PARALLEL_LARGE 4

/* LZ4_compressBound (lz4.h:212 / lz4.c:730). */
int lz4m_compress_bound(int input_size);

/* Runs the LDS lane-order self-test on the current device (synchronous, its
 * own stream): returns the number of test instructions whose same-address
 * exchanges were not applied in lane order (0 = the compressors' insert
 * order holds), or a negative HIP error.  Every compression entry point runs
 * it once per process and returns LZ4M_EDEVICE if it fails. */
int lz4m_selftest_lds_order(void);

/*
 * Batched lz4.block.compress(source, dict=D) for the non-HC modes
 * (_block.c:93-107: LZ4_resetStream + LZ4_loadDict, lz4.c:1541-1581, +
 * LZ4_compress_fast_continue, lz4.c:1632-1708), byte-identical.
 * d_dict_len[i] < 0: no dictionary (same as lz4m_compress_batch with
 * LZ4M_TABLE_U32_HASH5).  d_dict_len[i] >= 0: the dictionary's full length;
 * its last min(d_dict_len[i], 65536) bytes must be stored immediately before
 * block i in d_src (d_src + d_src_off[i] - that many bytes).  Like
 * LZ4_loadDict, a dictionary shorter than 8 bytes is not used as history but
 * still changes the parse (an empty dict= differs from no dict=).
 */
int lz4m_compress_dict_batch(const uint8_t* d_src, const int64_t* d_src_off, const int32_t* d_src_len,
                             const int32_t* d_dict_len, uint8_t* d_dst, const int64_t* d_dst_off,
                             const int32_t* d_dst_cap, int32_t* d_out_len, int64_t n, int acceleration,
                             lz4m_stream_t stream);

/*
 * The same call when the caller's dictionary memory ends exactly where the
 * source begins (lz4.block.compress(src, dict=D) with D and src slices of one
 * buffer, D >= 8 bytes): LZ4_compress_fast_continue then sees
 * dictEnd == source and compresses in prefix mode (lz4.c:1671-1676,
 * withPrefix64k) instead of usingExtDict: backward catch-up of every match
 * may reach into the dictionary (lowLimit = source - dictSize, lz4.c:967).
 * Same layout and arguments as lz4m_compress_dict_batch.
 */
int lz4m_compress_prefix_batch(const uint8_t* d_src, const int64_t* d_src_off, const int32_t* d_src_len,
                               const int32_t* d_dict_len, uint8_t* d_dst, const int64_t* d_dst_off,
                               const int32_t* d_dst_cap, int32_t* d_out_len, int64_t n, int acceleration,
                               lz4m_stream_t stream);

/*
 * Batched linked-block compression: the blocks of one stream are compressed
 * as consecutive LZ4_compress_fast_continue calls on one LZ4_stream_t that
 * was freshly initialised (LZ4F_compressBlock_continue, lz4frame.c:865-871;
 * LZ4F_compressFrame with blockLinked), byte-identical to the reference.
 * d_link[i] = 0 starts a new stream at block i, 1 continues the stream of
 * block i-1, whose bytes must end where block i starts in d_src.  Capacities
 * < LZ4_compressBound select limitedOutput (0 = did not fit; the frame stores
 * such a block raw, lz4frame.c:833-842, and the stream still continues).
 *   LZ4M_LINKED_SERIAL: one wavefront per stream, no scratch, stream-ordered.
 *   LZ4M_LINKED_SPECULATIVE: one wavefront per block, parallel within a
 *     stream (every block compressed from its predecessor's table,
 *     speculatively, in passes until no table changes).  Every block that has
 *     a successor in its stream must be >= 65536 B (frame blocks are; else
 *     LZ4M_EINVAL).  Needs lz4m_compress_linked_workspace_size(n) bytes of
 *     device scratch and SYNCHRONISES the stream once per pass (typically 3-6).
 */
#define LZ4M_LINKED_SERIAL      1
#define LZ4M_LINKED_SPECULATIVE 2
size_t lz4m_compress_linked_workspace_size(int64_t n);
/* passes the calling thread's last speculative call took (diagnostics) */
int lz4m_compress_linked_passes(void);
int lz4m_compress_linked_batch(const uint8_t* d_src, const int64_t* d_src_off, const int32_t* d_src_len,
                               const int32_t* d_link, uint8_t* d_dst, const int64_t* d_dst_off,
                               const int32_t* d_dst_cap, int32_t* d_out_len, int64_t n, int acceleration,
                               int mode, void* d_work, size_t work_bytes, lz4m_stream_t stream);

/*
 * LZ4M_PARSE_PARALLEL_LARGE for batches of few large blocks (lz4.frame with
 * 256 KiB - 4 MiB independent blocks and parse="parallel", no reference
 * counterpart: the reference compresses such a frame's blocks one by one,
 * lz4frame.c:865-871).  Each block is parsed as up to 16 segments of >= 256
 * KiB, one wavefront each, then joined (valid LZ4 blocks, not the exact
 * parse).  Blocks longer than max_len report 0 (not compressed).  Needs
 * lz4m_pcompress_large_workspace_size(n, max_len) bytes of device scratch
 * (about 16 x the largest block per block).  Stream-ordered, no sync.
 */
size_t lz4m_pcompress_large_workspace_size(int64_t n, int32_t max_len);
int lz4m_pcompress_large_batch(const uint8_t* d_src, const int64_t* d_src_off, const int32_t* d_src_len,
                               uint8_t* d_dst, const int64_t* d_dst_off, const int32_t* d_dst_cap,
                               int32_t* d_out_len, int64_t n, int32_t max_len, void* d_work, size_t work_bytes,
                               lz4m_stream_t stream);

/* Library identification (mirrors LZ4_versionNumber, lz4.c:728, of the
 * format version this codec is bit-compatible with: 10904). */
int lz4m_version_number(void);
const char* lz4m_version_string(void);

/*
 * Batched LZ4_decompress_safe (lz4.h:191-205, lz4.c:2344-2350).
 * Block i: input  d_src[d_src_off[i] .. + d_src_len[i]),
 *          output d_dst[d_dst_off[i] .. + d_dst_cap[i]).
 * d_status[i] = decoded size or -(pos)-1.  Bytes of a block's output slot
 * beyond its decoded size are unspecified (as in the reference).  Output
 * slots must not overlap.  Replaces the call at _block.c:357-359 and the
 * per-block call in LZ4F_decompress (lz4frame.c:1844-1847).
 * Every decoder gives identical bytes and statuses; they differ in speed:
 *   rows   -- large batches: a lane-per-block parse, then one 16-lane row per
 *             block with its recent output in LDS, then an exact lane-per-block
 *             finisher for each block's tail (needs the scratch of
 *             lz4m_decompress_workspace_size);
 *   hist   -- one wavefront per block with its recent output in LDS (small and
 *             mid-size batches, large blocks, and any batch without scratch);
 * This entry point takes no scratch, so it always uses the hist decoder; pass
 * scratch through lz4m_decompress_batch_ws for the rows decoder.
 */
int lz4m_decompress_batch(const uint8_t* d_src, const int64_t* d_src_off, const int32_t* d_src_len,
                          uint8_t* d_dst, const int64_t* d_dst_off, const int32_t* d_dst_cap,
                          int32_t* d_status, int64_t n, lz4m_stream_t stream);

/* Minimum device scratch of lz4m_decompress_batch_ws (64 bytes). */
size_t lz4m_decompress_workspace_bytes(void);

/* Device scratch for the fastest decode of n blocks whose compressed sizes
 * sum to at most src_bytes: 64 + 32 n bytes of counters and per-block
 * records, plus one byte per three compressed bytes for sequence lengths
 * (each block's lengths start 16-byte aligned: up to 16 more bytes a block).
 * Less scratch is accepted: blocks whose lengths do not fit are decoded by
 * the exact finisher alone, and below 64 + 32 n + 64 bytes the rows decoder
 * is not used. */
size_t lz4m_decompress_workspace_size(int64_t n, int64_t src_bytes);

/* lz4m_decompress_batch with caller-provided device scratch (8-byte aligned,
 * at least lz4m_decompress_workspace_bytes(), not shared with a concurrently
 * running call).  Picks the decoder by batch size and scratch: rows from
 * LZ4M_ROWS_MIN_BLOCKS (32 768) blocks when the scratch fits, else hist
 * (env LZ4M_DECODER=rows|hist forces one). */
int lz4m_decompress_batch_ws(const uint8_t* d_src, const int64_t* d_src_off, const int32_t* d_src_len,
                             uint8_t* d_dst, const int64_t* d_dst_off, const int32_t* d_dst_cap,
                             int32_t* d_status, int64_t n, void* d_work, size_t work_bytes,
                             lz4m_stream_t stream);

/* lz4m_decompress_batch_ws with an explicit decoder (tests, A/B runs); any
 * other id (1, 2, 5, 6 and 7 were retired decoders) returns LZ4M_EINVAL. */
#define LZ4M_DECODER_AUTO   0
#define LZ4M_DECODER_HIST   3
#define LZ4M_DECODER_ROWS   4
int lz4m_decompress_batch_sel(const uint8_t* d_src, const int64_t* d_src_off, const int32_t* d_src_len,
                              uint8_t* d_dst, const int64_t* d_dst_off, const int32_t* d_dst_cap,
                              int32_t* d_status, int64_t n, void* d_work, size_t work_bytes, int decoder,
                              lz4m_stream_t stream);

/*
 * Batched LZ4_decompress_safe_usingDict with the dictionary in a separate
 * buffer (usingExtDict, lz4.c:2612-2625, the `dict=` argument of
 * lz4.block.decompress, _block.c:357-359).  Dictionary i is
 * d_dict[d_dict_off[i] .. + d_dict_len[i]); d_dict_len[i] == 0 means none.
 */
int lz4m_decompress_batch_dict(const uint8_t* d_src, const int64_t* d_src_off, const int32_t* d_src_len,
                               uint8_t* d_dst, const int64_t* d_dst_off, const int32_t* d_dst_cap,
                               const uint8_t* d_dict, const int64_t* d_dict_off, const int32_t* d_dict_len,
                               int32_t* d_status, int64_t n, lz4m_stream_t stream);

/*
 * Batched LZ4_decompress_safe_usingDict (lz4.c:2612-2625) with the
 * dictionaries in a buffer laid out like d_dst: block i's dictionary is the
 * d_dict_len[i] bytes ending at d_dict_base + d_dst_off[i].  Built for
 * linked-block frames (LZ4F_decompress, lz4frame.c:1853-1856): the previous
 * round's output of the whole frame as d_dict_base, so block i sees the
 * last <= 64 KiB before its slot (lz4.frame's speculative rounds, DESIGN.md
 * section 3.3).  One wavefront per block (the on-chip-history decoder);
 * statuses and bytes are those of lz4m_decompress_batch_dict with the same
 * dictionaries.  The call must not write the dictionary bytes (d_dict_base
 * != d_dst unless the dictionaries lie outside every output slot).
 */
int lz4m_decompress_batch_prefix(const uint8_t* d_src, const int64_t* d_src_off, const int32_t* d_src_len,
                                 uint8_t* d_dst, const int64_t* d_dst_off, const int32_t* d_dst_cap,
                                 const uint8_t* d_dict_base, const int32_t* d_dict_len, int32_t* d_status, int64_t n,
                                 lz4m_stream_t stream);

/*
 * Linked-block frame decode (LZ4F_decompress on a blockLinked frame,
 * lz4frame.c:1844-1856): block i may reference the output of blocks < i, so
 * blocks decode in order on one wavefront, contiguously into d_dst (capacity
 * max_block per block).  d_raw_flag[i] != 0 marks a stored (uncompressed)
 * block, copied as is.  d_status[i] = decoded size or -(pos)-1; after the
 * first failing block the remaining statuses are -1.
 */
int lz4m_decompress_chain(const uint8_t* d_src, const int64_t* d_src_off, const int32_t* d_src_len,
                          const uint8_t* d_raw_flag, uint8_t* d_dst, int32_t* d_status, int64_t n,
                          int32_t max_block, lz4m_stream_t stream);

/*
 * Batched greedy compressor, bit-exact with the reference parse for the
 * chosen table layout (LZ4_compress_generic_validated, lz4.c:910-1302, fresh
 * table per block).  acceleration as LZ4_compress_fast (clamped to
 * [1, 65537], lz4.c:1350-1351).  d_out_len[i] = compressed size, or 0 when
 * the block does not fit in d_dst_cap[i] bytes (limitedOutput).
 * Replaces _block.c:233-235 (table U32_HASH5) and the per-block
 * LZ4_compress_fast_extState_fastReset in LZ4F_compressBlock
 * (lz4frame.c:853-863, table U16_HASH4 / AUTO).
 */
int lz4m_compress_batch(const uint8_t* d_src, const int64_t* d_src_off, const int32_t* d_src_len,
                        uint8_t* d_dst, const int64_t* d_dst_off, const int32_t* d_dst_cap,
                        int32_t* d_out_len, int64_t n, int table, int acceleration,
                        lz4m_stream_t stream);

/*
 * lz4m_decompress_solo: lz4m_decompress_batch_ws for ONE block whose input is
 * at most 66 KiB - 64 bytes (src_len_host, the same value as d_src_len[0]),
 * with the compressed block staged in LDS first (the lone decode then waits
 * on no input round trip).  Same bytes and status as the batched decoders
 * (LZ4_decompress_safe, lz4.c:2436-2441); used by lz4m_decompress_safe.
 * The input, its record (d_src_off .. d_dst_cap) and d_status may live in
 * mapped pinned host memory (hipHostMalloc; the device's address of it); the
 * output d_dst must be device memory.  h_out: nullptr, or a mapped pinned
 * host buffer that also receives the decoded bytes at the end of the launch.
 * h_done: nullptr, or a mapped pinned host int the launch sets to 1 with a
 * system-scope release once the status and h_out are in host memory (a
 * caller may poll it instead of synchronising the stream).
 */
int lz4m_decompress_solo(const uint8_t* d_src, const int64_t* d_src_off, const int32_t* d_src_len,
                         uint8_t* d_dst, const int64_t* d_dst_off, const int32_t* d_dst_cap,
                         int32_t* d_status, int32_t src_len_host, uint8_t* h_out, int32_t* h_done,
                         lz4m_stream_t stream);

/*
 * lz4m_compress_solo: lz4m_compress_batch for ONE block of len < 65547 bytes
 * (table U16_HASH4, U32_HASH5 or AUTO), with the block staged in LDS and the
 * compressed block assembled in LDS, so the latency-bound lone parse touches
 * no memory.  Same bytes as the batched kernel; used by the single-call host
 * functions below (lz4m_compress_default / lz4m_compress_block_api).
 * LZ4M_EINVAL when len is out of range.  d_src and d_out_len may live in
 * mapped pinned host memory; h_out: nullptr, or a mapped pinned host buffer
 * that receives the compressed bytes at the end of the launch; d_dst (device
 * memory) receives them instead when h_out is nullptr; h_done: as for
 * lz4m_decompress_solo.
 * *d_out_len: the compressed size (> 0), 0 (does not fit cap), or
 * LZ4M_SOLO_STAGE_FAIL (-2): the workgroup gave up waiting for the block to
 * be staged in LDS (bounded wait) and wrote no bytes -- not a result; redo
 * the call, e.g. through lz4m_compress_batch (what lz4m_host.hip does).
 */
#define LZ4M_SOLO_STAGE_FAIL (-2)
int lz4m_compress_solo(const uint8_t* d_src, int32_t len, uint8_t* d_dst, int32_t cap, int32_t* d_out_len,
                       int table, int acceleration, uint8_t* h_out, int32_t* h_done, lz4m_stream_t stream);

/*
 * Batched one-shot XXH32 (xxhash.c:392-416): d_out[i] = XXH32(block i, seed).
 * Replaces the per-block checksum calls of lz4frame.c:846 (block checksum)
 * and lz4frame.c:1819 (its verification).
 */
int lz4m_xxh32_batch(const uint8_t* d_src, const int64_t* d_off, const int64_t* d_len,
                     uint32_t seed, uint32_t* d_out, int64_t n, lz4m_stream_t stream);

/*
 * XXH32 of one long buffer (the frame content checksum, lz4frame.c:1042 and
 * :1171; XXH32_update/XXH32_digest over the whole content equal the one-shot
 * XXH32 of it, total length mod 2^32, xxhash.c:464-554).  Serial by
 * construction; runs on one wavefront.
 */
int lz4m_xxh32_long(const uint8_t* d_src, int64_t len, uint32_t seed, uint32_t* d_out,
                    lz4m_stream_t stream);

/*
 * Exclusive prefix sum of n int32 sizes (+ per-item constant `add`) into
 * int64 offsets starting at `base`; d_out has n+1 entries (the last one is
 * the total).  d_scratch holds lz4m_scan_scratch_entries(n) int64 values.
 * Used to compact variable-length block outputs.
 */
int64_t lz4m_scan_scratch_entries(int64_t n);
int lz4m_exclusive_scan(const int32_t* d_len, int64_t add, int64_t base, int64_t* d_out,
                        int64_t* d_scratch, int64_t n, lz4m_stream_t stream);

/*
 * Gather variable-length items into one contiguous buffer:
 * d_out[d_out_off[i] .. + d_len[i]) = d_src[d_src_off[i] .. + d_len[i]).
 */
int lz4m_gather(const uint8_t* d_src, const int64_t* d_src_off, const int32_t* d_len,
                uint8_t* d_out, const int64_t* d_out_off, int64_t n, lz4m_stream_t stream);

/*
 * Frame block emission for independent blocks (LZ4F_makeBlock,
 * lz4frame.c:825-850): for block i, with uncompressed bytes
 * d_raw[d_raw_off[i] .. + d_raw_len[i]) and compressed bytes
 * d_cmp[d_cmp_off[i] .. + d_cmp_len[i]) (0 = did not fit), writes at
 * d_frame[d_frame_off[i]] the LE32 block size (bit 31 set for a stored raw
 * block), the payload, and, if block_checksum, the LE32 XXH32 of the payload.
 * d_frame_off comes from lz4m_frame_block_sizes + lz4m_exclusive_scan.
 */
int lz4m_frame_block_sizes(const int32_t* d_raw_len, const int32_t* d_cmp_len, int block_checksum,
                           int32_t* d_rec_len, int64_t n, lz4m_stream_t stream);
int lz4m_frame_emit(const uint8_t* d_raw, const int64_t* d_raw_off, const int32_t* d_raw_len,
                    const uint8_t* d_cmp, const int64_t* d_cmp_off, const int32_t* d_cmp_len,
                    uint8_t* d_frame, const int64_t* d_frame_off, int block_checksum,
                    int64_t n, lz4m_stream_t stream);

/*
 * Single-buffer, HOST-pointer functions with the lz4.h contracts, for a C
 * caller replacing the reference's per-call lz4libs functions one for one
 * (lz4m_host.hip).  Synchronous.  A block of up to 64 KiB (compress: below
 * LZ4_64Klimit; decompress: input below 66 KiB) is a request to the thread's
 * persistent worker kernel (lz4m_single_call_worker below), or, with the
 * worker off, one launch of a lone-block kernel (lz4m_compress_solo /
 * lz4m_decompress_solo).  Either reads the input and its call record from
 * the thread's mapped pinned staging buffer, stages the block in LDS, writes
 * the result back into that buffer itself and releases a done flag the host
 * polls: no stream copies.  Larger inputs copy to the
 * device, run the batched kernel on a batch of one and copy back (device
 * scratch cached per thread).  Throughput comes from the batched functions
 * above.
 *   lz4m_decompress_safe    = LZ4_decompress_safe (lz4.h:191-205)
 *                             replaces _block.c:357-359 with dict size 0;
 *   lz4m_compress_default   = LZ4_compress_default (lz4.h:175-189);
 *   lz4m_compress_block_api = the lz4.block.compress parse (fresh stream,
 *                             LZ4_compress_fast_continue, _block.c:100-109);
 *   lz4m_xxh32              = XXH32 (xxhash.h, xxhash.c:392-416).
 */
int lz4m_decompress_safe(const char* src, char* dst, int compressedSize, int dstCapacity);
int lz4m_compress_default(const char* src, char* dst, int srcSize, int dstCapacity);
int lz4m_compress_block_api(const char* src, char* dst, int srcSize, int dstCapacity, int acceleration);
/*
 * The same two calls with the output left in the calling thread's pinned
 * staging buffer: *out points at it (valid until the thread's next call), so a
 * binding builds its result object with one copy (python-lz4's _block.c
 * allocates the bytes object and copies into it, :230-262, :365-386).
 * lz4m_compress_block_api_staged with header = 4 also writes the LE32 source
 * size just before the output (store_size, _block.c:239-243) and *out points
 * at that header; the return value excludes it.
 */
int lz4m_decompress_safe_staged(const char* src, int compressedSize, int dstCapacity, const char** out);
int lz4m_compress_block_api_staged(const char* src, int srcSize, int dstCapacity, int acceleration, int header,
                                   const char** out);
uint32_t lz4m_xxh32(const void* input, size_t length, uint32_t seed);

/*
 * Streaming XXH32 on the HOST CPU (xxhash.c:437-554, XXH32_reset / _update /
 * _digest; state fields as xxhash.h:264-274).  The frame content checksum is
 * one serial XXH32 stream over all uncompressed bytes (lz4frame.c:1041-1042,
 * :1170-1176, decode :1850, :1961): four multiply-rotate recurrences with no
 * associative combine, so a GPU cannot split it (lz4m_xxh32_long runs it on
 * one wavefront).  lz4.frame runs it here, on a host core, beside the device
 * work.  Pure host code: no device, no allocation.
 */
typedef struct {
    uint32_t total_len_32, large_len, v[4], mem32[4], memsize, reserved;
} lz4m_xxh32_state;
void lz4m_xxh32_host_reset(lz4m_xxh32_state* state, uint32_t seed);
void lz4m_xxh32_host_update(lz4m_xxh32_state* state, const void* input, size_t length);
uint32_t lz4m_xxh32_host_digest(const lz4m_xxh32_state* state);
uint32_t lz4m_xxh32_host(const void* input, size_t length, uint32_t seed);

/* The single-call functions above (lz4m_decompress_safe*, lz4m_compress_*
 * on blocks up to 64 KiB) are served by a persistent one-workgroup kernel per
 * host thread and kind that polls a mailbox in mapped pinned memory, so a
 * call while others keep coming pays no kernel launch; it exits after 2 ms
 * without a call or 2 ms after it started (whatever the call rate: work on a
 * stream that shares its hardware queue waits at most that long) and is
 * started again by the next call.  mode 1 = on (the
 * default; env LZ4M_WORKER=0 turns it off), 0 = off (one launch of the
 * lone-block kernel per call), -1 = query.  Returns the previous mode. */
int lz4m_single_call_worker(int mode);

/* count host copies dst[i] <- src[i] of n[i] bytes, spread over `threads`
 * threads (1..16; one below 4 MiB in total) of the same pool as
 * lz4m_host_copy: the packing and unpacking of lz4.block.compress_many /
 * decompress_many (one H2D and one D2H staging buffer per batch). */
void lz4m_host_copy_many(void* const* dst, const void* const* src, const size_t* n, size_t count, int threads);

/* Diagnostics of the calling thread's workers (tests, tools/probe_worker.py):
 * out[0..7] = decompress / compress mailbox seq, served, quit, and the two
 * launched flags; out[8..11] = per kind the requests its last launch served
 * and how that launch ended (1 idle, 2 quit, 3 lifetime); out[12..15] = per
 * kind the poll's real-time stamps (LZ4M_WORKER_TS builds).  Returns the
 * number of calls (process-wide) the worker path handed to the launch path:
 * a worker that neither served nor exited within 1 s, a stream error, more
 * than three restarts in one call, a failed start, a lone-block staging wait
 * that gave up.  Host memory only: no HIP call. */
int lz4m_single_call_worker_state(uint32_t out[16]);

/* Host memcpy of n bytes split over `threads` threads (1..16; one below
 * 4 MiB); when `hash` is not NULL, one more thread runs
 * lz4m_xxh32_host_update(hash, src, n) over the same source meanwhile.  The
 * staging copies of the drop-in frame calls (lz4.frame.compress / decompress
 * on host bytes, _frame.c:226-228, :1058-1063) and their content checksum
 * (lz4frame.c:1042, :1850) in one pass. */
void lz4m_host_copy(void* dst, const void* src, size_t n, int threads, lz4m_xxh32_state* hash);

/*
 * Block-record walk of an LZ4 frame already in device memory
 * (LZ4F_decompress, lz4frame.c:1643-1701 and 1926-1965): starting at the
 * first record (`pos` = header size), records k = 0.. get d_rec_pos[k] (the
 * payload position), d_rec_len[k] (stored size) and d_rec_raw[k] (bit 31 of
 * the record header: stored uncompressed).  d_result[4] = {records, state,
 * end position, content-checksum position or -1}; state 0 = complete frame,
 * 1 = incomplete, 2 = block size above max_block, 3 = content checksum
 * missing, 4 = more than max_rec records.  Serial over records (one lane).
 * Serves lz4.frame.decompress_device (device-resident frames).
 */
int lz4m_frame_scan(const uint8_t* d_frame, int64_t frame_len, int64_t pos, int block_checksum,
                    int content_checksum, int32_t max_block, int64_t max_rec, int64_t* d_rec_pos,
                    int32_t* d_rec_len, uint8_t* d_rec_raw, int64_t* d_result, lz4m_stream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* LZ4M_H */
