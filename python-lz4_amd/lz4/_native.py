"""Binding to the HIP C-ABI library ``_lz4m.so`` (include/lz4m.h).

The library is loaded into the process's HIP runtime -- the one PyTorch-ROCm
already loaded (same SONAME, libamdhip64.so.7) -- so device pointers of torch
tensors and torch's current HIP stream are passed straight through.

There is no CPU code path behind this module: if the library or a HIP device
is missing, every entry point raises ``RuntimeError``.
"""
from __future__ import annotations

import collections
import ctypes as C
import os
import sys
import threading

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "_lz4m.so")
if os.environ.get("LZ4M_LIB"):   # dev hook: an alternative build of the same library (A/B runs)
    LIB_PATH = os.environ["LZ4M_LIB"]

TABLE_U16_HASH4 = 0
TABLE_U32_HASH5 = 1
TABLE_AUTO = 2
PARSE_PARALLEL = 3   # parallel-parse compressor: valid blocks, ratio of LZ4_compress_default
PARSE_PARALLEL_LARGE = 4   # the same for blocks > 64 KiB
PARSE_PARALLEL_HQ = 5   # PARSE_PARALLEL with the reference's 13-bit table (ratio of LZ4_compress_default)
LINKED_SERIAL = 1        # lz4m_compress_linked_batch modes
LINKED_SPECULATIVE = 2
EINVAL = 0x10000
# decoder selector of lz4m_decompress_batch_sel (include/lz4m.h)
DECODERS = {"auto": 0, "hist": 3, "rows": 4}

_lock = threading.Lock()
_lib = None


def _declare(lib) -> None:
    vp, i32, i64, u32 = C.c_void_p, C.c_int, C.c_int64, C.c_uint32
    sig = {
        "lz4m_compress_bound": ([i32], i32),
        "lz4m_selftest_lds_order": ([], i32),
        "lz4m_version_number": ([], i32),
        "lz4m_version_string": ([], C.c_char_p),
        "lz4m_decompress_batch": ([vp, vp, vp, vp, vp, vp, vp, i64, vp], i32),
        "lz4m_decompress_workspace_bytes": ([], C.c_size_t),
        "lz4m_decompress_batch_ws": ([vp, vp, vp, vp, vp, vp, vp, i64, vp, C.c_size_t, vp], i32),
        "lz4m_decompress_workspace_size": ([i64, i64], C.c_size_t),
        "lz4m_decompress_batch_sel": ([vp, vp, vp, vp, vp, vp, vp, i64, vp, C.c_size_t, i32, vp], i32),
        "lz4m_decompress_batch_dict": ([vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, i64, vp], i32),
        "lz4m_decompress_batch_prefix": ([vp, vp, vp, vp, vp, vp, vp, vp, vp, i64, vp], i32),
        "lz4m_decompress_chain": ([vp, vp, vp, vp, vp, vp, i64, i32, vp], i32),
        "lz4m_compress_batch": ([vp, vp, vp, vp, vp, vp, vp, i64, i32, i32, vp], i32),
        "lz4m_compress_dict_batch": ([vp, vp, vp, vp, vp, vp, vp, vp, i64, i32, vp], i32),
        "lz4m_compress_prefix_batch": ([vp, vp, vp, vp, vp, vp, vp, vp, i64, i32, vp], i32),
        "lz4m_compress_linked_workspace_size": ([i64], C.c_size_t),
        "lz4m_compress_linked_passes": ([], i32),
        "lz4m_pcompress_large_workspace_size": ([i64, i32], C.c_size_t),
        "lz4m_pcompress_large_batch": ([vp, vp, vp, vp, vp, vp, vp, i64, i32, vp, C.c_size_t, vp], i32),
        "lz4m_compress_linked_batch": ([vp, vp, vp, vp, vp, vp, vp, vp, i64, i32, i32, vp, C.c_size_t, vp], i32),
        "lz4m_xxh32_batch": ([vp, vp, vp, u32, vp, i64, vp], i32),
        "lz4m_xxh32_long": ([vp, i64, u32, vp, vp], i32),
        "lz4m_scan_scratch_entries": ([i64], i64),
        "lz4m_exclusive_scan": ([vp, i64, i64, vp, vp, i64, vp], i32),
        "lz4m_gather": ([vp, vp, vp, vp, vp, i64, vp], i32),
        "lz4m_frame_block_sizes": ([vp, vp, i32, vp, i64, vp], i32),
        "lz4m_frame_emit": ([vp, vp, vp, vp, vp, vp, vp, vp, i32, i64, vp], i32),
        "lz4m_frame_scan": ([vp, i64, i64, i32, i32, i32, i64, vp, vp, vp, vp, vp], i32),
        "lz4m_decompress_safe": ([vp, vp, i32, i32], i32),
        "lz4m_compress_default": ([vp, vp, i32, i32], i32),
        "lz4m_compress_block_api": ([vp, vp, i32, i32, i32], i32),
        "lz4m_decompress_safe_staged": ([vp, i32, i32, C.POINTER(vp)], i32),
        "lz4m_compress_block_api_staged": ([vp, i32, i32, i32, i32, C.POINTER(vp)], i32),
        "lz4m_xxh32": ([vp, C.c_size_t, u32], u32),
        "lz4m_xxh32_host_reset": ([vp, u32], None),
        "lz4m_xxh32_host_update": ([vp, vp, C.c_size_t], None),
        "lz4m_xxh32_host_digest": ([vp], u32),
        "lz4m_xxh32_host": ([vp, C.c_size_t, u32], u32),
        "lz4m_host_copy": ([vp, vp, C.c_size_t, i32, vp], None),
        "lz4m_host_copy_many": ([vp, vp, vp, C.c_size_t, i32], None),
        "lz4m_single_call_worker": ([i32], i32),
        "lz4m_single_call_worker_state": ([vp], i32),
    }
    for name, (args, res) in sig.items():
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = res


def lib():
    """The loaded C-ABI library (raises if it is missing)."""
    global _lib
    if _lib is None:
        with _lock:
            if _lib is None:
                if not os.path.exists(LIB_PATH):
                    raise RuntimeError(
                        f"lz4 MI355X backend not built: {LIB_PATH} is missing "
                        "(run `make -C python-lz4_amd/csrc` or __graft_entry__.build())")
                l = C.CDLL(LIB_PATH)
                _declare(l)
                _lib = l
    return _lib


def device() -> torch.device:
    if not torch.cuda.is_available():
        raise RuntimeError("lz4 MI355X backend: no HIP device is visible; this package has no CPU code path")
    return torch.device("cuda", torch.cuda.current_device())


_GPU_SEEN = False


def require_device() -> None:
    """device()'s check for the single-call entry points, which pick the
    current HIP device in C: after the first success it costs nothing
    (torch.cuda.is_available + current_device are ~3 us of a ~50 us call)."""
    global _GPU_SEEN
    if not _GPU_SEEN:
        device()
        _GPU_SEEN = True


def stream_ptr(stream=None) -> int:
    s = stream if stream is not None else torch.cuda.current_stream()
    return int(s.cuda_stream)


def ptr(t: torch.Tensor | None) -> int | None:
    return None if t is None else int(t.data_ptr())


def check(rc: int, what: str) -> None:
    if rc != 0:
        raise RuntimeError(f"{what} failed to launch (code {rc:#x})")


def compress_bound(n: int) -> int:
    """LZ4_compressBound (lz4.h:212)."""
    return 0 if n < 0 or n > 0x7E000000 else n + n // 255 + 16


# ------------------------------------------------------------ raw launchers
def launch_decompress(src, src_off, src_len, dst, dst_off, dst_cap, status, n, stream=None,
                      dict_buf=None, dict_off=None, dict_len=None, decoder: str = "auto",
                      src_bytes: int | None = None) -> None:
    """Batched LZ4_decompress_safe(_usingDict).  ``decoder`` forces one of the
    decoders (``DECODERS``; "auto" picks by batch size); ``src_bytes`` bounds
    the blocks' total compressed size (default: all of ``src``) and sizes the
    large-batch decoder's scratch."""
    L = lib()
    sp = stream_ptr(stream)
    if dict_buf is None:
        work = _workspace(src.device, stream, n, src.numel() if src_bytes is None else src_bytes)
        rc = L.lz4m_decompress_batch_sel(ptr(src), ptr(src_off), ptr(src_len), ptr(dst), ptr(dst_off), ptr(dst_cap),
                                         ptr(status), n, ptr(work), work.numel(), DECODERS[decoder], sp)
    else:
        rc = L.lz4m_decompress_batch_dict(ptr(src), ptr(src_off), ptr(src_len), ptr(dst), ptr(dst_off),
                                          ptr(dst_cap), ptr(dict_buf), ptr(dict_off), ptr(dict_len), ptr(status),
                                          n, sp)
    check(rc, "lz4m_decompress_batch")


_WORK: "collections.OrderedDict" = collections.OrderedDict()
_WORK_STREAMS = 4   # scratch buffers kept (least recently used streams dropped first)


def _workspace(dev, stream, n: int = 0, src_bytes: int = 0) -> torch.Tensor:
    """Decoder scratch (lz4m_decompress_workspace_size), one buffer per
    (device, stream), grown on demand: calls on one stream are ordered, so
    they can share it.  The buffer is allocated on the stream that uses it,
    so when it is dropped (regrowth, eviction, release_workspaces) the
    caching allocator hands its memory only to work ordered after that
    stream's pending launches.  At most _WORK_STREAMS buffers are cached."""
    s = stream if stream is not None else torch.cuda.current_stream(dev)
    key = (dev, int(s.cuda_stream))
    need = int(lib().lz4m_decompress_workspace_size(n, src_bytes))
    w = _WORK.pop(key, None)
    if w is None or w.numel() < need:
        w = None
        with torch.cuda.stream(s):
            w = torch.empty(need, dtype=torch.uint8, device=dev)
    _WORK[key] = w
    while len(_WORK) > _WORK_STREAMS:
        _WORK.popitem(last=False)
    return w


def release_workspaces() -> None:
    """Drop the cached decoder scratch (it grows to ~1/3 of the largest
    compressed batch decoded)."""
    _WORK.clear()


def launch_decompress_prefix(src, src_off, src_len, dst, dst_off, dst_cap, dict_base, dict_len, status, n,
                             stream=None) -> None:
    """Batched LZ4_decompress_safe_usingDict, block i's dictionary the
    dict_len[i] bytes ending at offset dst_off[i] of ``dict_base`` (laid out
    like ``dst``; lz4m_decompress_batch_prefix)."""
    check(lib().lz4m_decompress_batch_prefix(ptr(src), ptr(src_off), ptr(src_len), ptr(dst), ptr(dst_off),
                                             ptr(dst_cap), ptr(dict_base), ptr(dict_len), ptr(status), n,
                                             stream_ptr(stream)),
          "lz4m_decompress_batch_prefix")


def launch_decompress_chain(src, src_off, src_len, raw_mask, dst, status, n, max_block, stream=None) -> None:
    raw = raw_mask.to(torch.uint8)
    rc = lib().lz4m_decompress_chain(ptr(src), ptr(src_off), ptr(src_len), ptr(raw), ptr(dst), ptr(status), n,
                                     max_block, stream_ptr(stream))
    check(rc, "lz4m_decompress_chain")


def launch_compress(src, src_off, src_len, dst, dst_off, dst_cap, out_len, n, table, accel, stream=None,
                    max_len: int | None = None) -> None:
    """Batched compression (lz4m_compress_batch).  PARSE_PARALLEL_LARGE with
    ``max_len`` (the longest block) parses each block as up to 16 segments
    (lz4m_pcompress_large_batch; LZ4M_PC_SEG=0: one wavefront per block)."""
    L = lib()
    if table == PARSE_PARALLEL_LARGE and max_len is not None and os.environ.get("LZ4M_PC_SEG", "1") != "0":
        s = stream if stream is not None else torch.cuda.current_stream(src.device)
        with torch.cuda.stream(s):   # (allocated on the stream that uses it)
            work = torch.empty(int(L.lz4m_pcompress_large_workspace_size(n, max_len)), dtype=torch.uint8,
                               device=src.device)
        rc = L.lz4m_pcompress_large_batch(ptr(src), ptr(src_off), ptr(src_len), ptr(dst), ptr(dst_off),
                                          ptr(dst_cap), ptr(out_len), n, max_len, ptr(work), work.numel(),
                                          stream_ptr(stream))
        check(rc, "lz4m_pcompress_large_batch")
        return
    rc = L.lz4m_compress_batch(ptr(src), ptr(src_off), ptr(src_len), ptr(dst), ptr(dst_off), ptr(dst_cap),
                               ptr(out_len), n, table, accel, stream_ptr(stream))
    check(rc, "lz4m_compress_batch")


def launch_compress_dict(src, src_off, src_len, dict_len, dst, dst_off, dst_cap, out_len, n, accel,
                         stream=None, prefix: bool = False) -> None:
    """lz4.block.compress(dict=) per block; the dictionary tail precedes each block in ``src``.
    ``prefix``: the caller's dictionary ends where the source begins (prefix mode,
    lz4m_compress_prefix_batch)."""
    name = "lz4m_compress_prefix_batch" if prefix else "lz4m_compress_dict_batch"
    rc = getattr(lib(), name)(ptr(src), ptr(src_off), ptr(src_len), ptr(dict_len), ptr(dst), ptr(dst_off),
                              ptr(dst_cap), ptr(out_len), n, accel, stream_ptr(stream))
    check(rc, name)


def launch_compress_linked(src, src_off, src_len, link, dst, dst_off, dst_cap, out_len, n, accel,
                           mode: int = LINKED_SPECULATIVE, stream=None) -> None:
    """Linked-block streams (lz4m_compress_linked_batch).  The speculative
    mode synchronises ``stream`` once per pass."""
    L = lib()
    work = None
    if mode == LINKED_SPECULATIVE:
        work = torch.empty(int(L.lz4m_compress_linked_workspace_size(n)), dtype=torch.uint8, device=src.device)
    rc = L.lz4m_compress_linked_batch(ptr(src), ptr(src_off), ptr(src_len), ptr(link), ptr(dst), ptr(dst_off),
                                      ptr(dst_cap), ptr(out_len), n, accel, mode, ptr(work),
                                      0 if work is None else work.numel(), stream_ptr(stream))
    check(rc, "lz4m_compress_linked_batch")


def launch_xxh32_batch(src, off, length, seed, out, n, stream=None) -> None:
    rc = lib().lz4m_xxh32_batch(ptr(src), ptr(off), ptr(length), seed & 0xFFFFFFFF, ptr(out), n, stream_ptr(stream))
    check(rc, "lz4m_xxh32_batch")


def launch_xxh32_long(src, length, seed, out, stream=None) -> None:
    rc = lib().lz4m_xxh32_long(ptr(src), length, seed & 0xFFFFFFFF, ptr(out), stream_ptr(stream))
    check(rc, "lz4m_xxh32_long")


def exclusive_scan(lengths: torch.Tensor, add: int = 0, base: int = 0, stream=None) -> torch.Tensor:
    """int64 offsets (n+1 entries, last = total) of int32 ``lengths`` (+add each)."""
    n = lengths.numel()
    out = torch.empty(n + 1, dtype=torch.int64, device=lengths.device)
    scratch = torch.empty(int(lib().lz4m_scan_scratch_entries(n)), dtype=torch.int64, device=lengths.device)
    rc = lib().lz4m_exclusive_scan(ptr(lengths), add, base, ptr(out), ptr(scratch), n, stream_ptr(stream))
    check(rc, "lz4m_exclusive_scan")
    return out


def gather(src, src_off, length, out, out_off, n, stream=None) -> None:
    rc = lib().lz4m_gather(ptr(src), ptr(src_off), ptr(length), ptr(out), ptr(out_off), n, stream_ptr(stream))
    check(rc, "lz4m_gather")


def frame_block_sizes(raw_len, cmp_len, block_checksum, rec_len, n, stream=None) -> None:
    rc = lib().lz4m_frame_block_sizes(ptr(raw_len), ptr(cmp_len), int(bool(block_checksum)), ptr(rec_len), n,
                                      stream_ptr(stream))
    check(rc, "lz4m_frame_block_sizes")


def frame_emit(raw, raw_off, raw_len, cmp, cmp_off, cmp_len, frame, frame_off, block_checksum, n,
               stream=None) -> None:
    rc = lib().lz4m_frame_emit(ptr(raw), ptr(raw_off), ptr(raw_len), ptr(cmp), ptr(cmp_off), ptr(cmp_len),
                               ptr(frame), ptr(frame_off), int(bool(block_checksum)), n, stream_ptr(stream))
    check(rc, "lz4m_frame_emit")


def frame_scan(frame, frame_len, pos, block_checksum, content_checksum, max_block, max_rec, rec_pos, rec_len,
               rec_raw, result, stream=None) -> None:
    rc = lib().lz4m_frame_scan(ptr(frame), frame_len, pos, int(bool(block_checksum)), int(bool(content_checksum)),
                               max_block, max_rec, ptr(rec_pos), ptr(rec_len), ptr(rec_raw), ptr(result),
                               stream_ptr(stream))
    check(rc, "lz4m_frame_scan")


# ------------------------------------------------------------ host XXH32
def _addr(buf):
    """(address, length, keep-alive) of any contiguous buffer, no copy."""
    import numpy as np
    if isinstance(buf, torch.Tensor):
        return buf.data_ptr(), buf.numel() * buf.element_size(), buf
    a = np.frombuffer(memoryview(buf).cast("B"), dtype=np.uint8)
    return a.ctypes.data, a.nbytes, a


class HostXXH32:
    """Streaming XXH32 on a host core (include/lz4m.h lz4m_xxh32_host_*).
    ctypes drops the GIL during each update, so it runs beside GPU work
    issued from other threads."""

    def __init__(self, seed: int = 0):
        self._st = (C.c_uint32 * 12)()
        lib().lz4m_xxh32_host_reset(self._st, seed & 0xFFFFFFFF)

    def update(self, buf, n: int | None = None) -> None:
        ptr, ln, keep = _addr(buf)
        lib().lz4m_xxh32_host_update(self._st, ptr, ln if n is None else n)
        del keep

    def update_ptr(self, ptr: int, n: int) -> None:
        lib().lz4m_xxh32_host_update(self._st, ptr, n)

    def digest(self) -> int:
        return int(lib().lz4m_xxh32_host_digest(self._st))


def xxh32_host(buf, seed: int = 0) -> int:
    """One-shot XXH32 of a host buffer on the calling host core."""
    ptr, ln, keep = _addr(buf)
    r = int(lib().lz4m_xxh32_host(ptr, ln, seed & 0xFFFFFFFF))
    del keep
    return r


_PIN = {}
_PIN_LOCK = threading.Lock()


def _pinned_pair(chunk: int):
    """Two pinned host buffers of `chunk` bytes from a process-wide pool
    (pinning 128 MiB costs tens of ms: never per call or per thread)."""
    with _PIN_LOCK:
        free = _PIN.setdefault(chunk, [])
        if free:
            return free.pop()
    return [torch.empty(chunk, dtype=torch.uint8, pin_memory=True) for _ in range(2)]


def _pinned_release(chunk: int, bufs) -> None:
    with _PIN_LOCK:
        _PIN.setdefault(chunk, []).append(bufs)


def xxh32_of_device(t: torch.Tensor, n: int, seed: int = 0, wait_stream=None, chunk: int = 64 << 20,
                    wait_event=None) -> int:
    """XXH32 of the first n bytes of a device tensor, hashed on a host core:
    chunks are copied to two pinned buffers on a side stream, each hashed
    while the next one copies (PCIe ~50 GB/s against ~13 GB/s of hashing).
    ``wait_event``: an event recorded when t was ready (preferred: a caller
    running this in a thread records it before queueing more work), else
    ``wait_stream``: the stream that produced t (default: current)."""
    st = HostXXH32(seed)
    if n <= 0:
        return st.digest()
    dev = t.device
    # a high-priority copy stream (LZ4M_HASH_STREAM_PRIORITY, default -1):
    # HIP multiplexes same-priority streams over a few hardware queues
    # (GPU_MAX_HW_QUEUES), and a copy stream on the compressing stream's
    # queue ran its copies after the kernel -- the config-4 frame with a
    # content checksum measured 8.4 GiB/s in the full bench, 11.9 with this
    side = torch.cuda.Stream(dev, priority=int(os.environ.get("LZ4M_HASH_STREAM_PRIORITY", "-1")))
    if wait_event is not None:
        side.wait_event(wait_event)
    else:
        side.wait_stream(wait_stream if wait_stream is not None else torch.cuda.current_stream(dev))
    bufs = _pinned_pair(chunk)
    evs = [torch.cuda.Event(), torch.cuda.Event()]
    spans = [(lo, min(n, lo + chunk)) for lo in range(0, n, chunk)]
    flat = t.view(-1)

    def issue(i):
        lo, hi = spans[i]
        with torch.cuda.stream(side):
            bufs[i & 1][: hi - lo].copy_(flat[lo:hi], non_blocking=True)
            evs[i & 1].record(side)

    try:
        issue(0)
        for i, (lo, hi) in enumerate(spans):
            if i + 1 < len(spans):
                issue(i + 1)   # its buffer was hashed in iteration i - 1
            evs[i & 1].synchronize()
            st.update_ptr(bufs[i & 1].data_ptr(), hi - lo)
    finally:
        for e in evs:
            e.synchronize()
        _pinned_release(chunk, bufs)
    return st.digest()


def xxh32_of_device_spans(t: torch.Tensor, spans, seed: int = 0, state: "HostXXH32 | None" = None,
                          chunk: int = 64 << 20) -> "HostXXH32":
    """Continue an XXH32 on a host core over device bytes t[lo:hi] of each
    span (lo, hi, event) in order, the spans contiguous: a span's copies are
    queued behind its event (the device work that writes those bytes), so
    the hash follows the producer instead of waiting for all of it.  Returns
    the state (``.digest()`` ends it).  The copy and pinned-buffer scheme is
    xxh32_of_device's."""
    st = state if state is not None else HostXXH32(seed)
    pieces = []
    for lo, hi, ev in spans:
        for a in range(lo, hi, chunk):
            pieces.append((a, min(hi, a + chunk), ev))
    if not pieces:
        return st
    dev = t.device
    side = torch.cuda.Stream(dev, priority=int(os.environ.get("LZ4M_HASH_STREAM_PRIORITY", "-1")))
    bufs = _pinned_pair(chunk)
    evs = [torch.cuda.Event(), torch.cuda.Event()]
    flat = t.view(-1)
    waited = set()

    def issue(i):
        lo, hi, ev = pieces[i]
        with torch.cuda.stream(side):
            if ev is not None and id(ev) not in waited:
                side.wait_event(ev)
                waited.add(id(ev))
            bufs[i & 1][: hi - lo].copy_(flat[lo:hi], non_blocking=True)
            evs[i & 1].record(side)

    try:
        issue(0)
        for i, (lo, hi, _ev) in enumerate(pieces):
            if i + 1 < len(pieces):
                issue(i + 1)
            evs[i & 1].synchronize()
            st.update_ptr(bufs[i & 1].data_ptr(), hi - lo)
    finally:
        for e in evs:
            e.synchronize()
        _pinned_release(chunk, bufs)
    return st


# ------------------------------------------------------------ host <-> device
# Large host <-> device moves (the drop-in frame calls on Python bytes) go
# through two pinned chunks: lz4m_host_copy fills / drains a chunk with a few
# host threads while the other chunk's DMA runs on a side stream; a content
# checksum can ride along (hashed from the chunk while it is copied).
_BIG = 32 << 20
_CHUNK = 64 << 20


def _copy_threads() -> int:
    try:
        vis = len(os.sched_getaffinity(0))
    except AttributeError:
        vis = os.cpu_count() or 1
    share = int(os.environ.get("OMP_NUM_THREADS", "16") or 16)
    return max(1, min(8, vis, share) - 1)   # one core left for the hash thread


def to_device(buf, dev=None, pad: int = 0) -> torch.Tensor:
    """Copy a bytes-like object to a device uint8 tensor (+pad zero bytes)."""
    dev = dev or device()
    mv = memoryview(buf).cast("B")
    n = mv.nbytes
    out = torch.empty(n + pad, dtype=torch.uint8, device=dev)
    if n >= _BIG:
        src, _, keep = _addr(mv)
        bufs = _pinned_pair(_CHUNK)
        evs = [None, None]
        side = torch.cuda.Stream(dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        thr = _copy_threads()
        try:
            for i, lo in enumerate(range(0, n, _CHUNK)):
                hi = min(n, lo + _CHUNK)
                b = bufs[i & 1]
                if evs[i & 1] is not None:
                    evs[i & 1].synchronize()   # this chunk's previous DMA has read it
                lib().lz4m_host_copy(b.data_ptr(), src + lo, hi - lo, thr, None)
                with torch.cuda.stream(side):
                    out[lo:hi].copy_(b[: hi - lo], non_blocking=True)
                    evs[i & 1] = torch.cuda.Event()
                    evs[i & 1].record(side)
            torch.cuda.current_stream(dev).wait_stream(side)
        finally:
            for e in evs:
                if e is not None:
                    e.synchronize()
            _pinned_release(_CHUNK, bufs)
            del keep
    elif n:
        import warnings
        with warnings.catch_warnings():   # read-only bytes: shared, only read
            warnings.simplefilter("ignore")
            host = torch.frombuffer(mv, dtype=torch.uint8)
        out[:n].copy_(host, non_blocking=False)
    if pad:
        out[n:].zero_()
    return out


_PyBytes_New = C.pythonapi.PyBytes_FromStringAndSize
_PyBytes_New.restype = C.py_object
_PyBytes_New.argtypes = [C.c_void_p, C.c_ssize_t]
_PyByteArray_New = C.pythonapi.PyByteArray_FromStringAndSize
_PyByteArray_New.restype = C.py_object
_PyByteArray_New.argtypes = [C.c_void_p, C.c_ssize_t]
_BYTES_DATA = sys.getsizeof(b"") - 1   # offset of a bytes object's data (CPython: the header, then the bytes)


_MADV_HUGEPAGE = 14
_HUGE = 2 << 20
_libc = None


def _advise_huge(addr: int, n: int) -> None:
    """Ask for transparent huge pages on the 2 MiB-aligned interior of a
    fresh host buffer (best effort).  Its first touch is the copy that fills
    it: with 4 KiB pages 8 GiB filled at 18 GB/s (a fault and a page zeroing
    per 4 KiB), with huge pages at 97 GB/s on the same 7 copy threads
    (profiles/r05/r05ab/fault.log; the GPU box runs THP in madvise mode)."""
    global _libc
    a = (addr + _HUGE - 1) & ~(_HUGE - 1)
    ln = (addr + n - a) & ~(_HUGE - 1)
    if ln <= 0 or os.environ.get("LZ4M_HUGEPAGES", "1") == "0":
        return
    if _libc is None:
        _libc = C.CDLL(None, use_errno=True)
        _libc.madvise.argtypes = [C.c_void_p, C.c_size_t, C.c_int]
        _libc.madvise.restype = C.c_int
    _libc.madvise(a, ln, _MADV_HUGEPAGE)


def _new_host_buffer(n: int, as_bytearray: bool):
    """An uninitialised bytes (or bytearray) of n bytes and its data address
    (filled before anyone else sees it; huge pages asked for when large)."""
    if as_bytearray:
        ba = _PyByteArray_New(None, n)
        addr = C.addressof((C.c_char * n).from_buffer(ba))
        obj = ba
    else:
        obj = _PyBytes_New(None, n)
        addr = id(obj) + _BYTES_DATA
    if n >= 4 * _HUGE:
        _advise_huge(addr, n)
    return obj, addr


def to_host_bytes(t: torch.Tensor, n: int, as_bytearray: bool = False, hash_seed: int | None = None):
    """The first n bytes of a device tensor as a new bytes (or bytearray).
    hash_seed: also return the XXH32 of those bytes, hashed on a host core
    from each staged chunk while it is copied -> (bytes, digest)."""
    if n <= 0:
        out = bytearray() if as_bytearray else b""
        return (out, HostXXH32(hash_seed).digest()) if hash_seed is not None else out
    if n < _BIG:
        h = t.view(-1)[:n].cpu().numpy()
        out = bytearray(h.tobytes()) if as_bytearray else h.tobytes()
        return (out, xxh32_host(out, hash_seed)) if hash_seed is not None else out
    out, dst = _new_host_buffer(n, as_bytearray)
    st = HostXXH32(hash_seed) if hash_seed is not None else None
    dev = t.device
    flat = t.view(-1)
    side = torch.cuda.Stream(dev)
    side.wait_stream(torch.cuda.current_stream(dev))
    bufs = _pinned_pair(_CHUNK)
    evs = [torch.cuda.Event(), torch.cuda.Event()]
    spans = [(lo, min(n, lo + _CHUNK)) for lo in range(0, n, _CHUNK)]
    thr = _copy_threads()

    def issue(i):
        lo, hi = spans[i]
        with torch.cuda.stream(side):
            bufs[i & 1][: hi - lo].copy_(flat[lo:hi], non_blocking=True)
            evs[i & 1].record(side)

    try:
        issue(0)
        for i, (lo, hi) in enumerate(spans):
            if i + 1 < len(spans):
                issue(i + 1)   # its buffer was drained in iteration i - 1
            evs[i & 1].synchronize()
            lib().lz4m_host_copy(dst + lo, bufs[i & 1].data_ptr(), hi - lo, thr, None if st is None else st._st)
    finally:
        for e in evs:
            e.synchronize()
        _pinned_release(_CHUNK, bufs)
    return (out, st.digest()) if st is not None else out

def host_copy_many(dsts, srcs, lens) -> None:
    """dsts[i] <- srcs[i], lens[i] bytes each (host addresses), over the copy
    pool (include/lz4m.h lz4m_host_copy_many)."""
    n = len(lens)
    if n == 0:
        return
    D = (C.c_void_p * n)(*dsts)
    S = (C.c_void_p * n)(*srcs)
    L = (C.c_size_t * n)(*lens)
    lib().lz4m_host_copy_many(D, S, L, n, _copy_threads())
