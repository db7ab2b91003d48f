"""``lz4.block`` on the MI355X codec.

Drop-in for the reference CPython extension ``lz4/block/_block.c``: same
function names, argument handling, return types, size header and exception
messages (``_block.c:127-400``).  Every call runs the HIP kernels of
``_lz4m.so``; single calls pay one H2D + launch + D2H, so the batched
entry points (``compress_batch`` / ``decompress_batch`` on device tensors,
``compress_many`` / ``decompress_many`` on host buffers) are the throughput
path.
"""
from __future__ import annotations

import ctypes as C
import operator
import os

import torch

from .. import _native as N

INT_MAX = 2**31 - 1
INT_MIN = -(2**31)
_HDR = 4   # _block.c:82, LE32 uncompressed size prefix

# lz4hc.h:47-50, exported by _block.c:508-511
HC_LEVEL_MIN = 3
HC_LEVEL_DEFAULT = 9
HC_LEVEL_OPT_MIN = 10
HC_LEVEL_MAX = 12


class LZ4BlockError(Exception):
    """Call to LZ4 library failed."""


LZ4BlockError.__module__ = "_block"


# -------------------------------------------------------------- arg helpers
def _c_int(value, name: str) -> int:
    """PyArg 'i' conversion: __index__ required, C int range enforced."""
    try:
        v = operator.index(value)
    except TypeError:
        raise TypeError(f"'{type(value).__name__}' object cannot be interpreted as an integer") from None
    if v > INT_MAX:
        raise OverflowError("signed integer is greater than maximum")
    if v < INT_MIN:
        raise OverflowError("signed integer is less than minimum")
    return v


def _buffer(obj, name: str = "source") -> memoryview:
    """PyArg 'y*' conversion: any contiguous buffer; str is rejected."""
    if isinstance(obj, str):
        raise TypeError(f"a bytes-like object is required, not '{type(obj).__name__}'")
    mv = memoryview(obj)
    if not mv.c_contiguous:
        raise BufferError("memoryview: underlying buffer is not C-contiguous")
    return mv.cast("B") if mv.format != "B" or mv.ndim != 1 else mv


def _mode_accel(mode, acceleration: int) -> int:
    if not isinstance(mode, str):
        raise TypeError(f"compress() argument 'mode' must be str, not {type(mode).__name__}")
    if mode == "default":
        return 1
    if mode == "fast":
        return acceleration
    if mode == "high_compression":
        raise NotImplementedError(
            "mode='high_compression' (LZ4 HC) is outside the MI355X codec's scope; "
            "use mode='default' or mode='fast'")
    raise ValueError(f"Invalid mode argument: {mode}. Must be one of: standard, fast, high_compression")


_probe = b"lz4m"
_BYTES_DATA = C.cast(C.c_char_p(_probe), C.c_void_p).value - id(_probe)   # measured, not assumed
del _probe


def _addr(view: memoryview):
    """Address of a contiguous host buffer (read-only ones too), None if empty.
    A whole bytes object (its data offset measured at import) or a writable
    buffer takes a fast path; numpy's .ctypes (~2.6 us) serves the rest."""
    if not view.nbytes:
        return None
    obj = view.obj
    if type(obj) is bytes and view.nbytes == len(obj):
        return id(obj) + _BYTES_DATA   # CPython: the bytes' data sits at a fixed offset in the object
    if not view.readonly:
        return C.addressof(C.c_char.from_buffer(view))
    return int(np.frombuffer(view, dtype=np.uint8).ctypes.data)


def _i64(vals, dev) -> torch.Tensor:
    return torch.tensor(vals, dtype=torch.int64, device=dev)


def _i32(vals, dev) -> torch.Tensor:
    return torch.tensor(vals, dtype=torch.int32, device=dev)


# ------------------------------------------------------------ single calls
def compress(source, mode="default", store_size=True, acceleration=1, compression=9,
             return_bytearray=False, dict=None):
    """compress(source, mode='default', acceleration=1, compression=0, return_bytearray=False)

    Compress source into one LZ4 block (``_block.c:127-271``), output
    byte-identical to the reference: ``lz4.block.compress`` resets an
    ``LZ4_stream_t`` and calls ``LZ4_compress_fast_continue`` (byU32 table,
    hash5), which ``TABLE_U32_HASH5`` reproduces.  With ``dict`` (any
    length, even empty) the stream is first loaded with ``LZ4_loadDict``
    (``_block.c:101-104``, ``lz4.c:1541-1581``) -- lz4m_compress_dict_batch.
    """
    src = _buffer(source)
    acceleration = _c_int(acceleration, "acceleration")
    _c_int(compression, "compression")
    if src.nbytes > INT_MAX:
        raise OverflowError("Input too large for LZ4 API")
    d = None
    if dict is not None:
        d = _buffer(dict, "dict")
        if d.nbytes > INT_MAX:
            raise OverflowError("Dictionary too large for LZ4 API")
    accel = _mode_accel(mode, acceleration)
    if d is None:   # one call: lz4m_compress_block_api (one launch on mapped pinned staging)
        N.require_device()
        n = src.nbytes
        hdr = _HDR if store_size else 0
        p = C.c_void_p()
        # the output (after the size header) stays in the thread's pinned buffer: one copy into the result
        r = N.lib().lz4m_compress_block_api_staged(_addr(src), n, max(N.compress_bound(n), 1), accel, hdr,
                                                   C.byref(p))
        if r <= 0:
            raise LZ4BlockError("Compression failed")
        out = C.string_at(p.value, hdr + r)
        return bytearray(out) if return_bytearray else out
    # dictionary memory that ends where the source begins: the reference's
    # LZ4_compress_fast_continue sees dictEnd == source and takes prefix mode
    # (lz4.c:1671-1676; LZ4_loadDict keeps no dictionary below 8 bytes)
    prefix = d.nbytes >= 8 and src.nbytes > 0 and _addr(d) + d.nbytes == _addr(src)
    out = compress_many([src], accel=accel, store_size=bool(store_size), as_bytearray=bool(return_bytearray),
                        dict=d, dict_prefix=prefix)[0]
    if out is None:
        raise LZ4BlockError("Compression failed")
    return out


def decompress(source, uncompressed_size=-1, return_bytearray=False, dict=None):
    """decompress(source, uncompressed_size=-1, return_bytearray=False)

    Decompress one LZ4 block (``_block.c:273-400``).  With
    ``uncompressed_size >= 0`` the whole source is the block and the value is
    a capacity; otherwise a LE32 size header leads the block and the decoded
    size must equal it.
    """
    src = _buffer(source)
    uncompressed_size = _c_int(uncompressed_size, "uncompressed_size")
    if src.nbytes > INT_MAX:
        raise OverflowError("Input too large for LZ4 API")
    dview = None
    if dict is not None:
        dview = _buffer(dict, "dict")
        if dview.nbytes > INT_MAX:
            raise OverflowError("Dictionary too large for LZ4 API")
    if dview is None or not dview.nbytes:   # one call: lz4m_decompress_safe
        N.require_device()
        if uncompressed_size >= 0:
            cap, skip = uncompressed_size, 0
        else:
            if src.nbytes < _HDR:
                raise ValueError("Input source data size too small")
            cap = int.from_bytes(src[:4], "little")
            if cap > INT_MAX:
                raise ValueError(f"Invalid size: 0x{cap}")
            skip = _HDR
        sp = _addr(src)
        p = C.c_void_p()
        # the output stays in the thread's pinned buffer: one copy into the result
        r = N.lib().lz4m_decompress_safe_staged(None if sp is None else sp + skip, src.nbytes - skip, cap, C.byref(p))
        if r < 0:
            raise LZ4BlockError(
                "Decompression failed: corrupt input or insufficient space in destination buffer. "
                f"Error code: {-r}")
        if r != cap and uncompressed_size < 0:
            raise LZ4BlockError(f"Decompressor wrote {r} bytes, but {cap} bytes expected from header")
        out = C.string_at(p.value, r) if r else b""
        return bytearray(out) if return_bytearray else out
    res = decompress_many([src], uncompressed_size=uncompressed_size, dict=dview,
                          as_bytearray=bool(return_bytearray), raise_errors=True)
    return res[0]


# ---------------------------------------------------- host-buffer batches
# A call from host memory moves everything through one pinned staging buffer
# per thread and device: block table + payload in ONE host-to-device copy,
# status/lengths + output in ONE device-to-host copy (the reference does one
# malloc + memcpy per call, _block.c:215, :256-263; a launch per small tensor
# would dominate a 64 KiB call).
import threading

import numpy as np

_tls = threading.local()
_ALIGN = 256


def _al(x: int) -> int:
    return (x + _ALIGN - 1) // _ALIGN * _ALIGN


def _stage(dev, host_bytes: int, dev_bytes: int):
    """(pinned host uint8, device uint8) buffers of at least these sizes,
    cached per thread and device, grown geometrically."""
    cache = getattr(_tls, "stage", None)
    if cache is None:
        cache = _tls.stage = {}
    h, d = cache.get(dev, (None, None))
    if h is None or h.numel() < host_bytes:
        h = torch.empty(max(host_bytes, 2 * (h.numel() if h is not None else 0), 1 << 20), dtype=torch.uint8,
                        pin_memory=True)
    if d is None or d.numel() < dev_bytes:
        d = torch.empty(max(dev_bytes, 2 * (d.numel() if d is not None else 0), 1 << 20), dtype=torch.uint8,
                        device=dev)
    cache[dev] = (h, d)
    return h, d


class _Layout:
    """Byte layout of one staged batch: n-entry tables, then payload, then
    (device only) the n-entry result table and the output region."""

    def __init__(self, n: int, payload: int, out_bytes: int):
        self.src_off = 0
        self.src_len = _al(8 * n)
        self.dst_off = self.src_len + _al(4 * n)
        self.dst_cap = self.dst_off + _al(8 * n)
        self.payload = self.dst_cap + _al(4 * n)
        self.h2d = self.payload + payload                  # bytes copied in
        self.result = _al(self.h2d)
        self.out = self.result + _al(4 * n)
        self.total = self.out + max(out_bytes, 1)            # device bytes
        self.d2h = self.total - self.result                  # bytes copied out


def _stage_in(dev, views, offs, lens, d_off, caps, skip=None):
    """Stage tables + packed payload, copy them to the device in one go;
    returns (layout, host, device) with the device views ready to launch on.
    ``views`` are packed back to back; ``offs``/``lens`` (one per block) say
    where the blocks are in that payload."""
    n = len(offs)
    payload = sum(v.nbytes for v in views)
    lay = _Layout(n, payload, sum(caps))
    h, d = _stage(dev, lay.total, lay.total)
    hn = h.numpy()
    hn[lay.src_off:lay.src_off + 8 * n].view(np.int64)[:] = offs if skip is None else np.add(offs, skip)
    hn[lay.src_len:lay.src_len + 4 * n].view(np.int32)[:] = lens if skip is None else np.subtract(lens, skip)
    hn[lay.dst_off:lay.dst_off + 8 * n].view(np.int64)[:] = d_off
    hn[lay.dst_cap:lay.dst_cap + 4 * n].view(np.int32)[:] = caps
    pos = lay.payload
    if len(views) >= _MANY and payload >= _MANY_BYTES:   # one pooled native copy of every block
        base = h.data_ptr()
        dsts, srcs, ns = [], [], []
        for v in views:
            dsts.append(base + pos)
            srcs.append(_addr(v))
            ns.append(v.nbytes)
            pos += v.nbytes
        N.host_copy_many(dsts, srcs, ns)
    else:
        for v in views:
            hn[pos:pos + v.nbytes] = np.frombuffer(v, dtype=np.uint8)
            pos += v.nbytes
    d[:lay.h2d].copy_(h[:lay.h2d], non_blocking=True)
    return lay, h, d


# batches of at least this many blocks and bytes pack and unpack through one
# pooled native copy (lz4m_host_copy_many) instead of a numpy copy per block
_MANY, _MANY_BYTES = 32, 4 << 20


def _results_many(host, d_off, sizes, hdr_lens, as_bytearray):
    """New bytes (or bytearrays) for blocks of sizes[i] >= 0 bytes at host
    offset d_off[i] (None where sizes[i] < 0), prefixed with the LE32 of
    hdr_lens[i] when hdr_lens is given; filled by one pooled copy."""
    base = host.ctypes.data
    res, dsts, srcs, ns = [], [], [], []
    for i, L in enumerate(sizes):
        if L < 0:
            res.append(None)
            continue
        hdr = 4 if hdr_lens is not None else 0
        b, addr = N._new_host_buffer(hdr + L, as_bytearray) if hdr + L else ((bytearray() if as_bytearray else b""), 0)
        if hdr:
            C.memmove(addr, hdr_lens[i].to_bytes(4, "little"), 4)
        if L:
            dsts.append(addr + hdr)
            srcs.append(base + int(d_off[i]))
            ns.append(L)
        res.append(b)
    N.host_copy_many(dsts, srcs, ns)
    return res


def _dev_views(lay: _Layout, d: torch.Tensor, n: int):
    def sl(a, nb, dt):
        return d[a:a + nb].view(dt)
    return (sl(lay.payload, max(lay.h2d - lay.payload, 1), torch.uint8), sl(lay.src_off, 8 * n, torch.int64),
            sl(lay.src_len, 4 * n, torch.int32), d[lay.out:lay.total], sl(lay.dst_off, 8 * n, torch.int64),
            sl(lay.dst_cap, 4 * n, torch.int32), sl(lay.result, 4 * n, torch.int32))


def _stage_out(lay: _Layout, h: torch.Tensor, d: torch.Tensor, n: int):
    """One device-to-host copy of the result table + output region."""
    h[lay.result:lay.total].copy_(d[lay.result:lay.total], non_blocking=True)
    torch.cuda.current_stream(d.device).synchronize()
    hn = h.numpy()
    return hn[lay.result:lay.result + 4 * n].view(np.int32).tolist(), hn[lay.out:lay.total]


def compress_many(blocks, accel: int = 1, store_size: bool = True, as_bytearray: bool = False,
                  table: int = N.TABLE_U32_HASH5, dict=None, dict_prefix: bool = False):
    """Compress a sequence of host buffers as independent blocks in one
    launch.  Returns a list of bytes (None for a block that failed, i.e.
    input larger than LZ4_MAX_INPUT_SIZE).  ``dict`` (a buffer, possibly
    empty): every block is compressed as lz4.block.compress(dict=dict) does;
    the dictionary's last 64 KiB are staged in front of each block.
    ``dict_prefix``: compress as the reference does when the dictionary's
    memory ends where each source begins (prefix mode, lz4.c:1671)."""
    views = [_buffer(b) for b in blocks]
    dev = N.device()
    n = len(views)
    if n == 0:
        return []
    lens = [v.nbytes for v in views]
    caps = [max(N.compress_bound(L), 1) for L in lens]
    d_off = np.concatenate([[0], np.cumsum(caps[:-1], dtype=np.int64)]) if n > 1 else np.zeros(1, np.int64)
    if dict is None:
        offs = np.concatenate([[0], np.cumsum(lens[:-1], dtype=np.int64)]) if n > 1 else np.zeros(1, np.int64)
        payload = views
    else:
        dv = _buffer(dict, "dict")
        tail = dv[-65536:] if dv.nbytes >= 8 else dv[:0]   # LZ4_loadDict keeps the last 64 KiB (lz4.c:1568)
        t = tail.nbytes
        offs = np.arange(1, n + 1, dtype=np.int64) * t + (np.concatenate([[0], np.cumsum(lens[:-1], dtype=np.int64)])
                                                            if n > 1 else np.zeros(1, np.int64))
        payload = [x for v in views for x in (tail, v)]
    lay, h, d = _stage_in(dev, payload, offs, lens, d_off, caps)
    d_src, src_off, src_len, d_dst, dst_off, dst_cap, out_len = _dev_views(lay, d, n)
    if dict is None:
        N.launch_compress(d_src, src_off, src_len, d_dst, dst_off, dst_cap, out_len, n, table, accel)
    else:
        dict_len = torch.full((n,), dv.nbytes, dtype=torch.int32, device=dev)
        N.launch_compress_dict(d_src, src_off, src_len, dict_len, d_dst, dst_off, dst_cap, out_len, n, accel,
                               prefix=dict_prefix and dv.nbytes >= 8)
    olen, host = _stage_out(lay, h, d, n)
    if n >= _MANY and sum(L for L in olen if L > 0) >= _MANY_BYTES:
        return _results_many(host, d_off, [L if L > 0 else -1 for L in olen], lens if store_size else None,
                             as_bytearray)
    res = []
    for i in range(n):
        L = olen[i]
        if L <= 0:
            res.append(None)
            continue
        o = int(d_off[i])
        body = host[o:o + L].tobytes()
        if store_size:
            body = lens[i].to_bytes(4, "little") + body
        res.append(bytearray(body) if as_bytearray else body)
    return res


def decompress_many(blocks, uncompressed_size=-1, dict=None, as_bytearray: bool = False,
                    raise_errors: bool = True):
    """Decompress a sequence of host buffers in one launch.

    ``uncompressed_size`` is one int for all blocks or a list; negative
    means "read the LE32 size header".  With ``raise_errors`` the first
    failing block raises the reference's exception; otherwise failing blocks
    yield the LZ4BlockError instance in their slot.
    """
    views = [_buffer(b) for b in blocks]
    n = len(views)
    if n == 0:
        return []
    sizes = list(uncompressed_size) if isinstance(uncompressed_size, (list, tuple)) else [uncompressed_size] * n
    caps, skip, errors = [], [], [None] * n
    for i, (v, us) in enumerate(zip(views, sizes)):
        if us >= 0:
            caps.append(us)
            skip.append(0)
        else:
            if v.nbytes < _HDR:
                err = ValueError("Input source data size too small")
                if raise_errors:
                    raise err
                errors[i] = err
                caps.append(0)
                skip.append(0)
                continue
            cap = int.from_bytes(v[:4], "little")
            if cap > INT_MAX:
                err = ValueError(f"Invalid size: 0x{cap}")
                if raise_errors:
                    raise err
                errors[i] = err
                caps.append(0)
                skip.append(0)
                continue
            caps.append(cap)
            skip.append(_HDR)
    dev = N.device()
    lens = [v.nbytes for v in views]
    offs = np.concatenate([[0], np.cumsum(lens[:-1], dtype=np.int64)]) if n > 1 else np.zeros(1, np.int64)
    d_off = np.concatenate([[0], np.cumsum(caps[:-1], dtype=np.int64)]) if n > 1 else np.zeros(1, np.int64)
    lay, h, d = _stage_in(dev, views, offs, lens, d_off, caps, skip=skip)
    d_src, src_off, src_len, d_dst, dst_off, dst_cap, status = _dev_views(lay, d, n)
    if dict is not None and _buffer(dict).nbytes:
        dv = _buffer(dict)
        d_dict = N.to_device(dv, dev)
        N.launch_decompress(d_src, src_off, src_len, d_dst, dst_off, dst_cap, status, n,
                            dict_buf=d_dict, dict_off=torch.zeros(n, dtype=torch.int64, device=dev),
                            dict_len=torch.full((n,), dv.nbytes, dtype=torch.int32, device=dev))
    else:
        N.launch_decompress(d_src, src_off, src_len, d_dst, dst_off, dst_cap, status, n,
                            src_bytes=int(sum(lens)))
    st, host = _stage_out(lay, h, d, n)
    if n >= _MANY and all(e is None for e in errors) and all(
            r >= 0 and (r == c or us >= 0) for r, c, us in zip(st, caps, sizes)) and sum(st) >= _MANY_BYTES:
        return _results_many(host, d_off, st, None, as_bytearray)   # every block decoded as asked
    res = []
    for i in range(n):
        if errors[i] is not None:
            res.append(errors[i])
            continue
        r = st[i]
        err = None
        if r < 0:
            err = LZ4BlockError(
                "Decompression failed: corrupt input or insufficient space in destination buffer. "
                f"Error code: {-r}")
        elif r != caps[i] and sizes[i] < 0:
            err = LZ4BlockError(f"Decompressor wrote {r} bytes, but {caps[i]} bytes expected from header")
        if err is not None:
            if raise_errors:
                raise err
            res.append(err)
            continue
        o = int(d_off[i])
        body = host[o:o + r].tobytes() if r else b""
        res.append(bytearray(body) if as_bytearray else body)
    return res


# ------------------------------------------------- device-resident batches
def compress_batch(src: torch.Tensor, src_off: torch.Tensor, src_len: torch.Tensor, *,
                   table: str | int = "block", acceleration: int = 1, dst: torch.Tensor | None = None,
                   dst_off: torch.Tensor | None = None, dst_cap: torch.Tensor | None = None, stream=None):
    """Compress n device-resident blocks in one stream-ordered launch.

    ``src`` uint8 (HBM), ``src_off`` int64[n], ``src_len`` int32[n].
    ``table``: "block" (lz4.block.compress parse, byU32/hash5), "default"
    (LZ4_compress_default's choice by size; byU16/hash4 below 65547 B) or a
    TABLE_* constant.  Output slots default to LZ4_compressBound(len) each.
    Returns (dst, dst_off, out_len) with out_len int32[n] (0 = did not fit).
    No host synchronisation.
    """
    tab = {"block": N.TABLE_U32_HASH5, "default": N.TABLE_AUTO, "u16": N.TABLE_U16_HASH4}.get(table, table)
    n = src_off.numel()
    dev = src.device
    if dst_cap is None:
        dst_cap = (src_len.to(torch.int64) + src_len.to(torch.int64) // 255 + 16).to(torch.int32)
    if dst_off is None:
        dst_off = N.exclusive_scan(dst_cap, stream=stream)[:n]
    if dst is None:
        total = int((dst_off[-1] + dst_cap[-1]).item()) if n else 1
        dst = torch.empty(max(total, 1), dtype=torch.uint8, device=dev)
    out_len = torch.empty(n, dtype=torch.int32, device=dev)
    N.launch_compress(src, src_off, src_len, dst, dst_off, dst_cap, out_len, n, int(tab), int(acceleration), stream)
    return dst, dst_off, out_len


def decompress_batch(src: torch.Tensor, src_off: torch.Tensor, src_len: torch.Tensor, dst_cap: torch.Tensor, *,
                     dst: torch.Tensor | None = None, dst_off: torch.Tensor | None = None,
                     dict_buf: torch.Tensor | None = None, dict_off: torch.Tensor | None = None,
                     dict_len: torch.Tensor | None = None, stream=None):
    """Decompress n device-resident blocks in one stream-ordered launch.

    Returns (dst, dst_off, status): status int32[n] is the decoded size or
    -(pos)-1 exactly as LZ4_decompress_safe(_usingDict) would return.
    """
    n = src_off.numel()
    dev = src.device
    if dst_off is None:
        dst_off = N.exclusive_scan(dst_cap, stream=stream)[:n]
    if dst is None:
        total = int((dst_off[-1] + dst_cap[-1]).item()) if n else 1
        dst = torch.empty(max(total, 1), dtype=torch.uint8, device=dev)
    status = torch.empty(n, dtype=torch.int32, device=dev)
    N.launch_decompress(src, src_off, src_len, dst, dst_off, dst_cap, status, n, stream,
                        dict_buf, dict_off, dict_len)
    return dst, dst_off, status


def compact(buf: torch.Tensor, off: torch.Tensor, length: torch.Tensor, stream=None):
    """Pack variable-length items (e.g. compress_batch output) contiguously:
    returns (packed uint8, offsets int64[n+1])."""
    n = off.numel()
    offs = N.exclusive_scan(length, stream=stream)
    total = int(offs[-1].item())
    out = torch.empty(max(total, 1), dtype=torch.uint8, device=buf.device)
    N.gather(buf, off, length, out, offs, n, stream)
    return out[:total], offs


def xxh32_batch(src: torch.Tensor, off: torch.Tensor, length: torch.Tensor, seed: int = 0, stream=None):
    """XXH32 of n device-resident items (uint32[n] as int64 tensor view)."""
    n = off.numel()
    out = torch.empty(n, dtype=torch.int32, device=src.device)
    N.launch_xxh32_batch(src, off, length.to(torch.int64), seed, out, n, stream)
    return out


def decompress_host(comp: torch.Tensor, comp_off: torch.Tensor, comp_len: torch.Tensor, out: torch.Tensor,
                    out_off: torch.Tensor, out_cap: torch.Tensor, *, chunk_blocks: int = 16384,
                    device=None) -> torch.Tensor:
    """Decode n blocks that start and end in HOST memory (a file's or
    socket's bytes), pipelined over PCIe: chunk i+1 is copied in while
    chunk i decodes and chunk i-1 is copied out (three HIP streams, two
    device buffer sets).  comp / out are uint8 host tensors (pin them for
    the copies to overlap); comp_off / out_off int64, comp_len / out_cap
    int32 host tensors, blocks in increasing position order in both.
    Returns the int32 status of every block (host), as LZ4_decompress_safe
    would return it.  Chunks of 32 768 blocks or more run the large-batch
    row decoder, smaller ones the one-wave-per-block decoder
    (lz4m_decompress_batch_sel's switch-over).  The
    call is bound by the download; smaller chunks start it sooner: 262 144
    silesia-like blocks ran at 42.8 / 45.2 / 46.2 GiB/s with chunks of
    65 536 / 32 768 / 16 384 blocks (the default; profiles/r05/r05at)."""
    dev = device or N.device()
    n = comp_off.numel()
    status = torch.empty(n, dtype=torch.int32, device=dev)
    if n == 0:
        return status.cpu()
    c_off, c_len = comp_off.to(torch.int64), comp_len.to(torch.int32)
    o_off, o_cap = out_off.to(torch.int64), out_cap.to(torch.int32)
    if bool((c_off[1:] < c_off[:-1] + c_len[:-1]).any()) or bool((o_off[1:] < o_off[:-1] + o_cap[:-1]).any()):
        raise ValueError("blocks must be in increasing, non-overlapping position order")
    chunks = [(lo, min(n, lo + chunk_blocks)) for lo in range(0, n, chunk_blocks)]

    def span(off, ln, lo, hi):
        return int(off[lo]), int(off[hi - 1]) + int(ln[hi - 1])

    in_max = max(b - a for a, b in (span(c_off, c_len, lo, hi) for lo, hi in chunks))
    out_max = max(b - a for a, b in (span(o_off, o_cap, lo, hi) for lo, hi in chunks))
    d_in = [torch.empty(in_max + 16, dtype=torch.uint8, device=dev) for _ in range(2)]
    d_out = [torch.empty(max(out_max, 1), dtype=torch.uint8, device=dev) for _ in range(2)]
    s_in, s_dec, s_out = torch.cuda.Stream(dev), torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    ev_in = [torch.cuda.Event() for _ in range(2)]
    ev_dec = [torch.cuda.Event() for _ in range(2)]
    ev_free = [None, None]
    # every chunk's block offsets, rebased to its buffers, in one upload (a
    # per-chunk upload from pageable memory would block the host thread)
    base_c = torch.zeros(n, dtype=torch.int64)
    base_o = torch.zeros(n, dtype=torch.int64)
    for lo, hi in chunks:
        base_c[lo:hi] = int(c_off[lo])
        base_o[lo:hi] = int(o_off[lo])
    meta = torch.stack([c_off - base_c, o_off - base_o]).to(dev)
    lens = torch.stack([c_len, o_cap]).to(dev)
    cur = torch.cuda.current_stream(dev)
    s_in.wait_stream(cur)
    s_out.wait_stream(cur)
    s_dec.wait_stream(cur)
    try:
        if os.environ.get("LZ4M_HOST_QUEUED") == "1":   # A/B: every copy queued up front behind its event
            for i, (lo, hi) in enumerate(chunks):
                b = i & 1
                a0, a1 = span(c_off, c_len, lo, hi)
                b0, b1 = span(o_off, o_cap, lo, hi)
                with torch.cuda.stream(s_in):
                    if ev_free[b] is not None:
                        s_in.wait_event(ev_free[b])                    # chunk i-2 has left buffer b
                    d_in[b][: a1 - a0].copy_(comp[a0:a1], non_blocking=True)
                    ev_in[b].record(s_in)
                with torch.cuda.stream(s_dec):
                    s_dec.wait_event(ev_in[b])
                    N.launch_decompress(d_in[b], meta[0, lo:hi], lens[0, lo:hi], d_out[b], meta[1, lo:hi],
                                        lens[1, lo:hi], status[lo:hi], hi - lo, s_dec)
                    ev_dec[b].record(s_dec)
                with torch.cuda.stream(s_out):
                    s_out.wait_event(ev_dec[b])
                    out[b0:b1].copy_(d_out[b][: b1 - b0], non_blocking=True)
                    ev_free[b] = torch.cuda.Event()
                    ev_free[b].record(s_out)
        else:
            # Copies are queued only once what they wait for is done (the host
            # waits on the event): a copy queued behind an event holds up the
            # copies in the other direction on the copy engine (the upload of
            # chunk i+1 waited for the decode of chunk i, r05ac/r05ad).
            def issue_out(b, b0, b1):
                ev_dec[b].synchronize()                                # its decode is done
                with torch.cuda.stream(s_out):
                    out[b0:b1].copy_(d_out[b][: b1 - b0], non_blocking=True)
                    ev_free[b] = torch.cuda.Event()
                    ev_free[b].record(s_out)

            pending = None
            for i, (lo, hi) in enumerate(chunks):
                b = i & 1
                a0, a1 = span(c_off, c_len, lo, hi)
                if ev_free[b] is not None:
                    ev_free[b].synchronize()                           # chunk i-2 has left buffer b
                with torch.cuda.stream(s_in):
                    d_in[b][: a1 - a0].copy_(comp[a0:a1], non_blocking=True)
                    ev_in[b].record(s_in)
                with torch.cuda.stream(s_dec):
                    s_dec.wait_event(ev_in[b])
                    N.launch_decompress(d_in[b], meta[0, lo:hi], lens[0, lo:hi], d_out[b], meta[1, lo:hi],
                                        lens[1, lo:hi], status[lo:hi], hi - lo, s_dec)
                    ev_dec[b].record(s_dec)
                if pending is not None:
                    issue_out(*pending)
                pending = (b,) + span(o_off, o_cap, lo, hi)
            issue_out(*pending)
    finally:
        # (on an error too: no copy or launch may still use the buffers freed on return)
        for s_ in (s_in, s_dec, s_out):
            s_.synchronize()
    cur.wait_stream(s_out)
    cur.wait_stream(s_dec)
    st = status.cpu()
    torch.cuda.synchronize(dev)
    return st
