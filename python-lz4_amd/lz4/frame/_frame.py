"""``lz4.frame`` one-shot API on the MI355X codec.

Mirrors the reference extension ``lz4/frame/_frame.c`` (compress 112-259,
get_frame_info 640-824, __decompress 938-1193) over the frame format of
``lz4libs/lz4frame.c``.  The host walks the frame structure (header bytes,
LE32 block records); every byte-level operation runs on the GPU:

* compress: the input is cut into blocks and compressed in one batched
  launch (cap = block size - 1, raw block when it does not fit,
  lz4frame.c:834-842) -- independent blocks with the
  LZ4_compress_fast_extState_fastReset parse (lz4frame.c:853-863 ->
  lz4.c:1378-1413), linked blocks (the default) as one
  LZ4_compress_fast_continue stream (lz4frame.c:865-871), speculatively in
  parallel (lz4m_compress_linked_batch); block records are emitted by
  ``lz4m_frame_emit`` at scanned offsets.  The content checksum (XXH32 over
  all input, lz4frame.c:1042, 1171) is one serial stream: it runs on a host
  core (lz4m_xxh32_host_*) in a thread beside the device work -- on the
  caller's bytes, or on device bytes streamed back over PCIe in chunks; the
  1-byte header checksum (lz4frame.c:341-345) too.
* decompress: independent blocks decode in one batched launch into slots of
  the frame's maximum block size (the capacity LZ4F_decompress gives,
  lz4frame.c:1844-1847), raw blocks are gathered, block checksums are
  verified on the device, the content checksum on a host core.  Linked-block frames decode
  block after block on one wavefront with the previous output as prefix.

Scope notes: every frame ``compress`` writes is byte-identical
to the reference's (``parse="parallel"`` on ``compress_device`` trades that
for speed); HC levels (>= 3) and the chunked / context streaming API are
outside this codec's scope.
"""
from __future__ import annotations

import os
import struct
import threading
import time

import torch

from .. import _native as N
from ..block._block import _buffer, _c_int

BLOCKSIZE_DEFAULT = 0
BLOCKSIZE_MAX64KB = 4
BLOCKSIZE_MAX256KB = 5
BLOCKSIZE_MAX1MB = 6
BLOCKSIZE_MAX4MB = 7

_MAGIC = 0x184D2204
_MAGIC_SKIPPABLE = 0x184D2A50
_BLOCK_SIZES = {4: 64 << 10, 5: 256 << 10, 6: 1 << 20, 7: 4 << 20}
_MIN_FH = 7        # lz4frame.c minFHSize
_BH = 4            # block header size
_UNCOMPRESSED = 0x80000000


def _err(fn: str, code: str) -> RuntimeError:
    return RuntimeError(f"{fn} failed with code: ERROR_{code}")


def _content_on_gpu() -> bool:
    """LZ4M_CONTENT_XXH32=gpu runs the content checksum on one wavefront
    (lz4m_xxh32_long, 1.7 GB/s) instead of a host core (A/B runs)."""
    return os.environ.get("LZ4M_CONTENT_XXH32", "host") == "gpu"


def _xxh32_dev(buf: bytes | memoryview | torch.Tensor, n: int | None = None, seed: int = 0) -> int:
    """XXH32 of a buffer: host bytes on this core; device bytes on a host
    core over pipelined PCIe copies (or on the GPU, _content_on_gpu)."""
    if not isinstance(buf, torch.Tensor):
        return N.xxh32_host(buf, seed)
    length = n if n is not None else buf.numel()
    if not _content_on_gpu():
        return N.xxh32_of_device(buf, length, seed)
    out = torch.empty(1, dtype=torch.int32, device=buf.device)
    N.launch_xxh32_long(buf, length, seed, out)
    return int(out.item()) & 0xFFFFFFFF


class _HashThread(threading.Thread):
    """The content checksum on a host core beside the device work."""

    def __init__(self, fn):
        super().__init__(daemon=True)
        self._fn = fn
        self.value = None
        self.error = None

    def run(self):
        try:
            self.value = self._fn()
        except BaseException as e:   # re-raised in the caller
            self.error = e

    def result(self) -> int:
        self.join()
        if self.error is not None:
            raise self.error
        return self.value


# ------------------------------------------------------------------ header
# linked frames with at least this many blocks compress speculatively in
# parallel (lz4m_compress_linked_batch); shorter ones one wavefront per frame
_SPEC_MIN_BLOCKS = int(os.environ.get("LZ4M_SPEC_MIN_BLOCKS", "4"))


def _optimal_bsid(requested: int, size: int) -> int:
    """LZ4F_optimalBSID (lz4frame.c:351-363)."""
    proposed, max_size = 4, 64 << 10
    while requested > proposed:
        if size <= max_size:
            return proposed
        proposed += 1
        max_size <<= 2
    return requested


def _header(bsid: int, linked: bool, block_checksum: bool, content_size: int, content_checksum: bool) -> bytes:
    """LZ4F_compressBegin_usingCDict header (lz4frame.c:752-780)."""
    flg = (1 << 6) | ((0 if linked else 1) << 5) | (int(block_checksum) << 4) \
        | (int(content_size > 0) << 3) | (int(content_checksum) << 2)
    body = bytes([flg, (bsid & 7) << 4])
    if content_size:
        body += struct.pack("<Q", content_size)
    hc = (_xxh32_dev(body) >> 8) & 0xFF
    return struct.pack("<I", _MAGIC) + body + bytes([hc])


def _parse_header(mv: memoryview):
    """LZ4F_getFrameInfo -> LZ4F_headerSize + LZ4F_decodeHeader
    (lz4frame.c:1291-1380, 1387-1463).  Returns (info dict, header size)."""
    fn = "LZ4F_getFrameInfo"
    n = mv.nbytes
    if n < 5:
        raise _err(fn, "frameHeader_incomplete")
    magic = struct.unpack_from("<I", mv, 0)[0]
    if (magic & 0xFFFFFFF0) == _MAGIC_SKIPPABLE:
        if n < 8:
            raise _err(fn, "frameHeader_incomplete")
        return {"skippable": True, "frame_size": struct.unpack_from("<I", mv, 4)[0]}, 8
    if magic != _MAGIC:
        raise _err(fn, "frameType_unknown")
    flg = mv[4]
    hsize = _MIN_FH + (8 if flg & 0x08 else 0) + (4 if flg & 0x01 else 0)
    if n < hsize:
        raise _err(fn, "frameHeader_incomplete")
    if (flg >> 1) & 1:
        raise _err(fn, "reservedFlag_set")
    if (flg >> 6) & 3 != 1:
        raise _err(fn, "headerVersion_wrong")
    bd = mv[5]
    bsid = (bd >> 4) & 7
    if (bd >> 7) & 1:
        raise _err(fn, "reservedFlag_set")
    if bsid < 4:
        raise _err(fn, "maxBlockSize_invalid")
    if bd & 0x0F:
        raise _err(fn, "reservedFlag_set")
    hc = (_xxh32_dev(bytes(mv[4:hsize - 1])) >> 8) & 0xFF
    if hc != mv[hsize - 1]:
        raise _err(fn, "headerChecksum_invalid")
    info = {
        "skippable": False,
        "block_size_id": bsid,
        "block_size": _BLOCK_SIZES[bsid],
        "block_linked": not bool((flg >> 5) & 1),
        "block_checksum": bool((flg >> 4) & 1),
        "content_checksum": bool((flg >> 2) & 1),
        "content_size": struct.unpack_from("<Q", mv, 6)[0] if flg & 0x08 else 0,
        "dict_id": struct.unpack_from("<I", mv, hsize - 5)[0] if flg & 0x01 else 0,
    }
    return info, hsize


def get_frame_info(data):
    """get_frame_info(data) -- frame parameters of the frame at the start of
    data (_frame.c:640-824)."""
    mv = _buffer(data)
    info, _ = _parse_header(mv)
    if info["skippable"]:
        return {"block_size": 64 << 10, "block_size_id": BLOCKSIZE_MAX64KB, "block_linked": True,
                "content_checksum": False, "block_checksum": False, "skippable": True, "content_size": 0}
    return {k: info[k] for k in ("block_size", "block_size_id", "block_linked", "content_checksum",
                                  "block_checksum", "skippable", "content_size")}


# ---------------------------------------------------------------- compress
def compress(data, compression_level=0, block_size=0, content_checksum=False, block_checksum=False,
             block_linked=True, store_size=True, return_bytearray=False):
    """compress(data, compression_level=0, block_size=0, content_checksum=0,
    block_checksum=0, block_linked=True, store_size=True,
    return_bytearray=False) -- one LZ4 frame (_frame.c:112-259 ->
    LZ4F_compressFrame, lz4frame.c:420-515)."""
    src = _buffer(data, "data")
    level = _c_int(compression_level, "compression_level")
    bsid_req = _c_int(block_size, "block_size")
    dev = N.device()
    d_src = N.to_device(src, dev, pad=1)
    frame = _compress_frame(d_src, src.nbytes, compression_level=level, block_size=bsid_req,
                            content_checksum=content_checksum, block_checksum=block_checksum,
                            block_linked=block_linked, store_size=store_size, host_src=src)[0]
    return N.to_host_bytes(frame, frame.numel(), bool(return_bytearray))


def compress_device(d_src: torch.Tensor, n: int | None = None, *, compression_level=0, block_size=0,
                    content_checksum=False, block_checksum=False, block_linked=True, store_size=True,
                    parse="exact", stream=None) -> torch.Tensor:
    """Device-resident LZ4F_compressFrame: the frame of d_src[:n] as a uint8
    device tensor (no host round trip).

    parse="exact": blocks byte-identical to LZ4_compress_default, i.e. the
    frame is byte-identical to the reference's for independent blocks.
    parse="parallel": the parallel-parse compressor (valid blocks at the
    ratio of LZ4_compress_default, not byte-identical; BASELINE config 4).

    The content checksum (one serial XXH32 stream over all of d_src) runs on
    a host core beside the block compression, over pipelined PCIe copies of
    d_src."""
    return _compress_frame(d_src, n, compression_level=compression_level, block_size=block_size,
                           content_checksum=content_checksum, block_checksum=block_checksum,
                           block_linked=block_linked, store_size=store_size, parse=parse, stream=stream)[0]


def _host_wait(stream) -> None:
    """Block until `stream` drains, with the GIL released (an event wait;
    tensor.item() waits holding the GIL, so a host hashing thread would sit
    idle for the whole device phase)."""
    ev = torch.cuda.Event()
    ev.record(stream)
    ev.synchronize()


def _compress_frame(d_src, n=None, *, compression_level=0, block_size=0, content_checksum=False,
                    block_checksum=False, block_linked=True, store_size=True, parse="exact", stream=None,
                    host_src=None):
    """compress_device, also returning the block records:
    (frame, {"data_off", "stored_len", "raw"}) with device tensors giving, per
    block, the payload position in the frame, its stored length and whether
    it is stored raw (None when the input is empty)."""
    n = d_src.numel() if n is None else int(n)
    level = int(compression_level)
    if level >= 3:
        raise NotImplementedError("LZ4 HC compression levels (>= 3) are outside the MI355X codec's scope")
    if parse not in ("exact", "parallel"):
        raise ValueError("parse must be 'exact' or 'parallel'")
    accel = -level + 1 if level < 0 else 1                     # lz4frame.c:855
    bsid = _optimal_bsid(int(block_size), n)
    if bsid == 0:
        bsid = BLOCKSIZE_MAX64KB                               # LZ4F_BLOCKSIZEID_DEFAULT
    if bsid not in _BLOCK_SIZES:
        raise RuntimeError("LZ4F_compressFrame failed with code: ERROR_maxBlockSize_invalid")
    bsize = _BLOCK_SIZES[bsid]
    linked = bool(block_linked) and n > bsize                  # lz4frame.c:441-442
    content_size = n if store_size else 0
    hdr = _header(bsid, linked, bool(block_checksum), content_size, bool(content_checksum))
    dev = d_src.device
    nb = (n + bsize - 1) // bsize
    total = 0
    body = None
    meta = None
    main = stream if stream is not None else torch.cuda.current_stream(dev)
    h = hthread = None
    if content_checksum:                                       # lz4frame.c:1042, 1170-1176
        if _content_on_gpu():
            side = torch.cuda.Stream(dev)
            side.wait_stream(main)
            h = torch.empty(1, dtype=torch.int32, device=dev)
            N.launch_xxh32_long(d_src, n, 0, h, side)
            h.record_stream(main)
        elif host_src is not None:   # the caller's bytes: hash them while the device compresses
            hthread = _HashThread(lambda: N.xxh32_host(host_src))
            hthread.start()
        else:                        # device bytes: streamed back and hashed while the device compresses
            ready = torch.cuda.Event()
            ready.record(main)       # before the compression is queued: the copies must not wait for it
            hthread = _HashThread(lambda: N.xxh32_of_device(d_src, n, wait_event=ready))
            hthread.start()
    if nb:
        raw_off = torch.arange(nb, dtype=torch.int64, device=dev) * bsize
        raw_len = torch.full((nb,), bsize, dtype=torch.int32, device=dev)
        raw_len[-1] = n - (nb - 1) * bsize
        cap = raw_len - 1                                      # lz4frame.c:835: dstCapacity = srcSize - 1
        slot = N.compress_bound(bsize)
        cmp = torch.empty(nb * slot, dtype=torch.uint8, device=dev)
        cmp_off = torch.arange(nb, dtype=torch.int64, device=dev) * slot
        cmp_len = torch.empty(nb, dtype=torch.int32, device=dev)
        if parse == "exact" and linked:   # one stream across the blocks (lz4frame.c:865-871)
            link = torch.ones(nb, dtype=torch.int32, device=dev)
            link[0] = 0
            mode = N.LINKED_SPECULATIVE if nb >= _SPEC_MIN_BLOCKS else N.LINKED_SERIAL
            N.launch_compress_linked(d_src, raw_off, raw_len, link, cmp, cmp_off, cap, cmp_len, nb, accel,
                                     mode=mode, stream=stream)
        else:
            if parse == "exact":
                table = N.TABLE_AUTO
            else:
                table = N.PARSE_PARALLEL if bsize <= 65536 else N.PARSE_PARALLEL_LARGE
            N.launch_compress(d_src, raw_off, raw_len, cmp, cmp_off, cap, cmp_len, nb, table, accel, stream,
                              max_len=bsize)
        rec_len = torch.empty(nb, dtype=torch.int32, device=dev)
        N.frame_block_sizes(raw_len, cmp_len, block_checksum, rec_len, nb, stream)
        frame_off = N.exclusive_scan(rec_len, stream=stream)
        if hthread is not None:   # wait with the GIL released: .item() waits holding it, stalling the hash thread
            _host_wait(main)
        total = int(frame_off[-1].item())
    tail = 4 + (4 if content_checksum else 0)
    out = torch.empty(len(hdr) + total + tail + 16, dtype=torch.uint8, device=dev)
    out[: len(hdr)] = torch.frombuffer(bytearray(hdr), dtype=torch.uint8).to(dev)
    if nb:
        body = out[len(hdr):]
        N.frame_emit(d_src, raw_off, raw_len, cmp, cmp_off, cmp_len, body, frame_off, block_checksum, nb, stream)
        del cmp
        stored = rec_len - 4 - (4 if block_checksum else 0)
        meta = {"data_off": frame_off[:nb] + len(hdr) + 4, "stored_len": stored,
                "raw": (cmp_len <= 0) | (cmp_len >= raw_len)}
    pos = len(hdr) + total
    out[pos: pos + 4] = 0                                      # endmark, lz4frame.c:1167
    if content_checksum:
        if hthread is not None:
            dig = hthread.result()
            out[pos + 4: pos + 8] = torch.frombuffer(bytearray(struct.pack("<I", dig)), dtype=torch.uint8).to(dev)
        else:
            main.wait_stream(side)
            out[pos + 4: pos + 8] = h.view(torch.uint8)
    return out[: pos + tail], meta


# -------------------------------------------------------------- decompress
def _scan_blocks(mv: memoryview, pos: int, info: dict):
    """Walk the block records the way LZ4F_decompress consumes them
    (lz4frame.c:1643-1701, 1926-1965).  Returns (records, end_state) where
    records = [(raw, data_pos, size, crc_pos)] and end_state is either
    ("end", bytes_read) or ("incomplete", hint) or ("error", code, index)."""
    n = mv.nbytes
    crc = 4 if info["block_checksum"] else 0
    maxb = info["block_size"]
    recs = []
    while True:
        if n - pos < _BH:
            return recs, ("incomplete", _BH - (n - pos))
        hdr = struct.unpack_from("<I", mv, pos)[0]
        pos += _BH
        if hdr == 0:                                           # endmark
            if info["content_checksum"]:
                if n - pos < 4:
                    return recs, ("incomplete_suffix", 4 - (n - pos), pos)
                return recs, ("end", pos + 4, pos)
            return recs, ("end", pos, None)
        size = hdr & 0x7FFFFFFF
        if size > maxb:
            return recs, ("error", "maxBlockSize_invalid", len(recs))
        raw = bool(hdr & _UNCOMPRESSED)
        avail = n - pos
        if raw:
            if avail < size + crc:
                got = min(avail, size)
                if avail <= size:
                    hint = (size - got) + crc + _BH
                else:
                    hint = crc - (avail - size) + _BH
                return recs, ("incomplete", hint if avail else _BH + size + crc)
        elif avail < size + crc:
            hint = (size + crc - avail) + crc + _BH if avail else _BH + size + crc
            return recs, ("incomplete", hint)
        recs.append((raw, pos, size, pos + size if crc else -1))
        pos += size + crc


def decompress(data, return_bytearray=False, return_bytes_read=False):
    """decompress(data, return_bytearray=False, return_bytes_read=False) --
    decode one full frame (_frame.c:1198-1258 -> __decompress 938-1193)."""
    mv = _buffer(data, "data")
    info, hsize = _parse_header(mv)
    if info["skippable"]:
        end = min(mv.nbytes, hsize + info["frame_size"])
        if mv.nbytes < hsize + info["frame_size"]:
            raise RuntimeError(f"Frame incomplete. LZ4F_decompress returned: {hsize + info['frame_size'] - mv.nbytes}")
        out = bytearray() if return_bytearray else b""
        return (out, end) if return_bytes_read else out
    recs, state = _scan_blocks(mv, hsize, info)
    if os.environ.get("LZ4M_FRAME_PIPELINE", "1") != "0":
        r = _decompress_pipelined(mv, info, recs, state, bool(return_bytearray))
        if r is not None:
            return (r, state[1]) if return_bytes_read else r
    dev = N.device()
    nb = len(recs)
    out_t, total, first_err = None, 0, None
    if nb:
        d_frame = N.to_device(mv, dev, pad=16)
        t = lambda v, dt: torch.tensor(v, dtype=dt, device=dev)   # noqa: E731
        args = (d_frame, info, nb, t([r[1] for r in recs], torch.int64), t([r[2] for r in recs], torch.int32),
                t([r[0] for r in recs], torch.bool), t([r[3] for r in recs], torch.int64))
        out_t, total, first_err = _decode_records(*args)
    _frame_errors(first_err, state, info, total)
    bytes_read = state[1]
    host_hash = info["content_checksum"] and not (total and _content_on_gpu())
    got = None
    if host_hash:   # on the copy the caller gets, hashed while it is staged (lz4frame.c:1850, :1959-1964)
        out, got = N.to_host_bytes(out_t, total, bool(return_bytearray), hash_seed=0)
    else:
        out = N.to_host_bytes(out_t, total, bool(return_bytearray))
    if info["content_checksum"]:
        want = struct.unpack_from("<I", mv, state[2])[0]
        if got is None:
            got = _xxh32_dev(out_t, total)
        if got != want:
            raise _err("LZ4F_decompress", "contentChecksum_invalid")
    if return_bytes_read:
        return out, bytes_read
    return out


class _FeedHash(threading.Thread):
    """The content XXH32 on a host core, over host ranges handed to it in
    order (put(ptr, n); put(None) ends it)."""

    def __init__(self):
        super().__init__(daemon=True)
        import queue
        self.q = queue.SimpleQueue()
        self.st = N.HostXXH32(0)
        self.error = None

    def put(self, ptr, n=0):
        self.q.put(None if ptr is None else (ptr, n))

    def run(self):
        try:
            while True:
                item = self.q.get()
                if item is None:
                    return
                self.st.update_ptr(*item)
        except BaseException as e:   # re-raised in the caller
            self.error = e

    def digest(self) -> int:
        self.put(None)
        self.join()
        if self.error is not None:
            raise self.error
        return self.st.digest()


def _decompress_pipelined(mv, info, recs, state, as_bytearray):
    """``decompress`` of a large well-formed frame of independent compressed
    blocks with a stored content size, as one pipeline: the frame goes to the
    device in 64 MiB chunks, the blocks decode in three block-ordered launches
    as their bytes land, the output comes back in 64 MiB chunks as
    their launch ends -- straight into the result bytes -- and a host core
    hashes the result behind the copies (the content checksum, lz4frame.c:1850,
    one serial stream: the bound).  The stages that ran one after another
    (upload, decode, download + hash) overlap.

    Every block but the last is taken to decode to the full block size (what
    LZ4F_compressFrame writes), so the slots are the output; this, the
    statuses and the block checksums are checked at the end, and on any
    mismatch this returns None and the caller decodes the frame the
    sequential way (which raises the reference's exact error).  Also None
    when the frame does not qualify.

    A launch takes about one block's decode time whatever its size (one
    wavefront per block; a 4 MiB block ~51 ms, profiles/r05/r05y), so the
    launches are few and growing -- 1/16, 3/16, 12/16 of the blocks -- and
    the first two run on two streams side by side: the first output is ready
    one block-decode after 1/16 of the frame has landed, and the rest stays
    ahead of the hash."""
    nb = len(recs)
    maxb = info["block_size"]
    total = info["content_size"]
    n = mv.nbytes
    if (state[0] != "end" or info["block_linked"] or nb < 32 or n < N._BIG
            or not total or not ((nb - 1) * maxb < total <= nb * maxb) or _content_on_gpu()
            or any(r[0] for r in recs)):
        return None
    dev = N.device()
    main = torch.cuda.current_stream(dev)
    up = torch.cuda.Stream(dev, priority=-1)
    down = torch.cuda.Stream(dev, priority=-1)
    side = torch.cuda.Stream(dev)          # the second decode stream
    crc = info["block_checksum"]
    c_off = torch.tensor([r[1] for r in recs], dtype=torch.int64, device=dev)
    c_len = torch.tensor([r[2] for r in recs], dtype=torch.int32, device=dev)
    status = torch.empty(nb, dtype=torch.int32, device=dev)
    sums = torch.empty(nb, dtype=torch.int32, device=dev) if crc else None
    slots = torch.empty(nb * maxb + 16, dtype=torch.uint8, device=dev)
    slot_off = torch.arange(nb, dtype=torch.int64, device=dev) * maxb
    caps = torch.full((nb,), maxb, dtype=torch.int32, device=dev)
    d_frame = torch.empty(n + 16, dtype=torch.uint8, device=dev)
    d_frame[n:].zero_()
    up.wait_stream(main)   # (after the allocations: their memory may be free only in main's order)
    side.wait_stream(main)
    C = N._CHUNK
    thr = N._copy_threads()
    src, _, keep = N._addr(mv)
    out, dst = N._new_host_buffer(total, as_bytearray)
    hasher = _FeedHash() if info["content_checksum"] else None
    if hasher is not None:
        hasher.start()
    # spans: block-ordered decode launches; span k needs the frame up to ends[k]
    bounds = [0, nb // 16, nb // 4, nb]
    K = len(bounds) - 1
    ends = [recs[bounds[k + 1] - 1][1] + recs[bounds[k + 1] - 1][2] + (4 if crc else 0) for k in range(K)]
    span_ev = [None] * K
    trace = [] if os.environ.get("LZ4M_PIPE_TRACE") else None
    t0 = time.perf_counter()
    fills = [(lo, min(n, lo + C)) for lo in range(0, n, C)]
    drains = [(lo, min(total, lo + C)) for lo in range(0, total, C)]
    # the span whose launch writes the last byte of each drain chunk
    need = [next(k for k in range(K) if (b - 1) // maxb < bounds[k + 1]) for _, b in drains]
    upb, downb = N._pinned_pair(C), N._pinned_pair(C)
    up_ev, down_ev = [None, None], [torch.cuda.Event(), torch.cuda.Event()]
    launched = 0
    fi = di = dd = 0   # next fill, next drain to issue, next drain to finish
    done = False
    try:
        while dd < len(drains):
            # a download is queued only once its launch is done: a copy queued
            # behind an event holds up the uploads (r05ac: the second launch
            # waited for the first launch's end)
            while di < len(drains) and di - dd < 2 and need[di] < launched and span_ev[need[di]].query():
                lo, hi = drains[di]
                with torch.cuda.stream(down):
                    downb[di & 1][: hi - lo].copy_(slots[lo:hi], non_blocking=True)
                    down_ev[di & 1].record(down)
                di += 1
            if dd < di and (fi == len(fills) or down_ev[dd & 1].query()):
                lo, hi = drains[dd]
                down_ev[dd & 1].synchronize()
                N.lib().lz4m_host_copy(dst + lo, downb[dd & 1].data_ptr(), hi - lo, thr, None)
                if hasher is not None:
                    hasher.put(dst + lo, hi - lo)
                if trace is not None:
                    trace.append(("drain", dd, time.perf_counter() - t0))
                dd += 1
                continue
            if fi < len(fills):   # upload the next frame chunk, launch the spans it completes
                lo, hi = fills[fi]
                b = upb[fi & 1]
                if up_ev[fi & 1] is not None:
                    up_ev[fi & 1].synchronize()
                N.lib().lz4m_host_copy(b.data_ptr(), src + lo, hi - lo, thr, None)
                with torch.cuda.stream(up):
                    d_frame[lo:hi].copy_(b[: hi - lo], non_blocking=True)
                    up_ev[fi & 1] = torch.cuda.Event()
                    up_ev[fi & 1].record(up)
                fi += 1
                while launched < K and ends[launched] <= hi:
                    k = launched
                    st = side if k == 1 else main
                    st.wait_event(up_ev[(fi - 1) & 1])
                    a, z = bounds[k], bounds[k + 1]
                    with torch.cuda.stream(st):
                        if crc:
                            N.launch_xxh32_batch(d_frame, c_off[a:z], c_len[a:z].to(torch.int64), 0, sums[a:z], z - a,
                                                 stream=st)
                        N.launch_decompress(d_frame, c_off[a:z], c_len[a:z], slots, slot_off[a:z], caps[a:z],
                                            status[a:z], z - a, stream=st)
                        span_ev[k] = torch.cuda.Event(enable_timing=trace is not None)
                        span_ev[k].record(st)
                    if trace is not None:
                        trace.append(("launch", k, time.perf_counter() - t0))
                    launched += 1
                continue
            if dd == di:   # everything uploaded and launched: wait for the next download's launch
                span_ev[need[di]].synchronize()
        done = True
    finally:
        if hasher is not None and not done:
            # the thread may still be hashing `out`, freed once the exception
            # leaves this function: it must have ended first
            hasher.put(None)
            hasher.join()
        # (on an error too: no copy or launch may still use the buffers freed on return)
        for e in up_ev + down_ev + span_ev:
            if e is not None:
                e.synchronize()
        N._pinned_release(C, upb)
        N._pinned_release(C, downb)
        del keep
    got = hasher.digest() if hasher is not None else None
    main.wait_stream(side)
    if trace is not None:
        import sys
        trace.append(("hash", 0, time.perf_counter() - t0))
        print("[lz4m] pipelined frame decode: " + " ".join(f"{a}{b}@{c * 1e3:.1f}" for a, b, c in trace
                                                          if a != "drain" or b % 16 == 0 or b == len(drains) - 1),
              file=sys.stderr, flush=True)
    ok = (status[: nb - 1] == maxb).all() & (status[nb - 1] == total - (nb - 1) * maxb)
    if crc:
        crc_pos = torch.tensor([r[3] for r in recs], dtype=torch.int64, device=dev)
        ok = ok & ((sums.to(torch.int64) & 0xFFFFFFFF) == _le32_at(d_frame, crc_pos)).all()
    if not bool(ok):
        return None
    if info["content_checksum"] and got != struct.unpack_from("<I", mv, state[2])[0]:
        raise _err("LZ4F_decompress", "contentChecksum_invalid")
    return out


def decompress_device(d_frame: torch.Tensor, n: int | None = None, stream=None) -> torch.Tensor:
    """Device-resident LZ4F_decompress: decode the frame in d_frame[:n] (a
    uint8 device tensor) into a new uint8 device tensor, with no host copy of
    the data (BASELINE config 4).  The header is parsed on
    the host from its first bytes; the block records are walked on the device
    (lz4m_frame_scan); independent blocks decode in one batched launch, linked
    ones on the chain kernel; block checksums are verified on the device, the
    content checksum on a host core over pipelined PCIe copies of the output.
    A malformed or truncated frame raises exactly what ``decompress`` raises
    for the same bytes."""
    n = d_frame.numel() if n is None else int(n)
    dev = d_frame.device
    head = bytes(d_frame[: min(n, 19)].cpu().numpy().tobytes())
    try:
        info, hsize = _parse_header(memoryview(head))
    except RuntimeError:
        if n <= 19:
            raise
        info, hsize = None, 0
    if info is None or info["skippable"] or n <= hsize:
        # errors and skippable frames: the host path's exact semantics
        out = decompress(d_frame[:n].cpu().numpy().tobytes())
        return torch.frombuffer(bytearray(out), dtype=torch.uint8).to(dev) if out else \
            torch.empty(0, dtype=torch.uint8, device=dev)
    crc = 4 if info["block_checksum"] else 0
    max_rec = n // 64 + 1024
    rec_pos = torch.empty(max_rec, dtype=torch.int64, device=dev)
    rec_len = torch.empty(max_rec, dtype=torch.int32, device=dev)
    rec_raw = torch.empty(max_rec, dtype=torch.uint8, device=dev)
    res = torch.zeros(4, dtype=torch.int64, device=dev)
    N.frame_scan(d_frame, n, hsize, info["block_checksum"], info["content_checksum"], info["block_size"], max_rec,
                 rec_pos, rec_len, rec_raw, res, stream)
    nb, st, _end, cpos = (int(v) for v in res.cpu().tolist())
    if st != 0:   # malformed / truncated (or > max_rec records): the host path's exact result or error
        out = decompress(d_frame[:n].cpu().numpy().tobytes())
        return torch.frombuffer(bytearray(out), dtype=torch.uint8).to(dev) if out else \
            torch.empty(0, dtype=torch.uint8, device=dev)
    out_t, total, first_err, got = None, 0, None, None
    if nb:
        crc_pos = rec_pos[:nb] + rec_len[:nb].to(torch.int64) if crc else torch.full((nb,), -1, dtype=torch.int64,
                                                                                      device=dev)
        follow = bool(info["content_checksum"]) and not _content_on_gpu() and \
            os.environ.get("LZ4M_FRAME_FOLLOW", "1") != "0"
        r = _decode_records(d_frame, info, nb, rec_pos[:nb], rec_len[:nb], rec_raw[:nb].to(torch.bool), crc_pos,
                            follow_hash=follow)
        out_t, total, first_err = r[:3]
        got = r[3] if follow else None
    _frame_errors(first_err, ("end", _end, cpos if cpos >= 0 else None), info, total)
    if info["content_checksum"]:
        want = int(_le32_at(d_frame, torch.tensor([cpos], dtype=torch.int64, device=dev)).item()) & 0xFFFFFFFF
        if got is None:
            got = _xxh32_dev(out_t, total) if total else _xxh32_dev(b"")
        if got != want:
            raise _err("LZ4F_decompress", "contentChecksum_invalid")
    if not total:
        return torch.empty(0, dtype=torch.uint8, device=dev)
    return out_t[:total]


def _le32_at(d_buf, pos):
    """LE32 values at device positions `pos` of d_buf (int64 tensor)."""
    idx = pos[:, None] + torch.arange(4, dtype=torch.int64, device=pos.device)
    b = d_buf[idx].to(torch.int64)
    return b[:, 0] | (b[:, 1] << 8) | (b[:, 2] << 16) | (b[:, 3] << 24)


def _frame_errors(first_err, state, info, total):
    """The error order of __decompress / LZ4F_decompress (lz4frame.c:1819,
    1844-1847, 1927): first failing block, then a structural error, then
    truncation, then the content size."""
    dec = "LZ4F_decompress"
    if first_err is not None:
        raise _err(dec, first_err[1])
    if state[0] == "error":
        raise _err(dec, state[1])
    if state[0] == "incomplete":
        raise RuntimeError(f"Frame incomplete. LZ4F_decompress returned: {state[1]}")
    if info["content_size"] and total != info["content_size"]:
        raise _err(dec, "frameSize_wrong")                     # lz4frame.c:1927
    if state[0] == "incomplete_suffix":
        raise RuntimeError(f"Frame incomplete. LZ4F_decompress returned: {state[1]}")


# block-ordered decode launches the content hash follows (decompress_device).
# A launch takes about one block's decode time whatever its size (4 MiB
# blocks: ~51 ms, profiles/r05/r05y): 16 launches (826 ms) fell behind the
# hash; 2, 4 and 8 launches measured 674-682 ms (r05y, r05ab)
_FOLLOW_CHUNKS = 4


def _decode_records(d_frame, info, nb, c_off, c_len, raw_mask, crc_pos, follow_hash=False):
    """Decode nb block records of a frame in device memory: payload at
    c_off[i] (int64), stored size c_len[i] (int32), raw_mask[i] = stored
    uncompressed, crc_pos[i] = position of its LE32 block checksum or -1.
    Returns (out tensor, total decoded bytes, first error or None), and with
    ``follow_hash`` a fourth item: the content XXH32 of the output, or None
    when the caller must hash it.

    ``follow_hash`` (independent blocks, no stored ones): the blocks decode
    in _FOLLOW_CHUNKS launches in block order, and a host thread hashes each
    launch's output as soon as it is done (lz4frame.c:1849-1850 hashes the
    output in order), reading it from the decode slots on the assumption
    that every block but the last decodes to the full block size (what
    LZ4F_compressFrame writes), so the slots are the output.  The assumption
    is checked once the decode is done; if it fails, the hash is discarded
    and the output gathered and hashed as before."""
    if follow_hash:
        r = _decode_records_follow(d_frame, info, nb, c_off, c_len, raw_mask, crc_pos)
        if r is not None:
            return r
        return _decode_records(d_frame, info, nb, c_off, c_len, raw_mask, crc_pos) + (None,)
    dev = d_frame.device
    maxb = info["block_size"]
    status = torch.empty(nb, dtype=torch.int32, device=dev)
    crc_bad = None
    if info["block_checksum"]:                                 # lz4frame.c:1819: verified first per block
        sums = torch.empty(nb, dtype=torch.int32, device=dev)
        N.launch_xxh32_batch(d_frame, c_off, c_len.to(torch.int64), 0, sums, nb)
        crc_bad = (sums.to(torch.int64) & 0xFFFFFFFF) != _le32_at(d_frame, crc_pos)
    slots = torch.empty(nb * maxb + 16, dtype=torch.uint8, device=dev)
    slot_off = torch.arange(nb, dtype=torch.int64, device=dev) * maxb
    linked = info["block_linked"] and nb > 1 and not bool(raw_mask.all())
    if linked:
        _decode_linked(d_frame, c_off, c_len, raw_mask, slots, status, maxb)
    else:
        # raw blocks are handed to the decoder with length 0 (immediate
        # reject, no work); they are gathered from the frame below
        caps = torch.full((nb,), maxb, dtype=torch.int32, device=dev)
        dec_len = torch.where(raw_mask, torch.zeros_like(c_len), c_len)
        N.launch_decompress(d_frame, c_off, dec_len, slots, slot_off, caps, status, nb)
    sizes = torch.where(raw_mask, c_len, status) if not linked else status
    bad_dec = (~raw_mask) & (status < 0)
    bad = bad_dec if crc_bad is None else (bad_dec | crc_bad)
    if bool(bad.any()):
        i = int(torch.nonzero(bad).flatten()[0])
        code = "blockChecksum_invalid" if crc_bad is not None and bool(crc_bad[i]) else "decompressionFailed"
        return None, 0, (i, code)
    if linked:
        return slots, int(sizes.to(torch.int64).sum()), None
    # no stored block and every block but the last full (what LZ4F_compressFrame
    # writes): the slots already are the output, no gather (one read-back)
    chk = torch.stack([(~raw_mask).all().to(torch.int64), (status[: nb - 1] == maxb).all().to(torch.int64),
                       status[nb - 1].to(torch.int64)]).cpu()
    if int(chk[0]) and int(chk[1]):
        return slots, (nb - 1) * maxb + int(chk[2]), None
    lens = sizes.to(torch.int32)
    offs = N.exclusive_scan(lens)
    total = int(offs[-1].item())
    out_t = torch.empty(total + 16, dtype=torch.uint8, device=dev)
    sel_c = torch.nonzero(~raw_mask).flatten()
    sel_r = torch.nonzero(raw_mask).flatten()
    if sel_c.numel():                                          # compressed blocks from the slots
        N.gather(slots, slot_off[sel_c], lens[sel_c], out_t, offs[sel_c], sel_c.numel())
    if sel_r.numel():                                          # raw blocks straight from the frame
        N.gather(d_frame, c_off[sel_r], lens[sel_r], out_t, offs[sel_r], sel_r.numel())
    return out_t, total, None


def _decode_records_follow(d_frame, info, nb, c_off, c_len, raw_mask, crc_pos):
    """_decode_records(follow_hash=True) for frames it applies to, else None."""
    if info["block_linked"] or nb < 2 * _FOLLOW_CHUNKS or bool(raw_mask.any()):
        return None
    dev = d_frame.device
    maxb = info["block_size"]
    status = torch.empty(nb, dtype=torch.int32, device=dev)
    crc_bad = None
    if info["block_checksum"]:
        sums = torch.empty(nb, dtype=torch.int32, device=dev)
        N.launch_xxh32_batch(d_frame, c_off, c_len.to(torch.int64), 0, sums, nb)
        crc_bad = (sums.to(torch.int64) & 0xFFFFFFFF) != _le32_at(d_frame, crc_pos)
    slots = torch.empty(nb * maxb + 16, dtype=torch.uint8, device=dev)
    slot_off = torch.arange(nb, dtype=torch.int64, device=dev) * maxb
    caps = torch.full((nb,), maxb, dtype=torch.int32, device=dev)
    bounds = [nb * k // _FOLLOW_CHUNKS for k in range(_FOLLOW_CHUNKS + 1)]
    spans = []
    for k in range(_FOLLOW_CHUNKS):
        lo, hi = bounds[k], bounds[k + 1]
        N.launch_decompress(d_frame, c_off[lo:hi], c_len[lo:hi], slots, slot_off[lo:hi], caps[lo:hi],
                            status[lo:hi], hi - lo)
        ev = torch.cuda.Event()
        ev.record()
        # full blocks only: the last block's size is known after the decode
        spans.append((lo * maxb, min(hi, nb - 1) * maxb, ev))
    hasher = _HashThread(lambda: N.xxh32_of_device_spans(slots, spans))
    hasher.start()
    try:
        # wait for the decode on the last launch's event, which releases the
        # GIL (a tensor read-back waits holding it, and the hash thread needs
        # it between chunks: r05p measured no overlap that way)
        spans[-1][2].synchronize()
        bad = status < 0
        if crc_bad is not None:
            bad = bad | crc_bad
        if bool(bad.any()):
            i = int(torch.nonzero(bad).flatten()[0])
            code = "blockChecksum_invalid" if crc_bad is not None and bool(crc_bad[i]) else "decompressionFailed"
            return None, 0, (i, code), None
        st = status.cpu()
        full = bool((st[: nb - 1] == maxb).all())
    finally:
        hasher.join()
    if not full:
        return None
    total = (nb - 1) * maxb + int(st[nb - 1])
    state = hasher.result()
    state = N.xxh32_of_device_spans(slots, [((nb - 1) * maxb, total, None)], state=state)
    return slots, total, None, state.digest()


def _decode_linked(d_frame, c_off, c_len, raw_mask, out, status, maxb):
    """Linked blocks: each block may reference the previous output
    (LZ4F_updateDict, lz4frame.c:1853-1856: LZ4_decompress_safe_usingDict
    with the last <= 64 KiB decoded), contiguously into `out`.

    Speculatively in rounds: every block decodes at once with the previous
    round's output as its dictionary (two buffers), until a round changes no
    byte and no status.  At that fixed point block k was decoded with the
    true output of block k-1 and, by induction from block 0 (no dictionary),
    every block equals the serial chain's.  A round is one launch of the
    one-wavefront-per-block decoder with the other buffer as dictionary
    (lz4m_decompress_batch_prefix; LZ4M_LINKED_DECODE=dict: the lane-per-
    block dictionary kernel).  This needs every block but the last to decode
    to exactly the block size (what LZ4F_compressFrame and the lz4 tool
    write); otherwise, or with LZ4M_LINKED_DECODE=serial, blocks decode in
    order on one wavefront (lz4m_decompress_chain)."""
    nb = c_off.numel()
    mode = os.environ.get("LZ4M_LINKED_DECODE", "")
    if nb <= 2 or mode == "serial":
        N.launch_decompress_chain(d_frame, c_off, c_len, raw_mask, out, status, nb, maxb)
        return
    dev = d_frame.device
    span = nb * maxb
    slot_off = torch.arange(nb, dtype=torch.int64, device=dev) * maxb
    caps = torch.full((nb,), maxb, dtype=torch.int32, device=dev)
    dec_len = torch.where(raw_mask, torch.zeros_like(c_len), c_len)
    dlen = torch.clamp(slot_off, max=65536)
    dict_off = slot_off - dlen
    dlen = dlen.to(torch.int32)
    # both buffers start zeroed: the decoder leaves a slot's bytes past the
    # block's decoded length untouched, so a short last block (or a failing
    # one) must see equal bytes there in both or the fixed point never shows
    out[:span].zero_()
    bufs = [out, torch.zeros_like(out)]
    sts = [torch.empty(nb, dtype=torch.int32, device=dev), torch.empty(nb, dtype=torch.int32, device=dev)]
    sel_r = torch.nonzero(raw_mask).flatten()
    for b in bufs:                                             # stored blocks: their bytes, every round
        if sel_r.numel():
            N.gather(d_frame, c_off[sel_r], c_len[sel_r], b, slot_off[sel_r], sel_r.numel())
    cur = 0
    for r in range(nb + 1):
        prev = cur ^ 1
        if mode == "dict":
            N.launch_decompress(d_frame, c_off, dec_len, bufs[cur], slot_off, caps, sts[cur], nb,
                                dict_buf=bufs[prev], dict_off=dict_off, dict_len=dlen)
        else:
            N.launch_decompress_prefix(d_frame, c_off, dec_len, bufs[cur], slot_off, caps, bufs[prev], dlen,
                                       sts[cur], nb)
        sts[cur] = torch.where(raw_mask, c_len, sts[cur])
        if r > 0 and torch.equal(sts[cur], sts[prev]) and torch.equal(bufs[cur][:span], bufs[prev][:span]):
            break
        cur = prev
    if bufs[cur] is not out:
        out[:span].copy_(bufs[cur][:span])
    _linked_status(d_frame, c_off, c_len, raw_mask, out, status, nb, maxb, sts[cur])


def _linked_status(d_frame, c_off, c_len, raw_mask, out, status, nb, maxb, st):
    """Accept the speculative result unless a block before the first failing
    one decoded short of the block size (then the blocks' positions differ
    from the slots: the serial chain decodes the frame instead)."""
    bad = st < 0
    upto = int(torch.nonzero(bad).flatten()[0]) if bool(bad.any()) else nb - 1
    if upto > 0 and not bool((st[:upto] == maxb).all()):       # a short block mid-frame: positions differ
        N.launch_decompress_chain(d_frame, c_off, c_len, raw_mask, out, status, nb, maxb)
        return
    status.copy_(st)
