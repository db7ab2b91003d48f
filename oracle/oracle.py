"""ctypes front-end for the CHECKERS (test infrastructure only).

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg import this module, and only to check or to time a
baseline.  The shipped package (``python-lz4_amd/lz4``) never imports it.

Two checkers live here:

* ``Oracle`` -- the CPU restatement in ``oracle/lz4_oracle.c``
  (``oracle/build/liboracle.so``);
* ``Reference`` -- the reference ``lz4libs`` v1.9.4 compiled from
  ``/root/reference`` by ``oracle/Makefile`` into ``oracle/_ref/``.  It is
  used to pin the restatement and to generate ``tests/golden``; it is absent
  on a box that never had the reference sources and no prebuilt ``_ref``.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ORACLE_SO = os.path.join(HERE, "build", "liboracle.so")
ORACLE_BENCH_SO = os.path.join(HERE, "build", "liboracle_bench.so")
REF_SO = os.path.join(HERE, "_ref", "libref_lz4.so")
REF_BENCH_SO = os.path.join(HERE, "_ref", "libref_bench.so")

TABLE_U16_HASH4 = 0
TABLE_U32_HASH5 = 1
LIMIT_64K = 65536 + 11


def build() -> None:
    """Compile the checkers (restatement always; reference when present)."""
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def _buf(data) -> tuple:
    arr = np.frombuffer(bytes(data), dtype=np.uint8) if not isinstance(data, np.ndarray) else data
    arr = np.ascontiguousarray(arr, dtype=np.uint8)
    return arr, arr.ctypes.data_as(C.c_void_p)


def compress_bound(n: int) -> int:
    return 0 if n < 0 or n > 0x7E000000 else n + n // 255 + 16


class Oracle:
    """The CPU restatement."""

    def __init__(self, path: str = ORACLE_SO):
        if not os.path.exists(path):
            build()
        lib = C.CDLL(path)
        vp, i32, i64, sz = C.c_void_p, C.c_int, C.c_int64, C.c_size_t
        lib.orc_compress.argtypes = [vp, i32, vp, i32, i32, i32]
        lib.orc_compress.restype = i32
        lib.orc_decompress_dict.argtypes = [vp, vp, i32, i32, vp, sz]
        lib.orc_decompress_dict.restype = i32
        lib.orc_xxh32.argtypes = [vp, sz, C.c_uint32]
        lib.orc_xxh32.restype = C.c_uint32
        lib.orc_xxh32_state_size.restype = sz
        lib.orc_xxh32_reset.argtypes = [vp, C.c_uint32]
        lib.orc_xxh32_update.argtypes = [vp, vp, sz]
        lib.orc_xxh32_digest.argtypes = [vp]
        lib.orc_xxh32_digest.restype = C.c_uint32
        lib.orc_compress_batch.argtypes = [vp, vp, vp, vp, vp, C.c_int32, vp, i64, i32, i32]
        lib.orc_decompress_batch.argtypes = [vp, vp, vp, vp, vp, vp, vp, i64]
        lib.orc_compress_dict.argtypes = [vp, i64, i32, vp, i32, i32]
        lib.orc_compress_dict.restype = i32
        lib.orc_compress_dict_mode.argtypes = [vp, i64, i32, vp, i32, i32, i32]
        lib.orc_compress_dict_mode.restype = i32
        lib.orc_compress_linked.argtypes = [vp, i64, i32, i32, vp, i64, vp]
        lib.orc_compress_linked.restype = i32
        self.lib = lib

    def compress(self, data, variant: int | None = None, accel: int = 1, cap: int | None = None) -> bytes | None:
        """``variant`` None = LZ4_compress_default's choice by size."""
        src, sp = _buf(data)
        n = src.size
        if variant is None:
            variant = TABLE_U16_HASH4 if n < LIMIT_64K else TABLE_U32_HASH5
        cap = compress_bound(n) if cap is None else cap
        dst = np.zeros(max(cap, 1), dtype=np.uint8)
        r = self.lib.orc_compress(sp, n, dst.ctypes.data_as(C.c_void_p), cap, variant, accel)
        return None if r <= 0 else dst[:r].tobytes()

    def compress_dict(self, data, dict_, accel: int = 1, prefix: bool = False) -> bytes | None:
        """lz4.block.compress(data, dict=dict_, store_size=False) (_block.c:93-107).
        ``prefix``: dict_'s memory ends where data begins (prefix mode, lz4.c:1671)."""
        d = bytes(dict_)
        tail = d[-65536:] if len(d) >= 8 else b""
        win, wp = _buf(tail + bytes(data))
        n = win.size - len(tail)
        cap = compress_bound(n)
        dst = np.zeros(max(cap, 1), dtype=np.uint8)
        r = self.lib.orc_compress_dict_mode(wp, len(d), n, dst.ctypes.data_as(C.c_void_p), cap, accel, int(prefix))
        return None if r <= 0 else dst[:r].tobytes()

    def compress_linked(self, data, block_size: int, accel: int = 1) -> list:
        """Per-block payloads of a linked frame: bytes, or None = stored raw."""
        src, sp = _buf(data)
        nb = (src.size + block_size - 1) // block_size
        stride = compress_bound(block_size)
        dst = np.zeros(max(nb, 1) * stride, dtype=np.uint8)
        out = np.zeros(max(nb, 1), dtype=np.int32)
        self.lib.orc_compress_linked(sp, src.size, block_size, accel, dst.ctypes.data_as(C.c_void_p), stride,
                                     out.ctypes.data_as(C.c_void_p))
        return [dst[k * stride: k * stride + out[k]].tobytes() if out[k] > 0 else None for k in range(nb)]

    def decompress(self, data, cap: int, dict_=None) -> tuple[int, bytes]:
        src, sp = _buf(data)
        dst = np.zeros(max(cap, 1) + 64, dtype=np.uint8)
        if dict_:
            d, dp = _buf(dict_)
            r = self.lib.orc_decompress_dict(sp, dst.ctypes.data_as(C.c_void_p), src.size, cap, dp, d.size)
        else:
            r = self.lib.orc_decompress_dict(sp, dst.ctypes.data_as(C.c_void_p), src.size, cap, None, 0)
        return r, (dst[:r].tobytes() if r >= 0 else b"")

    def xxh32(self, data, seed: int = 0) -> int:
        src, sp = _buf(data)
        return int(self.lib.orc_xxh32(sp, src.size, seed))

    def xxh32_stream(self, chunks, seed: int = 0) -> int:
        st = C.create_string_buffer(int(self.lib.orc_xxh32_state_size()))
        self.lib.orc_xxh32_reset(st, seed)
        for ch in chunks:
            a, ap = _buf(ch)
            self.lib.orc_xxh32_update(st, ap, a.size)
        return int(self.lib.orc_xxh32_digest(st))


class Reference:
    """The reference lz4libs built from /root/reference by oracle/Makefile."""

    def __init__(self, path: str = REF_SO):
        if not os.path.exists(path):
            build()
        if not os.path.exists(path):
            raise FileNotFoundError(path)
        lib = C.CDLL(path)
        vp, i32, sz = C.c_void_p, C.c_int, C.c_size_t
        lib.LZ4_compress_default.argtypes = [vp, vp, i32, i32]
        lib.LZ4_compress_default.restype = i32
        lib.LZ4_compress_fast.argtypes = [vp, vp, i32, i32, i32]
        lib.LZ4_compress_fast.restype = i32
        lib.LZ4_decompress_safe.argtypes = [vp, vp, i32, i32]
        lib.LZ4_decompress_safe.restype = i32
        lib.LZ4_decompress_safe_usingDict.argtypes = [vp, vp, i32, i32, vp, i32]
        lib.LZ4_decompress_safe_usingDict.restype = i32
        lib.LZ4_sizeofState.restype = i32
        lib.LZ4_resetStream.argtypes = [vp]
        lib.LZ4_compress_fast_continue.argtypes = [vp, vp, vp, i32, i32, i32]
        lib.LZ4_compress_fast_continue.restype = i32
        lib.LZ4_loadDict.argtypes = [vp, vp, i32]
        lib.LZ4_loadDict.restype = i32
        lib.XXH32.argtypes = [vp, sz, C.c_uint32]
        lib.XXH32.restype = C.c_uint32
        lib.LZ4_versionNumber.restype = i32
        lib.LZ4F_compressFrameBound.argtypes = [sz, vp]
        lib.LZ4F_compressFrameBound.restype = sz
        lib.LZ4F_compressFrame.argtypes = [vp, sz, vp, sz, vp]
        lib.LZ4F_compressFrame.restype = sz
        lib.LZ4F_isError.argtypes = [sz]
        lib.LZ4F_isError.restype = C.c_uint
        self.lib = lib

    def version(self) -> int:
        return int(self.lib.LZ4_versionNumber())

    def compress_default(self, data) -> bytes:
        src, sp = _buf(data)
        cap = compress_bound(src.size)
        dst = np.zeros(cap, dtype=np.uint8)
        r = self.lib.LZ4_compress_default(sp, dst.ctypes.data_as(C.c_void_p), src.size, cap)
        return dst[:r].tobytes()

    def compress_block_api(self, data, accel: int = 1) -> bytes:
        """lz4.block.compress(mode='default'|'fast', store_size=False): _block.c:93-121."""
        src, sp = _buf(data)
        cap = compress_bound(src.size)
        dst = np.zeros(cap, dtype=np.uint8)
        state = C.create_string_buffer(int(self.lib.LZ4_sizeofState()))
        self.lib.LZ4_resetStream(state)
        r = self.lib.LZ4_compress_fast_continue(state, sp, dst.ctypes.data_as(C.c_void_p), src.size, cap, accel)
        return dst[:r].tobytes()

    def compress_dict(self, data, dict_, accel: int = 1) -> bytes:
        """lz4.block.compress(data, dict=dict_, store_size=False): _block.c:93-107."""
        src, sp = _buf(data)
        d = np.frombuffer(bytes(dict_) + b"\0", dtype=np.uint8)   # never a NULL buffer, like Py_buffer
        cap = compress_bound(src.size)
        dst = np.zeros(max(cap, 1), dtype=np.uint8)
        state = C.create_string_buffer(int(self.lib.LZ4_sizeofState()))
        self.lib.LZ4_resetStream(state)
        self.lib.LZ4_loadDict(state, d.ctypes.data_as(C.c_void_p), d.size - 1)
        r = self.lib.LZ4_compress_fast_continue(state, sp, dst.ctypes.data_as(C.c_void_p), src.size, cap, accel)
        return dst[:r].tobytes()

    def compress_dict_prefix(self, data, dict_, accel: int = 1) -> bytes:
        """lz4.block.compress(data, dict=dict_) when dict_'s memory ends exactly
        where data begins (memoryview slices of one buffer): the reference's
        LZ4_compress_fast_continue then sees dictEnd == source (lz4.c:1671)."""
        buf = np.frombuffer(bytes(dict_) + bytes(data) + b"\0", dtype=np.uint8)
        base = buf.ctypes.data
        n = len(data)
        cap = compress_bound(n)
        dst = np.zeros(max(cap, 1), dtype=np.uint8)
        state = C.create_string_buffer(int(self.lib.LZ4_sizeofState()))
        self.lib.LZ4_resetStream(state)
        self.lib.LZ4_loadDict(state, C.c_void_p(base), len(dict_))
        r = self.lib.LZ4_compress_fast_continue(state, C.c_void_p(base + len(dict_)), dst.ctypes.data_as(C.c_void_p),
                                                n, cap, accel)
        return dst[:r].tobytes()

    def decompress(self, data, cap: int, dict_=None) -> tuple[int, bytes]:
        src, sp = _buf(data)
        dst = np.zeros(max(cap, 1) + 64, dtype=np.uint8)
        if dict_:
            d, dp = _buf(dict_)
            r = self.lib.LZ4_decompress_safe_usingDict(sp, dst.ctypes.data_as(C.c_void_p), src.size, cap, dp, d.size)
        else:
            r = self.lib.LZ4_decompress_safe(sp, dst.ctypes.data_as(C.c_void_p), src.size, cap)
        return r, (dst[:r].tobytes() if r >= 0 else b"")

    def xxh32(self, data, seed: int = 0) -> int:
        src, sp = _buf(data)
        return int(self.lib.XXH32(sp, src.size, seed))

    def compress_frame(self, data, block_size_id: int = 7, linked: bool = False,
                       content_checksum: bool = True, block_checksum: bool = False,
                       store_size: bool = True, level: int = 0) -> bytes:
        """LZ4F_compressFrame with explicit preferences (lz4frame.c:475-515)."""

        class FrameInfo(C.Structure):
            _fields_ = [("blockSizeID", C.c_int), ("blockMode", C.c_int),
                        ("contentChecksumFlag", C.c_int), ("frameType", C.c_int),
                        ("contentSize", C.c_ulonglong), ("dictID", C.c_uint),
                        ("blockChecksumFlag", C.c_int)]

        class Prefs(C.Structure):
            _fields_ = [("frameInfo", FrameInfo), ("compressionLevel", C.c_int),
                        ("autoFlush", C.c_uint), ("favorDecSpeed", C.c_uint),
                        ("reserved", C.c_uint * 3)]

        src, sp = _buf(data)
        p = Prefs()
        p.frameInfo.blockSizeID = block_size_id
        p.frameInfo.blockMode = 0 if linked else 1
        p.frameInfo.contentChecksumFlag = 1 if content_checksum else 0
        p.frameInfo.blockChecksumFlag = 1 if block_checksum else 0
        p.frameInfo.contentSize = src.size if store_size else 0
        p.compressionLevel = level
        cap = self.lib.LZ4F_compressFrameBound(src.size, C.byref(p))
        dst = np.zeros(cap, dtype=np.uint8)
        r = self.lib.LZ4F_compressFrame(dst.ctypes.data_as(C.c_void_p), cap, sp, src.size, C.byref(p))
        if self.lib.LZ4F_isError(r):
            raise RuntimeError("LZ4F_compressFrame failed")
        return dst[:r].tobytes()


    def decompress_frame_into(self, data, dst: np.ndarray) -> int:
        """LZ4F_decompress of one whole frame into dst (large enough for the
        content) in one call sequence (lz4frame.c:1556-2058); returns the
        bytes written (bench's frame CPU reference; errors raise)."""
        lib = self.lib
        vp, sz = C.c_void_p, C.c_size_t
        lib.LZ4F_createDecompressionContext.argtypes = [C.POINTER(vp), C.c_uint]
        lib.LZ4F_createDecompressionContext.restype = sz
        lib.LZ4F_freeDecompressionContext.argtypes = [vp]
        lib.LZ4F_decompress.argtypes = [vp, vp, C.POINTER(sz), vp, C.POINTER(sz), vp]
        lib.LZ4F_decompress.restype = sz
        src, sp = _buf(data)
        ctx = vp()
        lib.LZ4F_createDecompressionContext(C.byref(ctx), 100)
        pos = out = 0
        try:
            while True:
                dsz = sz(dst.size - out)
                ssz = sz(src.size - pos)
                r = lib.LZ4F_decompress(ctx, dst.ctypes.data + out, C.byref(dsz), src.ctypes.data + pos,
                                        C.byref(ssz), None)
                out += dsz.value
                pos += ssz.value
                if lib.LZ4F_isError(r):
                    raise RuntimeError("LZ4F_decompress failed")
                if r == 0:
                    return out
                if dsz.value == 0 and ssz.value == 0:
                    raise RuntimeError("LZ4F_decompress made no progress")
        finally:
            lib.LZ4F_freeDecompressionContext(ctx)


class CpuBench:
    """Throughput harness over the reference build (kind 'reference') or the
    restatement (kind 'port')."""

    def __init__(self):
        if os.path.exists(REF_BENCH_SO):
            self.kind, path = "reference", REF_BENCH_SO
        else:
            if not os.path.exists(ORACLE_BENCH_SO):
                build()
            self.kind, path = "port", ORACLE_BENCH_SO
        lib = C.CDLL(path)
        vp = C.c_void_p
        lib.cpu_bench_run.argtypes = [C.c_int, C.c_int, C.c_int, vp, vp, vp, vp, vp, vp, vp, C.c_int64]
        lib.cpu_bench_run.restype = C.c_double
        self.lib = lib

    def run(self, op: str, threads: int, reps: int, src: np.ndarray, src_off: np.ndarray,
            src_len: np.ndarray, dst: np.ndarray, dst_off: np.ndarray, dst_cap: np.ndarray) -> tuple[float, np.ndarray]:
        code = {"compress": 0, "decompress": 1, "xxh32": 2}[op]
        out = np.zeros(src_off.size, dtype=np.int32)
        ptr = lambda a: a.ctypes.data_as(C.c_void_p)
        secs = self.lib.cpu_bench_run(code, threads, reps, ptr(src), ptr(src_off), ptr(src_len),
                                      ptr(dst), ptr(dst_off), ptr(dst_cap), ptr(out), src_off.size)
        return secs, out


def ref_decompress_frame(ref: "Reference", data: bytes) -> tuple[int, bytes]:
    """Decode one frame with the reference LZ4F_decompress (test helper).
    Returns (error code or 0, decoded bytes)."""
    lib = ref.lib
    vp, sz = C.c_void_p, C.c_size_t
    lib.LZ4F_createDecompressionContext.argtypes = [C.POINTER(vp), C.c_uint]
    lib.LZ4F_createDecompressionContext.restype = sz
    lib.LZ4F_freeDecompressionContext.argtypes = [vp]
    lib.LZ4F_decompress.argtypes = [vp, vp, C.POINTER(sz), vp, C.POINTER(sz), vp]
    lib.LZ4F_decompress.restype = sz
    lib.LZ4F_getErrorName.argtypes = [sz]
    lib.LZ4F_getErrorName.restype = C.c_char_p
    ctx = vp()
    lib.LZ4F_createDecompressionContext(C.byref(ctx), 100)
    src = np.frombuffer(bytes(data), dtype=np.uint8)
    out = bytearray()
    pos = 0
    buf = np.zeros(1 << 23, dtype=np.uint8)
    try:
        while True:
            dsz = sz(buf.size)
            ssz = sz(src.size - pos)
            r = lib.LZ4F_decompress(ctx, buf.ctypes.data_as(vp), C.byref(dsz),
                                    (src.ctypes.data + pos) if src.size else None, C.byref(ssz), None)
            out += buf[:dsz.value].tobytes()
            pos += ssz.value
            if lib.LZ4F_isError(r):
                return -1, lib.LZ4F_getErrorName(r).decode()
            if r == 0:
                return 0, bytes(out)
            if pos >= src.size and dsz.value == 0:
                return 1, bytes(out)
    finally:
        lib.LZ4F_freeDecompressionContext(ctx)
