"""CPU tests of the drop-in boundary: the C-ABI library loads and exports
every symbol include/lz4m.h declares; argument checks that need no GPU."""
import ctypes as C
import os
import re

import pytest

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "lz4m.h")


def declared_symbols():
    txt = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:[\w\s\*]+?)\b(lz4m_\w+)\s*\(", txt, re.M)))


def test_header_declares_entry_points():
    syms = declared_symbols()
    for s in ["lz4m_decompress_batch", "lz4m_decompress_batch_dict", "lz4m_decompress_chain",
              "lz4m_compress_batch", "lz4m_xxh32_batch", "lz4m_xxh32_long", "lz4m_compress_bound",
              "lz4m_exclusive_scan", "lz4m_gather", "lz4m_frame_emit", "lz4m_frame_block_sizes",
              "lz4m_frame_scan", "lz4m_decompress_safe", "lz4m_compress_default", "lz4m_compress_block_api",
              "lz4m_xxh32"]:
        assert s in syms, s


def test_library_exports_every_declared_symbol():
    from lz4 import _native as N
    lib = N.lib()
    for s in declared_symbols():
        assert hasattr(lib, s), f"{s} declared in include/lz4m.h but not exported"


def test_compress_bound_and_version():
    from lz4 import _native as N
    lib = N.lib()
    for n in [0, 1, 255, 65536, 1 << 20, 0x7E000000]:
        assert lib.lz4m_compress_bound(n) == n + n // 255 + 16
    assert lib.lz4m_compress_bound(0x7E000001) == 0
    assert lib.lz4m_compress_bound(-1) == 0
    assert lib.lz4m_version_number() == 10904


def test_header_compiles_as_c():
    """include/lz4m.h is a plain C header (a cgo / ctypes / C-extension caller
    includes it): gcc -std=c99 -Wall accepts it."""
    import subprocess
    import tempfile
    with tempfile.TemporaryDirectory() as d:
        c = os.path.join(d, "t.c")
        open(c, "w").write('#include "lz4m.h"\nint main(void) { return LZ4M_TABLE_U16_HASH4; }\n')
        r = subprocess.run(["gcc", "-std=c99", "-Wall", "-Werror", "-I", os.path.dirname(HEADER), "-c", c, "-o",
                            os.path.join(d, "t.o")], capture_output=True, text=True)
        assert r.returncode == 0, r.stderr


def test_argument_validation_without_gpu():
    """n == 0 is a no-op and n < 0 is rejected before any HIP call."""
    from lz4 import _native as N
    lib = N.lib()
    assert lib.lz4m_decompress_batch(None, None, None, None, None, None, None, 0, None) == 0
    assert lib.lz4m_decompress_batch(None, None, None, None, None, None, None, -1, None) == N.EINVAL
    assert lib.lz4m_compress_batch(None, None, None, None, None, None, None, 0, 0, 1, None) == 0
    assert lib.lz4m_compress_batch(None, None, None, None, None, None, None, -5, 0, 1, None) == N.EINVAL
    assert lib.lz4m_compress_dict_batch(None, None, None, None, None, None, None, None, 0, 1, None) == 0
    assert lib.lz4m_compress_dict_batch(None, None, None, None, None, None, None, None, -1, 1, None) == N.EINVAL
    for mode in (N.LINKED_SERIAL, N.LINKED_SPECULATIVE):
        assert lib.lz4m_compress_linked_batch(None, None, None, None, None, None, None, None, 0, 1, mode,
                                              None, 0, None) == 0
    assert lib.lz4m_compress_linked_batch(None, None, None, None, None, None, None, None, 4, 1, 7,
                                          None, 0, None) == N.EINVAL
    # speculative mode without enough scratch is refused before any launch
    assert lib.lz4m_compress_linked_batch(None, None, None, None, None, None, None, None, 4, 1,
                                          N.LINKED_SPECULATIVE, None, 0, None) == N.EINVAL
    assert lib.lz4m_compress_linked_workspace_size(4) >= 4 * 2 * 16384
    # segmented large-block parse: no-op, bad sizes, missing scratch
    assert lib.lz4m_pcompress_large_batch(None, None, None, None, None, None, None, 0, 1 << 22, None, 0, None) == 0
    assert lib.lz4m_pcompress_large_batch(None, None, None, None, None, None, None, -1, 1 << 22, None, 0,
                                          None) == N.EINVAL
    assert lib.lz4m_pcompress_large_batch(None, None, None, None, None, None, None, 4, 1 << 22, None, 0,
                                          None) == N.EINVAL
    # 16 slots of >= LZ4_compressBound(256 KiB) per block, and 16 per-slot records
    assert lib.lz4m_pcompress_large_workspace_size(2, 1 << 22) >= 2 * 16 * (N.compress_bound(1 << 18) + 16)
    #  slots per block = the longest block's segment count: 256 KiB
    # blocks are one segment each, so the scratch is about the input's size
    n = 4096
    for size, segs in ((1 << 18, 1), (1 << 20, 4), ((1 << 20) + 1, 5)):
        ws = lib.lz4m_pcompress_large_workspace_size(n, size)
        assert n * segs * N.compress_bound(1 << 18) <= ws <= n * segs * (N.compress_bound(1 << 18) + 128) + 256
    assert lib.lz4m_xxh32_batch(None, None, None, 0, None, -1, None) == N.EINVAL
    # retired decoder ids (1 lane, 2 coop, 5 direct, 6) and unknown ids are rejected before any launch
    for dec in (1, 2, 5, 6, 8, -1):
        assert lib.lz4m_decompress_batch_sel(None, None, None, None, None, None, None, 0, None, 0, dec,
                                             None) == N.EINVAL
    for dec in N.DECODERS.values():
        assert lib.lz4m_decompress_batch_sel(None, None, None, None, None, None, None, 0, None, 0, dec, None) == 0
    assert lib.lz4m_xxh32_long(None, -1, 0, None, None) == N.EINVAL
    assert lib.lz4m_frame_scan(None, -1, 0, 0, 0, 65536, 1, None, None, None, None, None) == N.EINVAL
    assert lib.lz4m_frame_scan(None, 16, 0, 0, 0, 65536, 1, None, None, None, None, None) == N.EINVAL
    # host single-buffer functions reject bad sizes before touching a device
    assert lib.lz4m_decompress_safe(None, None, -1, 10) == -1
    assert lib.lz4m_compress_default(None, None, -1, 10) == 0
    assert lib.lz4m_compress_default(None, None, 0x7E000001, 10) == 0


def test_no_cpu_fallback():
    """Without a HIP device every compute entry point raises (no silent CPU path)."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    import lz4.block
    import lz4.frame
    with pytest.raises(RuntimeError, match="no HIP device"):
        lz4.block.compress(b"abc" * 100)
    with pytest.raises(RuntimeError, match="no HIP device"):
        lz4.block.decompress(b"\x01\x00\x00\x00\x10 ")
    with pytest.raises(RuntimeError, match="no HIP device"):
        lz4.frame.compress(b"abc")


def test_package_does_not_import_oracle():
    pkg = os.path.join(ROOT, "python-lz4_amd", "lz4")
    for dirpath, _, files in os.walk(pkg):
        for f in files:
            if f.endswith(".py"):
                src = open(os.path.join(dirpath, f)).read()
                assert "import oracle" not in src and "liboracle" not in src and "libref_" not in src, f


def test_block_api_argument_errors_without_gpu():
    """Argument checks of _block.c that happen before any codec call."""
    import lz4.block
    with pytest.raises(TypeError):
        lz4.block.compress("a str")
    with pytest.raises(OverflowError):
        lz4.block.decompress(b"abcd", uncompressed_size=(1 << 32) + 64)
    with pytest.raises(ValueError, match="Invalid mode argument"):
        lz4.block.compress(b"x", mode="nope")


def test_hot_kernels_use_no_scratch():
    """Every device kernel compiles without scratch (stack) memory: a spill
    of the lane state to scratch multiplies HBM traffic (observed: 25x the
    algorithmic write bytes).  Reads the compiler's resource report that the
    csrc Makefile keeps next to each object."""
    import glob
    import subprocess
    csrc = os.path.join(ROOT, "python-lz4_amd", "csrc")
    subprocess.run(["make", "-s", "-C", csrc], check=True, capture_output=True)
    reports = glob.glob(os.path.join(csrc, "build", "*.res"))
    assert reports, "no resource reports; build with the csrc Makefile"
    seen = 0
    for rep in reports:
        name = None
        for line in open(rep):
            m = re.search(r"Function Name: (\S+)", line)
            if m:
                name = m.group(1)
            m = re.search(r"ScratchSize \[bytes/lane\]: (\d+)", line)
            if m and name:
                assert int(m.group(1)) == 0, f"{name} uses {m.group(1)} B/lane of scratch"
                seen += 1
    assert seen >= 8


def test_host_xxh32_matches_oracle_and_golden():
    """The host streaming XXH32 of the C-ABI (the frame content checksum,
    lz4m_xxh32_host_*) equals the oracle and the golden XXH32 values, for any
    chunking of the stream (xxhash.c:437-554)."""
    import json
    import random

    import numpy as np
    import oracle as O
    from conftest import GOLDEN
    from lz4 import _native as N
    orc = O.Oracle()
    rnd = random.Random(7)
    for n in [0, 1, 3, 4, 15, 16, 17, 31, 32, 33, 255, 4096, 65536 + 3]:
        b = rnd.randbytes(n)
        for seed in (0, 1, 0x9E3779B1):
            assert N.xxh32_host(b, seed) == orc.xxh32(b, seed)
            h = N.HostXXH32(seed)
            pos = 0
            while pos < n:
                k = rnd.randrange(1, 40)
                h.update(b[pos:pos + k])
                pos += k
            assert h.digest() == orc.xxh32(b, seed)
    man = json.load(open(os.path.join(GOLDEN, "manifest.json")))
    arr = np.load(os.path.join(GOLDEN, "golden.npz"), allow_pickle=False)
    inputs = {e["name"]: arr[e["key"]].tobytes() for e in man["inputs"]}
    checked = 0
    for e in man["xxh32"]:
        data = inputs.get(e.get("input")) if "input" in e else arr[e["key"]].tobytes() if "key" in e else None
        if data is None:
            continue
        assert N.xxh32_host(data, e.get("seed", 0)) == e["value"], e
        checked += 1
    assert checked > 0


def test_single_call_worker_controls_without_gpu():
    """lz4m_single_call_worker switches and reports the single-call mode, and
    lz4m_single_call_worker_state reads this thread's (never started) workers:
    neither makes a HIP call, so both work without a GPU."""
    from lz4 import _native as N
    lib = N.lib()
    prev = lib.lz4m_single_call_worker(-1)
    assert prev in (0, 1)
    try:
        assert lib.lz4m_single_call_worker(1) == prev
        assert lib.lz4m_single_call_worker(-1) == 1
        assert lib.lz4m_single_call_worker(7) == 1       # not a mode: query only
        st = (C.c_uint32 * 16)()
        assert lib.lz4m_single_call_worker_state(st) == 0
        assert list(st) == [0] * 16
    finally:
        lib.lz4m_single_call_worker(prev)
