"""CPU tests: the oracle (oracle/lz4_oracle.c) against the golden vectors
generated from the reference lz4libs (tests/golden/make_golden.py), plus a
differential fuzz against the reference build when it is present."""
import json
import os
import random

import numpy as np
import pytest

from conftest import GOLDEN


@pytest.fixture(scope="module")
def golden():
    with open(os.path.join(GOLDEN, "manifest.json")) as f:
        man = json.load(f)
    arr = np.load(os.path.join(GOLDEN, "golden.npz"), allow_pickle=False)
    return man, arr


def _b(arr, key):
    return arr[key].tobytes()


def test_golden_is_v194(golden):
    man, _ = golden
    assert man["version"] == 10904


def test_compress_matches_golden(oracle, golden):
    man, arr = golden
    inputs = {e["name"]: _b(arr, e["key"]) for e in man["inputs"]}
    n = 0
    for e in man["compress"]:
        data = inputs[e["input"]]
        if e["mode"] == "default":
            got = oracle.compress(data)
        else:
            got = oracle.compress(data, 1, accel=e["accel"])
        assert got == _b(arr, e["key"]), (e["input"], e["mode"], e["accel"])
        n += 1
    assert n > 80


def test_decompress_status_matches_golden(oracle, golden):
    man, arr = golden
    for e in man["decompress"]:
        st, _ = oracle.decompress(_b(arr, e["key"]), e["cap"])
        assert st == e["status"], (e["key"], e["cap"])


def test_decompress_roundtrip_golden(oracle, golden):
    man, arr = golden
    inputs = {e["name"]: _b(arr, e["key"]) for e in man["inputs"]}
    for e in man["compress"]:
        data = inputs[e["input"]]
        st, out = oracle.decompress(_b(arr, e["key"]), len(data))
        assert st == len(data) and out == data


def test_kat(oracle, golden):
    man, arr = golden
    for e in man["kat"]:
        comp = _b(arr, e["key"])
        st, out = oracle.decompress(comp[4:], int.from_bytes(comp[:4], "little"))
        assert st == e["status"]
        assert out == _b(arr, e["plain"])


def test_xxh32_golden(oracle, golden):
    man, arr = golden
    inputs = {e["name"]: _b(arr, e["key"]) for e in man["inputs"]}
    rng = random.Random(4)
    for e in man["xxh32"]:
        data = inputs[e["input"]]
        assert oracle.xxh32(data, e["seed"]) == e["value"]
        # streaming in random chunks equals one-shot (xxhash.c:451-554)
        cuts = sorted(rng.randrange(len(data) + 1) for _ in range(3))
        chunks = [data[a:b] for a, b in zip([0] + cuts, cuts + [len(data)])]
        assert oracle.xxh32_stream(chunks, e["seed"]) == e["value"]


def test_xxh32_vs_pip_xxhash(oracle):
    xxhash = pytest.importorskip("xxhash")
    rng = np.random.default_rng(1)
    for n in list(range(0, 70)) + [1000, 4096, 65537]:
        d = rng.integers(0, 256, size=n, dtype=np.uint8).tobytes()
        assert oracle.xxh32(d) == xxhash.xxh32_intdigest(d)


def test_frame_fixtures_decode_with_oracle(oracle, golden):
    """The reference frames' block records parse with the host scanner of
    lz4.frame and every block decodes (oracle) to the original input."""
    import struct
    from lz4.frame._frame import _BLOCK_SIZES, _scan_blocks
    man, arr = golden
    inputs = {e["name"]: _b(arr, e["key"]) for e in man["inputs"]}
    for e in man["frames"]:
        fr = memoryview(_b(arr, e["key"]))
        flg, bd = fr[4], fr[5]
        hsize = 7 + (8 if flg & 8 else 0) + (4 if flg & 1 else 0)
        info = {"block_checksum": bool(flg & 0x10), "content_checksum": bool(flg & 4),
                "block_size": _BLOCK_SIZES[(bd >> 4) & 7], "block_linked": not (flg & 0x20)}
        recs, state = _scan_blocks(fr, hsize, info)
        assert state[0] == "end" and state[1] == len(fr)
        out = b""
        for raw, pos, size, crc in recs:
            blk = bytes(fr[pos:pos + size])
            if raw:
                out += blk
            elif info["block_linked"]:
                st, dec = oracle.decompress(blk, info["block_size"], dict_=out[-65536:] if out else None)
                assert st >= 0
                out += dec
            else:
                st, dec = oracle.decompress(blk, info["block_size"])
                assert st >= 0
                out += dec
            if crc >= 0:
                assert struct.unpack_from("<I", fr, crc)[0] == oracle.xxh32(blk)
        assert out == inputs[e["input"]]
        if info["content_checksum"]:
            assert struct.unpack_from("<I", fr, len(fr) - 4)[0] == oracle.xxh32(out)


def _frame_blocks(fr: bytes):
    """(block size, linked, [(raw, payload)]) of a frame, by the host scanner."""
    from lz4.frame._frame import _BLOCK_SIZES, _scan_blocks
    fr = memoryview(fr)
    flg, bd = fr[4], fr[5]
    hsize = 7 + (8 if flg & 8 else 0)
    info = {"block_checksum": bool(flg & 0x10), "content_checksum": bool(flg & 4),
            "block_size": _BLOCK_SIZES[(bd >> 4) & 7], "block_linked": not (flg & 0x20)}
    recs, state = _scan_blocks(fr, hsize, info)
    assert state[0] == "end"
    return info["block_size"], info["block_linked"], [(raw, bytes(fr[pos:pos + size])) for raw, pos, size, _ in recs]


def test_linked_frames_golden(oracle, golden):
    """orc_compress_linked reproduces every block of the reference's linked
    frames (LZ4F_compressBlock_continue, lz4frame.c:865-871)."""
    man, arr = golden
    inputs = {e["name"]: _b(arr, e["key"]) for e in man["inputs"]}
    n = 0
    for e in man["frames"]:
        o = e["opts"]
        if not o.get("linked"):
            continue
        bsize, linked, recs = _frame_blocks(_b(arr, e["key"]))
        assert linked
        lvl = o.get("level", 0)
        got = oracle.compress_linked(inputs[e["input"]], bsize, -lvl + 1 if lvl < 0 else 1)
        assert len(got) == len(recs)
        for g, (raw, payload) in zip(got, recs):
            assert (g is None) == raw
            if not raw:
                assert g == payload
        n += 1
    assert n >= 4


def test_dict_compress_golden(oracle, golden):
    """orc_compress_dict reproduces lz4.block.compress(dict=) (_block.c:101-104)."""
    man, arr = golden
    inputs = {e["name"]: _b(arr, e["key"]) for e in man["inputs"]}
    assert len(man["dict_compress"]) >= 10
    for e in man["dict_compress"]:
        got = oracle.compress_dict(inputs[e["input"]], _b(arr, e["dict"]), e["accel"])
        assert got == _b(arr, e["key"]), e


def test_dict_prefix_compress_golden(oracle, golden):
    """Dictionary memory ending where the source begins: the reference takes
    prefix mode (lz4.c:1671-1676), and the restatement reproduces it; at least
    a dozen of the golden cases differ from the extDict bytes."""
    man, arr = golden
    cases = man["dict_prefix_compress"]
    assert sum(e["extdict_differs"] for e in cases) >= 10
    for e in cases:
        data, d = _b(arr, e["input"]), _b(arr, e["dict"])
        assert oracle.compress_dict(data, d, e["accel"], prefix=True) == _b(arr, e["key"]), e
        assert (oracle.compress_dict(data, d, e["accel"]) != _b(arr, e["key"])) == e["extdict_differs"], e


def test_dict_prefix_vs_reference(oracle, reference):
    """Differential against the compiled reference: prefix-mode dict= over
    random cuts of one buffer (dictionary 8 B .. > 64 KiB)."""
    from lz4 import _synth
    rng = random.Random(1671)
    for kind in ("text", "records", "runs", "silesia"):
        blob = _synth.blocks(3, kind, seed=5).tobytes()
        for _ in range(25):
            cut = rng.randrange(8, len(blob) - 8)
            dl = min(rng.choice([8, 12, 50, 300, 5000, 65536, 70000]), cut)
            n = min(rng.choice([1, 13, 700, 4000, 65536]), len(blob) - cut)
            d, s = blob[cut - dl:cut], blob[cut:cut + n]
            acc = rng.choice([1, 2, 9])
            assert oracle.compress_dict(s, d, acc, prefix=True) == reference.compress_dict_prefix(s, d, acc), \
                (kind, cut, dl, n, acc)


def test_dict_and_linked_vs_reference(oracle, reference):
    """Differential: dictionary lengths around every LZ4_loadDict boundary
    (< 8, 64 KiB, > 64 KiB) and linked frames of every block size."""
    from lz4 import _synth
    rng = random.Random(12)
    for kind in ("text", "records", "random", "runs"):
        blob = _synth.blocks(4, kind, seed=21).tobytes()
        for dl in (0, 3, 7, 8, 9, 64, 5000, 65535, 65536, 65537, 131072):
            for sl in (0, 12, 13, 777, 65536, 70000):
                o = rng.randrange(0, len(blob) - sl - dl + 1)
                d, s = blob[o:o + dl], blob[o + dl:o + dl + sl]
                assert oracle.compress_dict(s, d) == reference.compress_dict(s, d), (kind, dl, sl)
        for bsid, bs in ((4, 65536), (5, 262144)):
            fr = reference.compress_frame(blob, block_size_id=bsid, linked=True, content_checksum=False)
            _, _, recs = _frame_blocks(fr)
            got = oracle.compress_linked(blob, bs)
            assert [g for g in got] == [None if raw else p for raw, p in recs], (kind, bs)


def test_optimal_bsid():
    from lz4.frame._frame import _optimal_bsid
    assert _optimal_bsid(0, 10) == 0
    assert _optimal_bsid(7, 10) == 4
    assert _optimal_bsid(7, 65537) == 5
    assert _optimal_bsid(7, 300000) == 6
    assert _optimal_bsid(7, 5 << 20) == 7
    assert _optimal_bsid(4, 5 << 20) == 4


def test_differential_vs_reference(oracle, reference):
    """Oracle vs the reference build on fresh random cases (this container)."""
    from lz4 import _synth
    rng = random.Random(99)
    blocks = _synth.blocks(16, "silesia", seed=123)
    for i in range(300):
        b = blocks[rng.randrange(16)].tobytes()
        n = rng.choice([0, 3, 13, 50, 700, 5000, 65536])
        o = rng.randrange(0, 65536 - n + 1)
        x = b[o:o + n]
        assert oracle.compress(x) == reference.compress_default(x)
        acc = rng.choice([1, 1, 3, 50])
        assert oracle.compress(x, 1, accel=acc) == reference.compress_block_api(x, acc)
        c = bytearray(reference.compress_default(x))
        for _ in range(rng.randrange(3)):
            if c:
                c[rng.randrange(len(c))] = rng.randrange(256)
        cap = rng.choice([n, n + 5, max(0, n - 2)])
        assert oracle.decompress(bytes(c), cap) == reference.decompress(bytes(c), cap)
        d = b[:rng.randrange(1, 70000)]
        if c:
            assert oracle.decompress(bytes(c), cap, dict_=d) == reference.decompress(bytes(c), cap, dict_=d)


def test_host_sanitizers():
    """the CPU restatement and the package's host XXH32
    (lz4m_xxh32_host.c) under AddressSanitizer + UBSan (oracle/Makefile
    `asan`, driver oracle/asan_check.c): exact-size buffers over valid,
    truncated, mutated and garbage blocks, dict= and linked streams, XXH32
    in random chunks."""
    import shutil
    import subprocess
    if shutil.which("gcc") is None:
        pytest.skip("no host C compiler")
    root = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "oracle")
    r = subprocess.run(["make", "-s", "-C", root, "asan"], capture_output=True, text=True, timeout=600)
    if r.returncode != 0 and "cannot find" in (r.stderr or "") and "asan" in r.stderr:
        pytest.skip("sanitizer runtime not installed")
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "asan_check: ok" in r.stdout
