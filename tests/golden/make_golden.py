"""Generate tests/golden/golden.npz + manifest.json from the REFERENCE.

Run in the build container (needs /root/reference): it builds oracle/_ref
(the reference lz4libs compiled from its own sources by oracle/Makefile) and
records inputs and the reference's outputs:
  * LZ4_compress_default and lz4.block.compress (LZ4_compress_fast_continue on
    a reset stream, _block.c:93-121) outputs, incl. acceleration variants;
  * LZ4_decompress_safe status (size or -(pos)-1) for valid and malformed
    blocks (mutations, truncations, capacities);
  * XXH32 of every input for several seeds;
  * LZ4F_compressFrame frames for several preference sets (independent and
    linked blocks);
  * lz4.block.compress(dict=) outputs (LZ4_resetStream + LZ4_loadDict +
    LZ4_compress_fast_continue, _block.c:93-107) for dictionaries of 0..100000 B;
  * the same with the dictionary's memory ending where the source begins
    (prefix mode, lz4.c:1671-1676), as memoryview slices of one buffer give;
  * the reference tests' own data file tests/block/numpy_byte_array.bin and
    the known-answer vectors of tests/block/test_block_1.py:128-149.
Vectors are data only; nothing of the reference's source is stored.
"""
import json
import os
import random
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "python-lz4_amd"))
import oracle as O  # noqa: E402
from lz4 import _synth  # noqa: E402

REF_DATA = "/root/reference/tests/block/numpy_byte_array.bin"


def main():
    O.build()
    ref = O.Reference()
    rng = random.Random(20261015)
    arrays, man = {}, {"version": ref.version(), "inputs": [], "compress": [], "decompress": [],
                       "xxh32": [], "frames": [], "kat": [], "dict_compress": []}

    def add(name, data):
        arrays[name] = np.frombuffer(bytes(data), dtype=np.uint8)
        return name

    inputs = []
    kinds = ["text", "source", "records", "markup", "random", "runs"]
    for k in kinds:
        b = _synth.blocks(2, k, seed=31)
        full = k in ("text", "records", "random", "runs")   # full 64 KiB blocks exercise the whole table
        inputs.append((f"{k}_64k" if full else f"{k}_16k", b[0].tobytes() if full else b[0].tobytes()[:16384]))
        inputs.append((f"{k}_ragged", b[1].tobytes()[: rng.randrange(1, 12000)]))
    with open(REF_DATA, "rb") as f:
        inputs.append(("numpy_byte_array", f.read()))
    for s in [0, 1, 4, 5, 11, 12, 13, 14, 15, 16, 17, 19, 31, 32, 63, 64, 65, 255, 256, 65535, 65536, 65546, 65547]:
        src = inputs[0][1] * 2
        inputs.append((f"text_len{s}", src[:s]))
    inputs.append(("zeros_64k", bytes(65536)))
    inputs.append(("ab_64k", b"ab" * 32768))
    inputs.append(("text_300k", _synth.blocks(5, "text", seed=9)[:, :61440].tobytes()))

    for name, data in inputs:
        key = add("in_" + name, data)
        man["inputs"].append({"name": name, "key": key, "len": len(data)})
        d = ref.compress_default(data)
        man["compress"].append({"input": name, "mode": "default", "accel": 1, "key": add(f"cd_{name}", d)})
        b = ref.compress_block_api(data, 1)
        man["compress"].append({"input": name, "mode": "block_api", "accel": 1, "key": add(f"cb_{name}", b)})
        if len(data) >= 4096:
            for acc in (2, 9):
                b = ref.compress_block_api(data, acc)
                man["compress"].append({"input": name, "mode": "block_api", "accel": acc,
                                        "key": add(f"cb{acc}_{name}", b)})
        for seed in (0, 1, 0x9E3779B1):
            man["xxh32"].append({"input": name, "seed": seed, "value": ref.xxh32(data, seed)})
        # decompress: valid at exact / larger / smaller capacity
        for cap in sorted({len(data), len(data) + 7, max(0, len(data) - 1)}):
            st, _ = ref.decompress(d, cap)
            man["decompress"].append({"key": f"cd_{name}", "cap": cap, "status": st})

    # malformed blocks (mutations / truncations) with the reference status
    base = [x for x in inputs if 64 <= len(x[1]) <= 65536]
    for i in range(400):
        name, full = base[rng.randrange(len(base))]
        n = rng.choice([20, 64, 100, 300, 1000, 3000])
        o = rng.randrange(0, max(1, len(full) - n))
        data = full[o:o + n]
        c = bytearray(ref.compress_default(data))
        for _ in range(rng.randrange(1, 4)):
            c[rng.randrange(len(c))] = rng.randrange(256)
        if rng.random() < 0.3:
            c = c[: rng.randrange(len(c) + 1)]
        cap = rng.choice([len(data), len(data) + 1, max(0, len(data) - 3), 100])
        st, _ = ref.decompress(bytes(c), cap)
        key = add(f"bad_{i}", c)
        man["decompress"].append({"key": key, "cap": cap, "status": st, "expected_from": name})

    # known-answer vectors of the reference tests (test_block_1.py:128-149)
    kat = [
        (b"\x00\x00\x00\x00\x00", b""),
        (b"\x01\x00\x00\x00\x10 ", b" "),
        (b"h\x00\x00\x00\xff\x0bLorem ipsum dolor sit amet\x1a\x006P amet", b"Lorem ipsum dolor sit amet" * 4),
        (b"\xb0\xb3\x00\x00\xff\x1fExcepteur sint occaecat cupidatat non proident.\x00" + b"\xff" * 180
         + b"\x1ePident", b"Excepteur sint occaecat cupidatat non proident" * 1000),
    ]
    for i, (comp, plain) in enumerate(kat):
        st, out = ref.decompress(comp[4:], int.from_bytes(comp[:4], "little"))
        assert out == plain, i
        man["kat"].append({"key": add(f"kat_{i}", comp), "status": st, "plain": add(f"katp_{i}", out)})

    # frames
    fdata = inputs[-1][1]
    for opts in [dict(block_size_id=7, linked=False, content_checksum=True),
                 dict(block_size_id=4, linked=False, content_checksum=True, block_checksum=True),
                 dict(block_size_id=4, linked=True, content_checksum=False),
                 dict(block_size_id=5, linked=True, content_checksum=True, store_size=False),
                 dict(block_size_id=4, linked=False, level=-3)]:
        fr = ref.compress_frame(fdata, **opts)
        man["frames"].append({"input": "text_300k", "opts": opts, "key": add(f"fr_{len(man['frames'])}", fr)})

    # more linked frames: ~513 KiB of mixed data, several block sizes / levels
    parts = {k: _synth.blocks(3, k, seed=41).tobytes() for k in ("silesia", "runs", "random", "text")}
    mixed = (parts["silesia"][:196608] + parts["random"][:65536] + parts["runs"][:65536]
             + parts["text"][:196608] + parts["random"][65536:65536 + 1000])   # a raw block mid-stream
    add("in_mixed_1m", mixed)
    man["inputs"].append({"name": "mixed_1m", "key": "in_mixed_1m", "len": len(mixed)})
    for opts in [dict(block_size_id=4, linked=True, content_checksum=True),
                 dict(block_size_id=4, linked=True, content_checksum=False, block_checksum=True, level=-2),
                 dict(block_size_id=5, linked=True, content_checksum=True)]:
        fr = ref.compress_frame(mixed, **opts)
        man["frames"].append({"input": "mixed_1m", "opts": opts, "key": add(f"fr_{len(man['frames'])}", fr)})

    # lz4.block.compress(dict=)
    dsrc = _synth.blocks(4, "text", seed=77).tobytes() + _synth.blocks(2, "records", seed=78).tobytes()
    dcases = [("text_64k", 0, 1), ("text_64k", 5, 1), ("text_64k", 8, 1), ("text_64k", 100, 1),
              ("text_64k", 20000, 1), ("text_64k", 65536, 1), ("text_64k", 100000, 1), ("text_64k", 20000, 3),
              ("records_ragged", 30000, 1), ("numpy_byte_array", 4096, 1), ("text_len13", 50, 1),
              ("text_len0", 1000, 1), ("text_300k", 65536, 2), ("zeros_64k", 300, 1)]
    for i, (name, dl, acc) in enumerate(dcases):
        data = dict(inputs)[name]
        dd = dsrc[len(dsrc) - dl:] if dl else b""
        c = ref.compress_dict(data, dd, acc)
        man["dict_compress"].append({"input": name, "dict": add(f"dict_{i}", dd), "accel": acc,
                                     "key": add(f"cdict_{i}", c)})

    # lz4.block.compress(source, dict=D) with D's memory ending where the
    # source begins (slices of one buffer): prefix mode (lz4.c:1671-1676)
    man["dict_prefix_compress"] = []
    blob = _synth.blocks(3, "silesia", seed=79).tobytes()
    pcases = [(65536, 8, 4000, 1), (65536, 65536, 65536, 1), (1000, 9, 13, 1), (100, 100, 5, 1)]
    prng = random.Random(1671)
    while len(pcases) < 16:   # plus cases whose prefix-mode bytes differ from extDict's
        cut = prng.randrange(8, len(blob) - 70000)
        dl = min(prng.choice([8, 12, 50, 300, 5000, 65536, 70000]), cut)
        n, acc = prng.choice([700, 4000, 12000, 65536]), prng.choice([1, 1, 2, 8])
        dd, data = blob[cut - dl:cut], blob[cut:cut + n]
        if ref.compress_dict_prefix(data, dd, acc) != ref.compress_dict(data, dd, acc):
            pcases.append((cut, dl, n, acc))
    for i, (cut, dl, n, acc) in enumerate(pcases):
        dd, data = blob[cut - dl:cut], blob[cut:cut + n]
        c = ref.compress_dict_prefix(data, dd, acc)
        man["dict_prefix_compress"].append({"input": add(f"pdict_src_{i}", data), "dict": add(f"pdict_{i}", dd),
                                            "accel": acc, "key": add(f"cpdict_{i}", c),
                                            "extdict_differs": c != ref.compress_dict(data, dd, acc)})

    np.savez_compressed(os.path.join(HERE, "golden.npz"), **arrays)
    with open(os.path.join(HERE, "manifest.json"), "w") as f:
        json.dump(man, f, indent=0)
    print("golden:", len(arrays), "arrays,", os.path.getsize(os.path.join(HERE, "golden.npz")), "bytes")


if __name__ == "__main__":
    main()
