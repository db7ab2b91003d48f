"""Dev probe: per-call lz4.block.compress / decompress latency on config 1's
data (random 64 KiB blocks), warm."""
import os
import random
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "python-lz4_amd"))
import lz4.block as B  # noqa: E402

rng = random.Random(12345)
blocks = [rng.randbytes(65536) for _ in range(int(os.environ.get("N", "200")))]
comp = [B.compress(b) for b in blocks]
for rep in range(2):
    t = time.perf_counter()
    comp = [B.compress(b) for b in blocks]
    tc = (time.perf_counter() - t) / len(blocks)
    t = time.perf_counter()
    back = [B.decompress(c) for c in comp]
    td = (time.perf_counter() - t) / len(blocks)
assert back == blocks
print(f"per call: compress {tc * 1e6:.1f} us, decompress {td * 1e6:.1f} us")

# fixed per-call cost: the same entry points on (almost) no work -- a 1-byte
# empty block (cap 0) and a 64 KiB run of zeros (one long match: 64 KiB back
# over PCIe, little kernel work); compress of 16 zero bytes
import ctypes as C  # noqa: E402
import lz4._native as N  # noqa: E402
lib = N.lib()
z = bytes(65536)
cz = B.compress(z, store_size=False)
out = C.create_string_buffer(65536 + 64)
cases = {"decompress empty (cap 0)": lambda: lib.lz4m_decompress_safe(b"\x00", out, 1, 0),
         "decompress 64 KiB zeros": lambda: lib.lz4m_decompress_safe(cz, out, len(cz), 65536),
         "compress 16 zero bytes": lambda: lib.lz4m_compress_default(bytes(16), out, 16, 64)}
for name, f in cases.items():
    for _ in range(20):
        f()
    t = time.perf_counter()
    for _ in range(500):
        f()
    print(f"{name}: {(time.perf_counter() - t) / 500 * 1e6:.1f} us per call")

# the same calls on compressible data (silesia-like mix, lz4/_synth.py)
if os.environ.get("C1_SYNTH", "1") == "1":
    import numpy as np  # noqa: E402
    from lz4 import _synth  # noqa: E402
    for kind in ("silesia", "text", "records"):
        sb = [bytes(x) for x in _synth.blocks(64, kind, seed=5)]
        sc = [B.compress(b) for b in sb]
        for rep in range(2):
            t = time.perf_counter()
            sc = [B.compress(b) for b in sb]
            tc = (time.perf_counter() - t) / len(sb)
            t = time.perf_counter()
            back = [B.decompress(c) for c in sc]
            td = (time.perf_counter() - t) / len(sb)
        assert back == sb
        ratio = sum(map(len, sb)) / sum(map(len, sc))
        print(f"{kind} (ratio {ratio:.2f}): per call compress {tc * 1e6:.1f} us, decompress {td * 1e6:.1f} us")
