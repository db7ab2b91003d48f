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
