"""Dev probe: lz4.block.compress_many / decompress_many on 1 000 x 64 KiB
random blocks (BASELINE config 1), first call and the following calls."""
import os
import random
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "python-lz4_amd"))
import lz4.block as LB  # noqa: E402

rnd = random.Random(12345)
blocks = [rnd.randbytes(65536) for _ in range(1000)]
tot = len(blocks) * 65536
LB.decompress(LB.compress(blocks[0]))
for rep in range(4):
    t0 = time.perf_counter()
    cm = LB.compress_many(blocks)
    t1 = time.perf_counter()
    bm = LB.decompress_many(cm)
    t2 = time.perf_counter()
    assert bm == blocks
    print(f"rep {rep}: compress_many {(t1 - t0) * 1e3:.2f} ms = {tot / (t1 - t0) / 2**30:.2f} GiB/s, "
          f"decompress_many {(t2 - t1) * 1e3:.2f} ms = {tot / (t2 - t1) / 2**30:.2f} GiB/s", flush=True)
