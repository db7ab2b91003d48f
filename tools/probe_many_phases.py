"""Dev probe: where a compress_many / decompress_many call of 1 000 x 64 KiB
random blocks spends its time (host phases around the GPU work)."""
import os
import random
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "python-lz4_amd"))
import numpy as np  # noqa: E402
import lz4.block as LB  # noqa: E402
from lz4.block import _block as K  # noqa: E402
from lz4 import _native as N  # noqa: E402

rnd = random.Random(12345)
blocks = [rnd.randbytes(65536) for _ in range(1000)]
LB.decompress_many(LB.compress_many(blocks))
for rep in range(4):
    t = [time.perf_counter()]
    views = [K._buffer(b) for b in blocks]
    dev = N.device()
    n = len(views)
    lens = [v.nbytes for v in views]
    caps = [max(N.compress_bound(L), 1) for L in lens]
    d_off = np.concatenate([[0], np.cumsum(caps[:-1], dtype=np.int64)])
    offs = np.concatenate([[0], np.cumsum(lens[:-1], dtype=np.int64)])
    t.append(time.perf_counter())
    lay, h, d = K._stage_in(dev, views, offs, lens, d_off, caps)
    t.append(time.perf_counter())
    d_src, src_off, src_len, d_dst, dst_off, dst_cap, out_len = K._dev_views(lay, d, n)
    N.launch_compress(d_src, src_off, src_len, d_dst, dst_off, dst_cap, out_len, n, N.TABLE_U32_HASH5, 1)
    t.append(time.perf_counter())
    olen, host = K._stage_out(lay, h, d, n)
    t.append(time.perf_counter())
    res = K._results_many(host, d_off, olen, lens, False)
    t.append(time.perf_counter())
    del res
    t.append(time.perf_counter())
    ph = ["prep", "stage_in(pack+h2d enqueue)", "launch", "stage_out(sync d2h)", "results", "free"]
    print(f"rep {rep}: " + ", ".join(f"{p} {1e3 * (b - a):.2f}" for p, a, b in zip(ph, t, t[1:])) +
          f" ms; total {1e3 * (t[-2] - t[0]):.2f}", flush=True)
