"""Dev probe: decoder choice for small batches -- the cooperative kernel
(LZ4M_DECODER=coop) vs the lane kernel (LZ4M_DECODER=lane) on one 64 KiB
block, 64 / 2 048 / 16 384 blocks of 64 KiB, and 2 048 blocks of 4 MiB (the
config-4 frame).  Run once per LZ4M_DECODER value."""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "python-lz4_amd"))
sys.path.insert(0, ROOT)
import bench as B  # noqa: E402
from lz4 import _native as N  # noqa: E402

dev = torch.device("cuda", 0)
mode = os.environ.get("LZ4M_DECODER", "auto")


def case(nb, bs):
    per = bs // 65536
    src = B.make_batch(nb * per, min(4096, nb * per), os.environ.get("KIND", "silesia"), 7, dev)
    so = torch.arange(nb, dtype=torch.int64, device=dev) * bs
    sl = torch.full((nb,), bs, dtype=torch.int32, device=dev)
    cap = ((bs + bs // 255 + 16 + 15) // 16) * 16
    soff = torch.arange(nb, dtype=torch.int64, device=dev) * cap
    scap = torch.full((nb,), cap, dtype=torch.int32, device=dev)
    slots = torch.empty(nb * cap, dtype=torch.uint8, device=dev)
    olen = torch.empty(nb, dtype=torch.int32, device=dev)
    table = N.PARSE_PARALLEL_LARGE if bs > 65536 else N.TABLE_U16_HASH4
    N.launch_compress(src, so, sl, slots, soff, scap, olen, nb, table, 1)
    dst = torch.zeros(nb * bs, dtype=torch.uint8, device=dev)
    st = torch.empty(nb, dtype=torch.int32, device=dev)
    N.launch_decompress(slots, soff, olen, dst, so, sl, st, nb)
    torch.cuda.synchronize()
    ok = bool((st == bs).all()) and torch.equal(dst, src)
    ts = []
    for _ in range(3):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(); N.launch_decompress(slots, soff, olen, dst, so, sl, st, nb); b.record(); torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
    t = min(ts)
    print(f"{mode}: {nb} x {bs >> 10} KiB: {t:.3f} ms = {nb * bs / t / 1e6:.2f} GB/s, {'ok' if ok else 'FAILED'}",
          flush=True)


sizes = os.environ.get("SIZES")
todo = [tuple(int(x) for x in t.split("x")) for t in sizes.split(",")] if sizes else \
    [(1, 65536), (64, 65536), (2048, 65536), (16384, 65536), (2048, 4 << 20)]
for nb, bs in todo:
    case(nb, bs)
