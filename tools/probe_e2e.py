"""Dev probe: lz4.block.decompress_host (host -> H2D -> decode -> D2H)
rates by chunk size on NB silesia-like blocks."""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "python-lz4_amd"))
sys.path.insert(0, ROOT)
import bench as B  # noqa: E402
import lz4.block as LB  # noqa: E402
from lz4 import _native as N  # noqa: E402

dev = torch.device("cuda", 0)
n = int(os.environ.get("NB", 1 << 18))
src = B.make_batch(n, min(4096, n), "silesia", 2026, dev)
so, sl, slots, soff, scap, olen = B.compress_all(src, n, 0, dev)
N.launch_compress(src, so, sl, slots, soff, scap, olen, n, N.TABLE_U16_HASH4, 1)
coff = torch.cumsum(olen.to(torch.int64), 0) - olen.to(torch.int64)
tot = int(olen.to(torch.int64).sum())
packed = torch.empty(tot, dtype=torch.uint8, device=dev)
N.gather(slots, soff, olen, packed, coff, n)
h_comp = torch.empty(tot, dtype=torch.uint8, pin_memory=True)
h_comp.copy_(packed)
h_out = torch.empty(n * 65536, dtype=torch.uint8, pin_memory=True)
h_coff, h_clen = coff.cpu(), olen.cpu()
h_ooff = torch.arange(n, dtype=torch.int64) * 65536
h_ocap = torch.full((n,), 65536, dtype=torch.int32)
del slots, packed
for how in ["engine"]:
    for cb in [int(x) for x in os.environ.get("CHUNKS", "32768,65536,131072").split(",")]:
        LB.decompress_host(h_comp, h_coff, h_clen, h_out, h_ooff, h_ocap, chunk_blocks=cb)
        ts = []
        for _ in range(2):
            h_out.zero_()
            t = time.perf_counter()
            st = LB.decompress_host(h_comp, h_coff, h_clen, h_out, h_ooff, h_ocap, chunk_blocks=cb)
            ts.append(time.perf_counter() - t)
        ok = bool((st == 65536).all()) and torch.equal(h_out[-65536 * 8:].to(dev), src[-65536 * 8:]) \
            and torch.equal(h_out[:65536 * 8].to(dev), src[:65536 * 8])
        print(f"{how:6s} chunk {cb:6d}: {n * 65536 / min(ts) / 2**30:.2f} GiB/s  {'ok' if ok else 'FAILED'}",
              flush=True)
