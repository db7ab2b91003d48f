"""Dev probe: lz4.block.decompress_host end to end (pinned host bytes -> H2D ->
decode -> D2H) on NB x 64 KiB silesia-like blocks, per chunk size, with the
copies queued as their waits complete (default) or all up front
(LZ4M_HOST_QUEUED=1)."""
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
src = B.make_batch(n, 4096, "silesia", 2026, dev)
so, sl, slots, soff, scap, olen = B.compress_all(src, n, 0, dev)
N.launch_compress(src, so, sl, slots, soff, scap, olen, n, N.TABLE_U16_HASH4, 1)
offs = N.exclusive_scan(olen)
tot = int(offs[n])
comp = torch.empty(tot, dtype=torch.uint8, device=dev)
N.gather(slots, soff, olen, comp, offs, n)
del slots
h_comp = torch.empty(tot, dtype=torch.uint8, pin_memory=True)
h_comp.copy_(comp)
h_out = torch.empty(n * 65536, dtype=torch.uint8, pin_memory=True)
h_coff, h_clen = offs[:n].cpu(), olen.cpu()
h_ooff = torch.arange(n, dtype=torch.int64) * 65536
h_ocap = torch.full((n,), 65536, dtype=torch.int32)
for mode in ("0", "1"):
    os.environ["LZ4M_HOST_QUEUED"] = mode
    for cb in (65536, 32768, 16384):
        best = 1e9
        for rep in range(3):
            torch.cuda.synchronize()
            t = time.perf_counter()
            st = LB.decompress_host(h_comp, h_coff, h_clen, h_out, h_ooff, h_ocap, chunk_blocks=cb)
            torch.cuda.synchronize()
            best = min(best, time.perf_counter() - t)
        ok = bool((st == 65536).all()) and torch.equal(h_out[-65536:], src[-65536:].cpu())
        print(f"queued={mode} chunk={cb}: {n * 65536 / best / 2**30:.2f} GiB/s ({best * 1e3:.1f} ms) ok={ok}", flush=True)
