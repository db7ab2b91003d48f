"""Dev probe: config 4's device-resident frame decode without a content
checksum (8 GiB, 4 MiB independent blocks), three warm calls."""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "python-lz4_amd"))
sys.path.insert(0, ROOT)
import bench as B  # noqa: E402
import lz4.frame  # noqa: E402

dev = torch.device("cuda", 0)
L = int(os.environ.get("GIB", "8")) << 30
src = B.make_batch(L // 65536, 4096, "silesia", 77, dev).view(-1)[:L]
frame = lz4.frame.compress_device(src, L, block_size=7, content_checksum=False, block_linked=False, parse="parallel")
for rep in range(4):
    torch.cuda.synchronize()
    t = time.perf_counter()
    out = lz4.frame.decompress_device(frame)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t
    ok = torch.equal(out, src)
    del out
    print(f"rep {rep}: {dt * 1e3:.1f} ms = {L / dt / 2**30:.2f} GiB/s ok={ok}", flush=True)
