"""Dev probe: config 4's device-resident frame decode with a content
checksum (8 GiB, 4 MiB independent blocks), the content hash following the
block-ordered decode (default) vs after it (LZ4M_FRAME_FOLLOW=0), and the
host hash rate alone."""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "python-lz4_amd"))
sys.path.insert(0, ROOT)
import bench as B  # noqa: E402
import lz4.frame  # noqa: E402
from lz4 import _native as N  # noqa: E402

dev = torch.device("cuda", 0)
L = int(os.environ.get("GIB", "8")) << 30
src = B.make_batch(L // 65536, 4096, "silesia", 2026, dev).view(-1)[:L]
frame = lz4.frame.compress_device(src, L, block_size=7, content_checksum=True, block_linked=False, parse="parallel")
torch.cuda.synchronize()
print(f"frame {frame.numel() / 2**30:.2f} GiB", flush=True)
t = time.perf_counter()
h = N.xxh32_of_device(src, L)
print(f"host hash of the device bytes alone: {L / (time.perf_counter() - t) / 1e9:.2f} GB/s", flush=True)
for mode in ("1", "0", "1", "0"):
    os.environ["LZ4M_FRAME_FOLLOW"] = mode
    torch.cuda.synchronize()
    t = time.perf_counter()
    out = lz4.frame.decompress_device(frame)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t
    ok = torch.equal(out, src)
    del out
    print(f"follow={mode}: {dt * 1e3:.1f} ms = {L / dt / 2**30:.2f} GiB/s ok={ok}", flush=True)
