"""Dev probe: config 4's device frame compress without a content checksum
(8 GiB, 4 MiB independent blocks, parallel parse): the whole call against
its compression launch alone, and the compressed size (LZ4M_PC_SEG A/B; the LZ4M_PC_LARGE / LZ4M_PC_SEGHB knobs left the sources in round 6)."""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "python-lz4_amd"))
sys.path.insert(0, ROOT)
import bench as B  # noqa: E402
from lz4 import _native as N  # noqa: E402
from lz4.frame._frame import _compress_frame  # noqa: E402

dev = torch.device("cuda", 0)
L = int(os.environ.get("GIB", "8")) << 30
FB = 4 << 20
src = B.make_batch(L // 65536, 4096, "silesia", 77, dev).view(-1)[:L]
nb = L // FB
for rep in range(3):
    torch.cuda.synchronize()
    t = time.perf_counter()
    fr, _ = _compress_frame(src, L, content_checksum=False, block_size=7, block_linked=False, parse="parallel")
    torch.cuda.synchronize()
    dt = time.perf_counter() - t
    print(f"whole call: {dt * 1e3:.1f} ms = {L / dt / 2**30:.2f} GiB/s", flush=True)
    del fr
raw_off = torch.arange(nb, dtype=torch.int64, device=dev) * FB
raw_len = torch.full((nb,), FB, dtype=torch.int32, device=dev)
slot = N.compress_bound(FB)
cmp = torch.empty(nb * slot, dtype=torch.uint8, device=dev)
cmp_off = torch.arange(nb, dtype=torch.int64, device=dev) * slot
cmp_len = torch.empty(nb, dtype=torch.int32, device=dev)
for rep in range(2):
    torch.cuda.synchronize()
    t = time.perf_counter()
    N.launch_compress(src, raw_off, raw_len, cmp, cmp_off, raw_len - 1, cmp_len, nb, N.PARSE_PARALLEL_LARGE, 1,
                      max_len=FB)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t
    print(f"compression launch alone: {dt * 1e3:.1f} ms", flush=True)
tot = int(cmp_len.to(torch.int64).sum())
tag = " ".join(f"{k}={os.environ[k]}" for k in ("LZ4M_PC_LARGE", "LZ4M_PC_SEG", "LZ4M_PC_SEGHB") if k in os.environ)
print(f"[{tag or 'default'}] {tot} bytes, ratio {L / tot:.4f}", flush=True)
