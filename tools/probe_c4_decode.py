"""Dev probe: where config 4's frame decompress with a content checksum
spends its time (lz4.frame.decompress_device on an 8 GiB frame of 4 MiB
independent blocks): each stage of _frame.decompress_device timed with a
device synchronisation around it, and the whole call untimed-instrumented."""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "python-lz4_amd"))
sys.path.insert(0, ROOT)
import bench as B  # noqa: E402
import lz4.frame  # noqa: E402
import lz4.frame._frame as FF  # noqa: E402
from lz4 import _native as N  # noqa: E402

dev = torch.device("cuda", 0)
gib = int(os.environ.get("GIB", "8"))
L = gib << 30
n = L // 65536
src = B.make_batch(n, 4096, "silesia", 2026, dev).view(-1)[:L]
frame = lz4.frame.compress_device(src, L, block_size=7, content_checksum=True, block_linked=False, parse="parallel")
torch.cuda.synchronize()
print(f"frame {frame.numel() / 2**30:.2f} GiB", flush=True)

acc = {}


def wrap(mod, name):
    f = getattr(mod, name)

    def g(*a, **k):
        torch.cuda.synchronize()
        t = time.perf_counter()
        r = f(*a, **k)
        torch.cuda.synchronize()
        acc[name] = acc.get(name, 0.0) + time.perf_counter() - t
        return r
    setattr(mod, name, g)


for rep in range(3):
    torch.cuda.synchronize()
    t = time.perf_counter()
    out = lz4.frame.decompress_device(frame)
    torch.cuda.synchronize()
    print(f"plain: {(time.perf_counter() - t) * 1e3:.1f} ms ({L / (time.perf_counter() - t) / 2**30:.2f} GiB/s)",
          flush=True)
assert out.numel() == L
for name in ("frame_scan",):
    wrap(N, name)
for name in ("_decode_records", "_xxh32_dev", "_frame_errors", "_le32_at"):
    wrap(FF, name)
acc.clear()
torch.cuda.synchronize()
t = time.perf_counter()
out = lz4.frame.decompress_device(frame)
torch.cuda.synchronize()
tot = time.perf_counter() - t
print(f"instrumented: {tot * 1e3:.1f} ms; " + ", ".join(f"{k} {v * 1e3:.1f} ms" for k, v in acc.items())
      + f"; rest {(tot - sum(acc.values())) * 1e3:.1f} ms", flush=True)
h = torch.empty(1, dtype=torch.int32, device=dev)
t = time.perf_counter()
N.xxh32_of_device(out, L)
print(f"xxh32_of_device alone: {(time.perf_counter() - t) * 1e3:.1f} ms", flush=True)
