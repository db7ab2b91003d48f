"""Dev probe: host<->device transfer rates for decompress_host's copies --
copy engine (one stream / four streams) vs a gather kernel reading or
writing pinned host memory directly (UVA)."""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "python-lz4_amd"))
from lz4 import _native as N  # noqa: E402

GiB = 1 << 30
nb = 65536
BLK = 65536
size = nb * BLK
dev = torch.device("cuda", 0)
h = torch.empty(size, dtype=torch.uint8, pin_memory=True)
h.fill_(3)
d = torch.empty(size, dtype=torch.uint8, device=dev)
offs = torch.arange(nb, dtype=torch.int64, device=dev) * BLK
lens = torch.full((nb,), BLK, dtype=torch.int32, device=dev)


def t(fn, reps=3):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return size * reps / (time.perf_counter() - t0) / 1e9


streams = [torch.cuda.Stream() for _ in range(4)]


def multi(dst, src):
    cur = torch.cuda.current_stream()
    q = size // 4
    for i, s in enumerate(streams):
        s.wait_stream(cur)
        with torch.cuda.stream(s):
            dst[i * q:(i + 1) * q].copy_(src[i * q:(i + 1) * q], non_blocking=True)
    for s in streams:
        cur.wait_stream(s)


class HostView:   # a uint8 "tensor" whose data_ptr is the pinned host buffer
    def __init__(self, t):
        self.t = t

    def data_ptr(self):
        return self.t.data_ptr()


print(f"H2D copy_ 1 stream : {t(lambda: d.copy_(h, non_blocking=True)):.1f} GB/s", flush=True)
print(f"D2H copy_ 1 stream : {t(lambda: h.copy_(d, non_blocking=True)):.1f} GB/s", flush=True)
print(f"H2D copy_ 4 streams: {t(lambda: multi(d, h)):.1f} GB/s", flush=True)
print(f"D2H copy_ 4 streams: {t(lambda: multi(h, d)):.1f} GB/s", flush=True)
print(f"D2H gather kernel  : {t(lambda: N.gather(d, offs, lens, HostView(h), offs, nb)):.1f} GB/s", flush=True)
print(f"H2D gather kernel  : {t(lambda: N.gather(HostView(h), offs, lens, d, offs, nb)):.1f} GB/s", flush=True)
ok = torch.equal(h[:BLK * 4].to(dev), d[:BLK * 4])
print("gather host round trip", "ok" if ok else "MISMATCH")
