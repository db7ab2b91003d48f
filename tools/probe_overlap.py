"""Dev probe: does the content-checksum copy/hash pipeline overlap the frame
compression?  Times compress alone, hash alone and both, and logs when each
64 MiB chunk reaches the host during the combined run."""
import os
import sys
import threading
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "python-lz4_amd"))
sys.path.insert(0, ROOT)
from lz4 import _native as N  # noqa: E402
from lz4.frame._frame import _compress_frame  # noqa: E402
import bench as B  # noqa: E402

dev = torch.device("cuda", 0)
GI = int(os.environ.get("GIB", 4))
L = GI << 30
src = B.make_batch(L // 65536, 4096, "silesia", 77, dev)
kw = dict(block_size=7, block_linked=False, parse="parallel")
for _ in range(2):
    _compress_frame(src, L, content_checksum=False, **kw)
torch.cuda.synchronize()


def timed(fn):
    torch.cuda.synchronize()
    t = time.perf_counter()
    fn()
    torch.cuda.synchronize()
    return time.perf_counter() - t


tc = timed(lambda: _compress_frame(src, L, content_checksum=False, **kw))
th = timed(lambda: N.xxh32_of_device(src, L))
tb = timed(lambda: _compress_frame(src, L, content_checksum=True, **kw))
print(f"compress {tc:.3f} s, hash {th:.3f} s, both {tb:.3f} s (sum {tc + th:.3f})", flush=True)

# chunk arrival times while a compression runs
marks = []
orig = N.HostXXH32.update_ptr


def upd(self, ptr, n):
    marks.append(time.perf_counter())
    return orig(self, ptr, n)


N.HostXXH32.update_ptr = upd
torch.cuda.synchronize()
t0 = time.perf_counter()
ready = torch.cuda.Event()
ready.record()
box = {}
th_ = threading.Thread(target=lambda: box.__setitem__("h", N.xxh32_of_device(src, L, wait_event=ready)))
th_.start()
_compress_frame(src, L, content_checksum=False, **kw)
ev = torch.cuda.Event()
ev.record()
ev.synchronize()
tcomp = time.perf_counter() - t0
th_.join()
tall = time.perf_counter() - t0
rel = [m - t0 for m in marks]
before = sum(1 for r in rel if r < tcomp)
print(f"compress done at {tcomp:.3f} s, hash done at {tall:.3f} s; {before}/{len(rel)} chunks hashed "
      f"before the compression ended; first chunk at {rel[0]:.3f} s", flush=True)
print("chunk times:", " ".join(f"{r:.2f}" for r in rel[:: max(1, len(rel) // 16)]), flush=True)
