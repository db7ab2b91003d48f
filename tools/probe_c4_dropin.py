"""Dev probe: the drop-in config-4 calls on host bytes -- lz4.frame.compress
(4 MiB independent blocks, content checksum, exact parse) and
lz4.frame.decompress of its result (pipelined, and LZ4M_FRAME_PIPELINE=0) -- with a stage split.  env: GIB (8)."""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "python-lz4_amd"))
sys.path.insert(0, ROOT)
import bench as B  # noqa: E402
import lz4.frame as F  # noqa: E402
from lz4 import _native as N  # noqa: E402

dev = torch.device("cuda", 0)
L = int(os.environ.get("GIB", "8")) << 30
src = B.make_batch(L // 65536, 4096, "silesia", 77, dev)
t0 = time.perf_counter()
hb = src.cpu().numpy().tobytes()
print(f"host bytes ready ({time.perf_counter() - t0:.2f}s)", flush=True)
kw = dict(block_size=F.BLOCKSIZE_MAX4MB, block_linked=False, content_checksum=True)
F.decompress(F.compress(hb[: 64 << 20], **kw))
from lz4.frame._frame import _compress_frame  # noqa: E402
for rep in range(2):   # the device part alone: exact parse of 4 MiB independent blocks, no content checksum
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    fx, _ = _compress_frame(src.view(-1), L, content_checksum=False, block_size=7, block_linked=False, parse="exact")
    torch.cuda.synchronize()
    print(f"device exact frame compress (no content checksum): {L / (time.perf_counter() - t0) / 2**30:.2f} GiB/s",
          flush=True)
    del fx
for rep in range(2):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    d = N.to_device(hb, dev, pad=1)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    fr = F.compress(hb, **kw)
    t2 = time.perf_counter()
    out = F.decompress(fr)
    t3 = time.perf_counter()
    ok = out == hb
    t4 = time.perf_counter()
    del out
    os.environ["LZ4M_FRAME_PIPELINE"] = "0"
    t5 = time.perf_counter()
    out0 = F.decompress(fr)
    t6 = time.perf_counter()
    os.environ["LZ4M_FRAME_PIPELINE"] = "1"
    print(f"  sequential decompress (LZ4M_FRAME_PIPELINE=0) {L / (t6 - t5) / 2**30:.2f} GiB/s, ok={out0 == hb}",
          flush=True)
    out = out0
    del d
    print(f"rep {rep}: to_device {L / (t1 - t0) / 2**30:.2f} GiB/s; compress {L / (t2 - t1) / 2**30:.2f} GiB/s "
          f"({t2 - t1:.2f}s, ratio {L / len(fr):.3f}); decompress {L / (t3 - t2) / 2**30:.2f} GiB/s ({t3 - t2:.2f}s); "
          f"ok={ok} (compare {t4 - t3:.2f}s)", flush=True)
    ts = time.perf_counter()
    x = N.to_host_bytes(src, L, hash_seed=0)
    te = time.perf_counter()
    print(f"  to_host_bytes+hash {L / (te - ts) / 2**30:.2f} GiB/s; hash ok={x[1] == N.xxh32_host(hb)}", flush=True)
    del out, fr, x
