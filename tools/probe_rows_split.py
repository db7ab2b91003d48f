"""Dev probe: the config-2 batch (NBLK x 64 KiB, row decoder) decoded as one
launch against SPLIT launches of equal block ranges on as many streams (each
its own scratch), joined on the current stream: does one half's parse run
under the other half's execution?  Wall time per call (host clock around a
synchronize), output verified."""
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
n = int(os.environ.get("NBLK", 1 << 20))
src = B.make_batch(n, min(4096, n), "silesia", 7, dev)
so, sl, slots, soff, scap, olen = B.compress_all(src, n, 0, dev)
N.launch_compress(src, so, sl, slots, soff, scap, olen, n, N.TABLE_U16_HASH4, 1)
offs = N.exclusive_scan(olen)
tot = int(offs[n])
comp = torch.empty(tot, dtype=torch.uint8, device=dev)
N.gather(slots, soff, olen, comp, offs, n)
coff = offs[:n].clone()
del slots
torch.cuda.empty_cache()
dst = torch.empty(n * 65536, dtype=torch.uint8, device=dev)
doff = torch.arange(n, dtype=torch.int64, device=dev) * 65536
dcap = torch.full((n,), 65536, dtype=torch.int32, device=dev)
st = torch.empty(n, dtype=torch.int32, device=dev)
cur = torch.cuda.current_stream(dev)
streams = [torch.cuda.Stream(dev) for _ in range(4)]


def run(parts, offset_ms=0):
    if parts == 1:
        N.launch_decompress(comp, coff, olen, dst, doff, dcap, st, n, src_bytes=tot)
        return
    b = [n * k // parts for k in range(parts + 1)]
    for k in range(parts):
        s = streams[k]
        s.wait_stream(cur)
        lo, hi = b[k], b[k + 1]
        nbytes = int(offs[hi]) - int(offs[lo]) if False else tot
        N.launch_decompress(comp, coff[lo:hi], olen[lo:hi], dst, doff[lo:hi], dcap[lo:hi], st[lo:hi], hi - lo,
                            stream=s, src_bytes=tot)
    for k in range(parts):
        cur.wait_stream(streams[k])


for parts in [int(x) for x in os.environ.get("PARTS", "1,2,4,1,2").split(",")]:
    dst.zero_()
    run(parts)
    torch.cuda.synchronize()
    ok = bool((st == 65536).all()) and torch.equal(dst, src)
    ts = []
    for _ in range(4):
        torch.cuda.synchronize()
        t = time.perf_counter()
        run(parts)
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t) * 1e3)
    ms = min(ts)
    print(f"parts={parts}: {ms:.1f} ms (all {[round(x, 1) for x in ts]}) {n * 65536 / ms / 1e-3 / 2**30:.1f} GiB/s ok={ok}",
          flush=True)
