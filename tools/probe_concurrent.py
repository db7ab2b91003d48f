"""Dev probe: can a plain copy run beside the row decoder for free?  Times
config 2's decode alone, an 11 GB device copy alone (the size of the
incompressible blocks' literals in the mix) and both launched together on two
streams.  env: NBLK (1048576), COPY_GB (5.5: bytes read = bytes written)."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "python-lz4_amd"))
sys.path.insert(0, ROOT)
import bench as B  # noqa: E402
from lz4 import _native as N  # noqa: E402

dev = torch.device("cuda", 0)
n = int(os.environ.get("NBLK", 1 << 20))
src = B.make_batch(n, 4096, "silesia", 2026, dev)
so, sl, slots, soff, scap, olen = B.compress_all(src, n, 0, dev)
N.launch_compress(src, so, sl, slots, soff, scap, olen, n, N.TABLE_U16_HASH4, 1)
offs = N.exclusive_scan(olen)
tot = int(offs[n])
comp = torch.empty(tot, dtype=torch.uint8, device=dev)
N.gather(slots, soff, olen, comp, offs, n)
coff = offs[:n].clone()
del slots, soff, scap, so, sl
torch.cuda.empty_cache()
dst = torch.empty(n * 65536, dtype=torch.uint8, device=dev)
doff = torch.arange(n, dtype=torch.int64, device=dev) * 65536
dcap = torch.full((n,), 65536, dtype=torch.int32, device=dev)
st = torch.empty(n, dtype=torch.int32, device=dev)
cb = int(float(os.environ.get("COPY_GB", 5.5)) * 1e9)
ca = torch.empty(cb, dtype=torch.uint8, device=dev)
cc = torch.empty(cb, dtype=torch.uint8, device=dev)
side = torch.cuda.Stream(dev)


def dec():
    N.launch_decompress(comp, coff, olen, dst, doff, dcap, st, n)


def cpy():
    with torch.cuda.stream(side):
        cc.copy_(ca)


def timed(fn, reps=3):
    ts = []
    for _ in range(reps + 1):
        torch.cuda.synchronize()
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        torch.cuda.current_stream().wait_stream(side)
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
    return sorted(ts[1:])


res = {"decode": timed(dec), "copy": timed(cpy)}
res["both"] = timed(lambda: (cpy(), dec()))


def cpy_late():
    # the copy after ~25 ms (past the parse kernel): beside the row execution
    with torch.cuda.stream(side):
        torch.cuda._sleep(int(os.environ.get("SLEEP_CYCLES", 60_000_000)))
        cc.copy_(ca)


def sleep_only():
    with torch.cuda.stream(side):
        torch.cuda._sleep(int(os.environ.get("SLEEP_CYCLES", 60_000_000)))


res["sleep"] = timed(sleep_only)
res["decode_beside_sleep"] = timed(lambda: (sleep_only(), dec()))
res["both_late"] = timed(lambda: (cpy_late(), dec()))
ok = bool((st == 65536).all()) and torch.equal(dst, src)
res["ok"] = ok
print(json.dumps(res))
