"""Dev probe: config-3 parallel-parse compress and config-4 pieces (XXH32
long, 4 MiB-block frame) timings on one GPU."""
import os, sys, time
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "python-lz4_amd")); sys.path.insert(0, ROOT)
from lz4 import _native as N
import lz4.frame
import bench as B

dev = torch.device("cuda", 0)
def tm(fn, reps=3):
    fn(); torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps): fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps

n = int(os.environ.get("NB", 1 << 18))
src = B.make_batch(n, 4096, "silesia", 2026, dev)
so, sl, slots, soff, scap, olen = B.compress_all(src, n, 0, dev)
for name, tab in (("exact", N.TABLE_U16_HASH4), ("parallel", N.PARSE_PARALLEL)):
    t = tm(lambda: N.launch_compress(src, so, sl, slots, soff, scap, olen, n, tab, 1), 1 if tab == 0 else 3)
    tot = int(olen.to(torch.int64).sum())
    print(f"compress {name}: {n*65536/t/2**30:.2f} GiB/s ratio {n*65536/tot:.4f} fails {(olen<=0).sum().item()}", flush=True)
del slots
for gib in (1,):
    L = gib << 30
    buf = src[:L]
    out = torch.empty(1, dtype=torch.int32, device=dev)
    t = tm(lambda: N.launch_xxh32_long(buf, L, 0, out), 2)
    print(f"xxh32_long {gib} GiB: {L/t/1e9:.2f} GB/s", flush=True)
    t = tm(lambda: lz4.frame.compress_device(buf, L, block_size=7, content_checksum=False, block_linked=False, parse="parallel"), 2)
    print(f"frame 4MiB parallel, no content checksum, {gib} GiB: {L/t/2**30:.2f} GiB/s", flush=True)
    t = tm(lambda: lz4.frame.compress_device(buf, L, block_size=7, content_checksum=False, block_linked=False, parse="exact"), 1)
    print(f"frame 4MiB exact, no content checksum, {gib} GiB: {L/t/2**30:.2f} GiB/s", flush=True)
