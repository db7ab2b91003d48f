"""Dev probe: decode time per decoder (LZ4M decoders via lz4m_decompress_batch_sel)
on NBLK x 64 KiB blocks of each KIND, verified against the input.
env: NBLK (default 262144), KINDS (silesia), DECS (rows,hist), REPS (3), SEED (7; the bench: 2026)."""
import json
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
n = int(os.environ.get("NBLK", 262144))
reps = int(os.environ.get("REPS", 3))
res = {}
for kind in os.environ.get("KINDS", "silesia").split(","):
    src = B.make_batch(n, min(4096, n), kind, int(os.environ.get("SEED", 7)), dev)
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
    for dec in os.environ.get("DECS", "rows,hist").split(","):
        dst.zero_()
        t0 = time.time()
        N.launch_decompress(comp, coff, olen, dst, doff, dcap, st, n, decoder=dec)
        torch.cuda.synchronize()
        first = time.time() - t0
        ok = bool((st == 65536).all()) and torch.equal(dst, src)
        ts = []
        for _ in range(reps):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            N.launch_decompress(comp, coff, olen, dst, doff, dcap, st, n, decoder=dec)
            b.record()
            torch.cuda.synchronize()
            ts.append(a.elapsed_time(b))
        ms = min(ts)
        r = {"ok": ok, "ms": round(ms, 3), "GiB_s": round(n * 65536 / ms / 1e-3 / 2**30, 1),
             "ratio": round(n * 65536 / tot, 3), "first_s": round(first, 2)}
        res[f"{kind}/{dec}"] = r
        print(kind, dec, r, flush=True)
    del src, comp, dst
    torch.cuda.empty_cache()
print(json.dumps(res))
