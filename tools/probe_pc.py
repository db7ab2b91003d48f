"""Dev probe: parallel-parse compressor throughput and ratio (vs the exact
LZ4_compress_default parse) on NB silesia-like blocks; every block is
decoded back by the GPU decoder.  Optional A/B: LZ4M_LIB=<other build>."""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "python-lz4_amd"))
sys.path.insert(0, ROOT)
from lz4 import _native as N  # noqa: E402
import bench as B  # noqa: E402

dev = torch.device("cuda", 0)
n = int(os.environ.get("NB", 1 << 18))
kinds = os.environ.get("KINDS", "silesia").split(",")
for kind in kinds:
    src = B.make_batch(n, min(4096, n), kind, 2026, dev)
    so, sl, slots, soff, scap, olen = B.compress_all(src, n, 0, dev)
    N.launch_compress(src, so, sl, slots, soff, scap, olen, n, N.TABLE_U16_HASH4, 1)
    exact = int(olen.to(torch.int64).sum())
    ts = []
    for _ in range(3):
        torch.cuda.synchronize()
        t = time.perf_counter()
        N.launch_compress(src, so, sl, slots, soff, scap, olen, n, N.PARSE_PARALLEL, 1)
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t)
    par = int(olen.to(torch.int64).sum())
    import hashlib
    sizes_digest = hashlib.sha1(olen.cpu().numpy().tobytes()).hexdigest()[:12]
    dst = torch.empty(n * 65536, dtype=torch.uint8, device=dev)
    st = torch.empty(n, dtype=torch.int32, device=dev)
    N.launch_decompress(slots, soff, olen, dst, so, sl, st, n)
    ok = bool((st == 65536).all()) and torch.equal(dst, src)
    print(f"{kind}: parallel {n * 65536 / min(ts) / 2**30:.2f} GiB/s, ratio {n * 65536 / par:.4f} "
          f"(exact {n * 65536 / exact:.4f}, {par / exact - 1:+.2%} size), round trip {'ok' if ok else 'FAILED'}, "
          f"sizes {sizes_digest}",
          flush=True)
    del src, slots, dst
    torch.cuda.empty_cache()
