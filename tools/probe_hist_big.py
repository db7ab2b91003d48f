"""Dev probe: hist_decompress_kernel on large blocks (config 4's 4 MiB) --
decode time of NB blocks of BS bytes per launch, verified; A/B via LZ4M_LIB.
env: BS (4194304), NBS (32,2048), KINDS (silesia), REPS (3)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "python-lz4_amd"))
sys.path.insert(0, ROOT)
import bench as B  # noqa: E402
from lz4 import _native as N  # noqa: E402

dev = torch.device("cuda", 0)
bs = int(os.environ.get("BS", 4 << 20))
reps = int(os.environ.get("REPS", 3))
for kind in os.environ.get("KINDS", "silesia").split(","):
    for nb in [int(x) for x in os.environ.get("NBS", "32,2048").split(",")]:
        src = B.make_batch(nb * bs // 65536, min(4096, nb * bs // 65536), kind, 77, dev)
        so = torch.arange(nb, dtype=torch.int64, device=dev) * bs
        sl = torch.full((nb,), bs, dtype=torch.int32, device=dev)
        cap = N.compress_bound(bs)
        soff = torch.arange(nb, dtype=torch.int64, device=dev) * cap
        scap = torch.full((nb,), cap, dtype=torch.int32, device=dev)
        slots = torch.empty(nb * cap + 16, dtype=torch.uint8, device=dev)
        olen = torch.empty(nb, dtype=torch.int32, device=dev)
        N.launch_compress(src, so, sl, slots, soff, scap, olen, nb, N.TABLE_AUTO, 1)
        dst = torch.empty(nb * bs, dtype=torch.uint8, device=dev)
        st = torch.empty(nb, dtype=torch.int32, device=dev)
        ts = []
        for _ in range(reps + 1):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            N.launch_decompress(slots, soff, olen, dst, so, sl, st, nb, decoder="hist")
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        ok = bool((st == bs).all()) and torch.equal(dst, src)
        ms = min(ts[1:])
        print(f"{kind} {nb} x {bs >> 10} KiB: {ms:.2f} ms {nb * bs / ms / 1e6:.1f} GB/s ok={ok}", flush=True)
        del src, slots, dst
        torch.cuda.empty_cache()
