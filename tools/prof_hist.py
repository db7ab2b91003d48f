"""Dev probe: per-phase cycle split of hist_decompress_kernel.  Needs the
diagnostic build (tools/prof_hist.sh -> tools/_prof/_lz4m_prof.so, compiled
with -DLZ4M_HIST_PROF) loaded through LZ4M_LIB, and LZ4M_DECODER=hist."""
import ctypes as C
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "python-lz4_amd"))
sys.path.insert(0, ROOT)
import bench as B  # noqa: E402
from lz4 import _native as N  # noqa: E402

dev = torch.device("cuda", 0)
lib = N.lib()
NAMES = ["restage", "walk", "parse+prefix+ok", "literals", "passes", "flush", "long-literal", "exact tail",
         "rounds", "passes#", "seqs#", "blocks#", "", "", "", "block setup"]
for kind in os.environ.get("KINDS", "silesia,text").split(","):
    nb, bs = int(os.environ.get("NB", "32768")), int(os.environ.get("BS", "65536"))   # BS: block size
    src = B.make_batch(nb * bs // 65536, min(4096, nb * bs // 65536), kind, 7, dev)
    so = torch.arange(nb, dtype=torch.int64, device=dev) * bs
    sl = torch.full((nb,), bs, dtype=torch.int32, device=dev)
    cap = ((bs + bs // 255 + 16 + 15) // 16) * 16
    soff = torch.arange(nb, dtype=torch.int64, device=dev) * cap
    scap = torch.full((nb,), cap, dtype=torch.int32, device=dev)
    slots = torch.empty(nb * cap, dtype=torch.uint8, device=dev)
    olen = torch.empty(nb, dtype=torch.int32, device=dev)
    N.launch_compress(src, so, sl, slots, soff, scap, olen, nb, N.TABLE_U16_HASH4 if bs <= 65536 else N.TABLE_AUTO, 1)
    dst = torch.zeros(nb * bs, dtype=torch.uint8, device=dev)
    st = torch.empty(nb, dtype=torch.int32, device=dev)
    buf = (C.c_ulonglong * 16)()
    torch.cuda.synchronize()
    lib.lz4m_hist_prof(buf, 1)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    N.launch_decompress(slots, soff, olen, dst, so, sl, st, nb)
    e1.record()
    torch.cuda.synchronize()
    print(f"{kind}: launch {e0.elapsed_time(e1):.2f} ms", flush=True)
    lib.lz4m_hist_prof(buf, 1)
    ok = bool((st == bs).all()) and torch.equal(dst, src)
    v = list(buf)
    tot = sum(v[i] for i in (0, 1, 2, 3, 4, 5, 6, 7, 15))
    rounds = max(v[8], 1)
    print(f"{kind}: {nb} blocks ok={ok} rounds/block={v[8] / nb:.1f} seqs/round={v[10] / rounds:.1f} "
          f"passes/round={v[9] / rounds:.2f} cycles/round={tot / rounds:.0f}", flush=True)
    for i in (0, 1, 2, 3, 4, 5, 6, 7, 15):
        print(f"   {NAMES[i]:>16}: {100 * v[i] / max(tot, 1):5.1f} %  {v[i] / rounds:8.0f} cyc/round", flush=True)
