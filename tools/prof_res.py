"""Dev probe: per-phase wave-cycle split of the block-resident executor.
Needs the diagnostic build (-DLZ4M_RES_PROF; tools/ab_build.sh-style, loaded
through LZ4M_LIB).  env: NB (262144), KINDS (silesia)."""
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
PH = {0: "block setup/prologue", 1: "parse", 2: "output-position wait", 3: "literals", 4: "prepare (+input-position wait)",
      5: "match loop", 6: "end barrier wait", 7: "copy-out + next block"}
for kind in os.environ.get("KINDS", "silesia").split(","):
    nb = int(os.environ.get("NB", "262144"))
    src = B.make_batch(nb, min(4096, nb), kind, 7, dev)
    so, sl, slots, soff, scap, olen = B.compress_all(src, nb, 0, dev)
    N.launch_compress(src, so, sl, slots, soff, scap, olen, nb, N.TABLE_U16_HASH4, 1)
    dst = torch.zeros(nb * 65536, dtype=torch.uint8, device=dev)
    doff = torch.arange(nb, dtype=torch.int64, device=dev) * 65536
    dcap = torch.full((nb,), 65536, dtype=torch.int32, device=dev)
    st = torch.empty(nb, dtype=torch.int32, device=dev)
    buf = (C.c_ulonglong * 16)()
    torch.cuda.synchronize()
    lib.lz4m_res_prof(buf, 1)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    N.launch_decompress(slots, soff, olen, dst, doff, dcap, st, nb, decoder="resident")
    b.record()
    torch.cuda.synchronize()
    lib.lz4m_res_prof(buf, 1)
    ok = bool((st == 65536).all()) and torch.equal(dst, src)
    v = list(buf)
    tot = sum(v[i] for i in PH)
    print(f"{kind}: {nb} blocks ok={ok} ms={a.elapsed_time(b):.2f} (incl. parse + finisher)")
    print(f"  chunks {v[10]}, match-loop iterations {v[11]} ({v[11] / max(v[10], 1):.2f} per chunk), blocks {v[12]}")
    print(f"  wave-cycles per chunk: {tot / max(v[10], 1):.0f}")
    for i, nm in PH.items():
        print(f"    {nm:32s} {100 * v[i] / max(tot, 1):5.1f} %  {v[i] / max(v[10], 1):8.0f} per chunk")
