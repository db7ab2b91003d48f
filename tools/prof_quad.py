"""Dev probe: per-phase wave-cycle split of the quad executor (quad_exec_kernel,
lz4m_rows.hip).  Needs the diagnostic build (tools/prof_rows.sh ->
tools/_prof/_lz4m_rprof.so) loaded through LZ4M_LIB."""
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
EN = {8: "grab", 9: "big path", 10: "rebase", 11: "sub-steps", 12: "flush", 13: "decode", 14: "L->I",
      15: "L issue"}
for kind in os.environ.get("KINDS", "silesia").split(","):
    nb = int(os.environ.get("NB", "262144"))
    src = B.make_batch(nb, min(4096, nb), kind, 7, dev)
    so, sl, slots, soff, scap, olen = B.compress_all(src, nb, 0, dev)
    N.launch_compress(src, so, sl, slots, soff, scap, olen, nb, N.TABLE_U16_HASH4, 1)
    dst = torch.zeros(nb * 65536, dtype=torch.uint8, device=dev)
    doff = torch.arange(nb, dtype=torch.int64, device=dev) * 65536
    dcap = torch.full((nb,), 65536, dtype=torch.int32, device=dev)
    st = torch.empty(nb, dtype=torch.int32, device=dev)
    buf = (C.c_ulonglong * 32)()
    for rep in range(2):
        torch.cuda.synchronize()
        lib.lz4m_rows_prof(buf, 1)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        N.launch_decompress(slots, soff, olen, dst, doff, dcap, st, nb, decoder="quad")
        b.record()
        torch.cuda.synchronize()
        lib.lz4m_rows_prof(buf, 1)
    ok = bool((st == 65536).all()) and torch.equal(dst, src)
    v = list(buf)
    it = max(v[16], 1)
    et = sum(v[i] for i in EN)
    print(f"{kind}: {nb} blocks ok={ok} {a.elapsed_time(b):.2f} ms (prof build)")
    print(f"  wave iterations {v[16]}  quad-rounds executed {v[17]} ({v[17] / it:.2f}/iter) decoded {v[20]} "
          f"seqs {v[21]} ({v[21] / max(v[17], 1):.2f}/round)  big {v[18]}  rebases {v[19]} "
          f"cycles/iter {et / it:.0f}")
    for i in EN:
        print(f"     {EN[i]:>10}: {100 * v[i] / max(et, 1):5.1f} %  {v[i] / it:7.0f} cyc/iter")
    del src, slots, dst
    torch.cuda.empty_cache()
