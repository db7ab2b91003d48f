"""Dev probe: per-phase wave-cycle split of the row decoder (parse and
execution kernels).  Needs the diagnostic build (tools/prof_rows.sh ->
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
PN = {0: "assign", 1: "general step", 2: "fast loop"}
EN = {14: "block grab", 8: "sync parse", 10: "use==0 paths", 11: "literal", 12: "pass setup",
      13: "passes", 15: "parse ahead", 9: "flush+rebase", 20: "block end flush", 21: "non-fit copy", 22: "nseq0 skip"}
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
    torch.cuda.synchronize()
    lib.lz4m_rows_prof(buf, 1)
    N.launch_decompress(slots, soff, olen, dst, doff, dcap, st, nb, decoder="rows")
    torch.cuda.synchronize()
    lib.lz4m_rows_prof(buf, 1)
    ok = bool((st == 65536).all()) and torch.equal(dst, src)
    v = list(buf)
    pt = sum(v[i] for i in PN)
    print(f"{kind}: {nb} blocks ok={ok}")
    print(f"  parse: fast steps {v[3]} (lanes/step {v[5] / max(v[3], 1):.1f}), general steps {v[4]} "
          f"(lanes/step {v[6] / max(v[4], 1):.1f}); cycles/fast step {v[2] / max(v[3], 1):.0f}, "
          f"cycles/general step {v[1] / max(v[4], 1):.0f}")
    for i in PN:
        print(f"     {PN[i]:>14}: {100 * v[i] / max(pt, 1):5.1f} %")
    et = sum(v[i] for i in EN)
    rounds = max(v[16], 1)
    print(f"  exec: rounds {v[16]} seqs/round(row0) {v[18] / rounds:.1f} passes/round {v[17] / rounds:.2f} "
          f"sync-load rounds {v[19] / 16 / rounds:.3f} cycles/round {et / rounds:.0f}")
    print(f"  blocks grabbed {v[23]} nseq0 {v[24]} non-fit seqs {v[25]}")
    for i in EN:
        print(f"     {EN[i]:>14}: {100 * v[i] / max(et, 1):5.1f} %  {v[i] / rounds:7.0f} cyc/round")
    del src, slots, dst
    torch.cuda.empty_cache()
