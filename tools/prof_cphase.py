"""Dev probe: per-phase wave-cycle split of the exact compressor
(compress_block_w).  Needs the diagnostic build with -DLZ4M_COMPRESS_PROF
(tools/_prof/_lz4m_cprof.so) loaded through LZ4M_LIB."""
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
lib.lz4m_compress_prof.argtypes = [C.c_void_p, C.c_int]
PH = {0: "fetch", 1: "table+groups", 2: "gather+hit", 3: "catch-up", 4: "literals", 5: "count", 6: "test-next",
      7: "last literals"}
for kind in os.environ.get("KINDS", "silesia").split(","):
    nb = int(os.environ.get("NB", "16384"))
    src = B.make_batch(nb, min(2048, nb), kind, 7, dev)
    so, sl, slots, soff, scap, olen = B.compress_all(src, nb, 0, dev)
    buf = (C.c_ulonglong * 32)()
    torch.cuda.synchronize()
    lib.lz4m_compress_prof(buf, 1)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    N.launch_compress(src, so, sl, slots, soff, scap, olen, nb, N.TABLE_U16_HASH4, 1)
    b.record()
    torch.cuda.synchronize()
    lib.lz4m_compress_prof(buf, 1)
    v = list(buf)
    tot = sum(v[i] for i in PH)
    seq = max(v[9] + v[10], 1)
    print(f"{kind}: {nb} blocks {a.elapsed_time(b):.1f} ms; sequences {seq} ({v[10]} via test-next), "
          f"search steps {v[8]}, group iters {v[11]}, long counts {v[12]}, long catch-ups {v[13]}, "
          f"global-fetch lanes {v[15]}")
    print(f"  wave-cycles per sequence {tot / seq:.0f}: " +
          ", ".join(f"{PH[i]} {v[i] / seq:.0f}" for i in PH))

if os.environ.get("SINGLE"):
    # the single-call path (persistent worker, LDS-staged block) on config 1's random blocks
    import random
    rnd = random.Random(12345)
    blocks = [rnd.randbytes(65536) for _ in range(200)]
    out = C.create_string_buffer(70000)
    for b in blocks[:20]:
        lib.lz4m_compress_default(b, out, 65536, 70000)
    buf = (C.c_ulonglong * 32)()
    lib.lz4m_compress_prof(buf, 1)
    for b in blocks:
        lib.lz4m_compress_default(b, out, 65536, 70000)
    lib.lz4m_compress_prof(buf, 1)
    v = list(buf)
    n = len(blocks)
    print(f"single-call random 64 KiB: per call {sum(v[i] for i in PH) / n:.0f} wave-cycles, search steps "
          f"{v[8] / n:.1f}, group iters {v[11] / n:.1f}, global-fetch lanes {v[15] / n:.1f}; " +
          ", ".join(f"{PH[i]} {v[i] / n:.0f}" for i in PH))
