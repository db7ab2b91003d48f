"""Dev probe for tools/micro/coop_decode.hip (the cooperative-decoder
prototype): decoded-prefix coverage, bit-exactness of that prefix, and time,
next to the lane decoder on the same blocks."""
import ctypes as C
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "python-lz4_amd"))
sys.path.insert(0, ROOT)
import bench as B  # noqa: E402
from lz4 import _native as N  # noqa: E402

lib = C.CDLL(os.path.join(ROOT, "tools", "micro", "coop_decode.so"))
vp = C.c_void_p
lib.coop_decode.argtypes = [vp, vp, vp, vp, vp, vp, vp, C.c_int64, vp, C.c_int, vp]
lib.coop_decode.restype = C.c_int
dev = torch.device("cuda", 0)
n = int(os.environ.get("NB", 1 << 18))
grid = int(os.environ.get("GRID", 1024))
for kind in os.environ.get("KINDS", "silesia,text").split(","):
    src = B.make_batch(n, min(4096, n), kind, 2026, dev)
    so, sl, slots, soff, scap, olen = B.compress_all(src, n, 0, dev)
    N.launch_compress(src, so, sl, slots, soff, scap, olen, n, N.TABLE_U16_HASH4, 1)
    dst = torch.zeros(n * 65536, dtype=torch.uint8, device=dev)
    prog = torch.zeros(2 * n, dtype=torch.int32, device=dev)
    q = torch.zeros(4, dtype=torch.int64, device=dev)
    run = lambda: lib.coop_decode(slots.data_ptr(), soff.data_ptr(), olen.data_ptr(), dst.data_ptr(), so.data_ptr(),
                                  sl.data_ptr(), prog.data_ptr(), n, q.data_ptr(), grid, None)
    assert run() == 0
    torch.cuda.synchronize()
    r, p_, sg, sq = q.tolist()
    print(f"{kind}: per block {r / n:.1f} rounds, {p_ / max(r, 1):.2f} passes/round, {sg / n:.1f} single steps, "
          f"{sq / max(r - sg, 1):.1f} sequences/round", flush=True)
    ts = []
    for _ in range(3):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(); run(); b.record(); torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
    why = prog.view(n, 2)[:, 0]
    print(kind, "debug caps hit:", int((why == -1).sum()), "rounds,", int((why == -2).sum()), "passes", flush=True)
    op = prog.view(n, 2)[:, 1].to(torch.int64)
    cov = float(op.sum()) / (n * 65536)
    bad = 0
    for lo in range(0, n, 8192):
        hi = min(n, lo + 8192)
        d = dst[lo * 65536:hi * 65536].view(-1, 65536)
        s = src[lo * 65536:hi * 65536].view(-1, 65536)
        mask = torch.arange(65536, device=dev)[None, :] < op[lo:hi, None]
        bad += int(((d != s) & mask).any(dim=1).sum())
    st = torch.empty(n, dtype=torch.int32, device=dev)
    out2 = torch.empty_like(dst)
    N.launch_decompress(slots, soff, olen, out2, so, sl, st, n)
    torch.cuda.synchronize()
    lt = []
    for _ in range(3):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(); N.launch_decompress(slots, soff, olen, out2, so, sl, st, n); b.record(); torch.cuda.synchronize()
        lt.append(a.elapsed_time(b))
    t = min(ts)
    print(f"{kind}: coop {t:.2f} ms for {cov * 100:.1f}% of the output = {cov * n * 65536 / t / 1e6:.1f} GB/s "
          f"(prefix mismatches in {bad} blocks); lane decoder {min(lt):.2f} ms = {n * 65536 / min(lt) / 1e6:.1f} GB/s",
          flush=True)
    del src, slots, dst, out2
    torch.cuda.empty_cache()
