"""Time linked-block compression (serial vs speculative) on device data.
usage: python tools/time_linked.py [MiB] [kinds...]"""
import os, sys, time
sys.path.insert(0, "python-lz4_amd")
import torch
import lz4._native as N
from lz4 import _synth

mib = int(sys.argv[1]) if len(sys.argv) > 1 else 64
kinds = sys.argv[2:] or ["silesia"]
dev = torch.device("cuda", 0)
L = N.lib()
BENCH_DATA = os.environ.get("DATA") == "bench"   # bench.py's config-4 input (make_batch, seed 77)
for kind in kinds:
    if BENCH_DATA:
        sys.path.insert(0, ".")
        import bench as B
        d = B.make_batch(mib * 16, 4096, kind, 77, dev)
    else:
        data = _synth.blocks(mib * 16, kind, seed=3)
        d = torch.from_numpy(data.reshape(-1)).to(dev)
    n = d.numel()
    for bsize in [int(x) for x in os.environ.get("BSIZES", "65536,4194304").split(",")]:
        nb = (n + bsize - 1) // bsize
        off = torch.arange(nb, dtype=torch.int64, device=dev) * bsize
        ln = torch.full((nb,), bsize, dtype=torch.int32, device=dev)
        ln[-1] = n - (nb - 1) * bsize
        link = torch.ones(nb, dtype=torch.int32, device=dev)
        link[0] = 0
        slot = N.compress_bound(bsize)
        out = torch.empty(nb * slot, dtype=torch.uint8, device=dev)
        oo = torch.arange(nb, dtype=torch.int64, device=dev) * slot
        olen = torch.empty(nb, dtype=torch.int32, device=dev)
        res = {}
        for mode, name in ((N.LINKED_SPECULATIVE, "spec"), (N.LINKED_SERIAL, "serial")):
            if name == "serial" and nb > 64 and mib > 16:
                continue
            N.launch_compress_linked(d, off, ln, link, out, oo, ln - 1, olen, nb, 1, mode=mode)
            torch.cuda.synchronize()
            t = time.perf_counter()
            N.launch_compress_linked(d, off, ln, link, out, oo, ln - 1, olen, nb, 1, mode=mode)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t
            res[name] = (dt, olen.clone())
            print(f"{kind} {mib}MiB bsize={bsize} nb={nb} {name}: {dt*1e3:.1f} ms {n/dt/2**30:.3f} GiB/s"
                  + (f" passes={L.lz4m_compress_linked_passes()}" if name == "spec" else ""), flush=True)
        if "serial" in res:
            print("  same lengths:", bool(torch.equal(res["spec"][1], res["serial"][1])), flush=True)
# the whole default-frame call as bench.py times it (frame records, emit, header) on the same bytes
if os.environ.get("FRAME", "1") != "0":
    from lz4.frame._frame import _compress_frame
    if not BENCH_DATA:
        data = _synth.blocks(mib * 16, kinds[0], seed=3)
        d = torch.from_numpy(data.reshape(-1)).to(dev)
    for rep in range(3):
        torch.cuda.synchronize()
        t = time.perf_counter()
        fr, _ = _compress_frame(d, d.numel())
        torch.cuda.synchronize()
        dt = time.perf_counter() - t
        print(f"_compress_frame (64 KiB linked, exact): {dt * 1e3:.1f} ms {d.numel() / dt / 2**30:.3f} GiB/s "
              f"passes={L.lz4m_compress_linked_passes()}", flush=True)
