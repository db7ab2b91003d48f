"""Decoder profiling driver: per-kind timing of the batched decode kernel."""
import os, sys, time, json
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "python-lz4_amd"))
import torch
from lz4 import _native as N, _synth
sys.path.insert(0, ROOT)
import bench

dev = torch.device("cuda", 0)
n = int(os.environ.get("NBLK", 65536))
kinds = os.environ.get("KINDS", "silesia,text,source,records,markup,random,runs").split(",")
reps = int(os.environ.get("REPS", 3))
out = {}
for kind in kinds:
    src = bench.make_batch(n, min(2048, n), kind, 7, dev)
    so, sl, slots, soff, scap, olen = bench.compress_all(src, n, 0, dev)
    N.launch_compress(src, so, sl, slots, soff, scap, olen, n, N.TABLE_U16_HASH4, 1)
    torch.cuda.synchronize()
    cbytes = int(olen.to(torch.int64).sum())
    dst = torch.empty(n * 65536, dtype=torch.uint8, device=dev)
    doff = torch.arange(n, dtype=torch.int64, device=dev) * 65536
    dcap = torch.full((n,), 65536, dtype=torch.int32, device=dev)
    st = torch.empty(n, dtype=torch.int32, device=dev)
    N.launch_decompress(slots, soff, olen, dst, doff, dcap, st, n)
    torch.cuda.synchronize()
    assert torch.equal(dst, src)
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(); N.launch_decompress(slots, soff, olen, dst, doff, dcap, st, n); b.record()
        torch.cuda.synchronize(); ts.append(a.elapsed_time(b))
    ms = min(ts)
    out[kind] = {"ms": round(ms, 3), "ratio": round(n * 65536 / cbytes, 3), "GiB_s": round(n * 65536 / ms / 1e-3 / 2**30, 1),
                 "algo_GB_s": round((cbytes + n * 65536) / ms / 1e6, 1)}
    print(kind, out[kind], flush=True)
    del src, slots, dst
    torch.cuda.empty_cache()
print(json.dumps(out))
