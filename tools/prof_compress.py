"""Compressor timing per data kind: exact (LZ4_compress_default parse) vs
parallel parse.  env: NBLK, KINDS, REPS, MODES (exact,parallel)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "python-lz4_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402
from lz4 import _native as N  # noqa: E402

dev = torch.device("cuda", 0)
n = int(os.environ.get("NBLK", 65536))
kinds = os.environ.get("KINDS", "silesia,text,source,records,markup,random,runs").split(",")
modes = os.environ.get("MODES", "exact,parallel").split(",")
reps = int(os.environ.get("REPS", 2))
out = {}
for kind in kinds:
    src = bench.make_batch(n, min(2048, n), kind, 7, dev)
    so, sl, slots, soff, scap, olen = bench.compress_all(src, n, 0, dev)
    row = {}
    for mode in modes:
        table = N.TABLE_U16_HASH4 if mode == "exact" else N.PARSE_PARALLEL
        N.launch_compress(src, so, sl, slots, soff, scap, olen, n, table, 1)
        torch.cuda.synchronize()
        ts = []
        for _ in range(reps):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            N.launch_compress(src, so, sl, slots, soff, scap, olen, n, table, 1)
            b.record()
            torch.cuda.synchronize()
            ts.append(a.elapsed_time(b))
        tot = int(olen.to(torch.int64).sum())
        nocheck = os.environ.get("NOCHECK") == "1"   # timing probes whose output is wrong on purpose
        assert nocheck or int((olen <= 0).sum()) == 0
        # round trip through the GPU decoder
        dst = torch.empty(n * 65536, dtype=torch.uint8, device=dev)
        doff = torch.arange(n, dtype=torch.int64, device=dev) * 65536
        dcap = torch.full((n,), 65536, dtype=torch.int32, device=dev)
        st = torch.empty(n, dtype=torch.int32, device=dev)
        if not nocheck:
            N.launch_decompress(slots, soff, olen, dst, doff, dcap, st, n)
            torch.cuda.synchronize()
            assert torch.equal(dst, src), (kind, mode)
        del dst
        ms = min(ts)
        row[mode] = {"ms": round(ms, 2), "GiB_s": round(n * 65536 / ms / 1e-3 / 2**30, 2), "bytes": tot,
                     "ratio": round(n * 65536 / tot, 4)}
    if "exact" in row and "parallel" in row:
        row["size_vs_exact"] = round(row["parallel"]["bytes"] / row["exact"]["bytes"] - 1, 5)
    out[kind] = row
    print(kind, row, flush=True)
    del src, slots
    torch.cuda.empty_cache()
print(json.dumps(out))
