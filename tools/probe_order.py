"""Dev probe: does the order in which the row decoder's kernels take blocks
matter (the tails of rows_parse_kernel / rows_exec_kernel)?  Builds config 2's
batch like bench.py (seed 2026, pool 4096, exact LZ4_compress_default parse),
then decodes (a) prefixes of M blocks in natural order -- time(M) = a + b*M,
the intercept a is the kernels' ramp and tail -- and (b) the whole batch in
other block orders (the batch's arrays permuted; every output still lands in
its own slot, so the bytes check is the same).  Run it under rocprofv3
--kernel-trace --stats for the per-kernel split.
env: NBLK (1048576), REPS (3), ORDERS (natural,len_desc,len_asc), PREFIX (block counts),
SUBSETS (lo:hi compressed-length ranges, e.g. 0:5000,5000:99999)."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "python-lz4_amd"))
sys.path.insert(0, ROOT)
import bench as B  # noqa: E402
from lz4 import _native as N  # noqa: E402

dev = torch.device("cuda", 0)
n = int(os.environ.get("NBLK", 1 << 20))
reps = int(os.environ.get("REPS", 3))
src = B.make_batch(n, 4096, "silesia", 2026, dev)
so, sl, slots, soff, scap, olen = B.compress_all(src, n, 0, dev)
N.launch_compress(src, so, sl, slots, soff, scap, olen, n, N.TABLE_U16_HASH4, 1)
offs = N.exclusive_scan(olen)
tot = int(offs[n])
comp = torch.empty(tot, dtype=torch.uint8, device=dev)
N.gather(slots, soff, olen, comp, offs, n)
coff = offs[:n].clone()
clen = olen.clone()
del slots, soff, scap, so, sl
torch.cuda.empty_cache()
dst = torch.empty(n * 65536, dtype=torch.uint8, device=dev)
doff = torch.arange(n, dtype=torch.int64, device=dev) * 65536
dcap = torch.full((n,), 65536, dtype=torch.int32, device=dev)
st = torch.empty(n, dtype=torch.int32, device=dev)
print(f"ratio {n * 65536 / tot:.3f}", flush=True)


def run(tag, co, cl, do, dc, m, check):
    N.launch_decompress(comp, co, cl, dst, do, dc, st[:m], m)   # untimed (scratch)
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        N.launch_decompress(comp, co, cl, dst, do, dc, st[:m], m)
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
    ok = bool((st[:m] == 65536).all())
    if check:
        ok = ok and torch.equal(dst, src)
    r = {"blocks": m, "ms": sorted(ts), "ok": ok}
    print(tag, json.dumps(r), flush=True)
    return r


res = {}
for m in [int(x) for x in os.environ.get("PREFIX", "262144,524288,786432").split(",") if x]:
    res[f"prefix_{m}"] = run(f"prefix_{m}", coff[:m], clen[:m], doff[:m], dcap[:m], m, False)
for order in os.environ.get("ORDERS", "natural,len_desc,len_asc").split(","):
    if order == "natural":
        perm = torch.arange(n, device=dev)
    elif order == "len_desc":
        perm = torch.argsort(clen, descending=True, stable=True)
    elif order == "len_asc":
        perm = torch.argsort(clen, stable=True)
    else:
        raise SystemExit(order)
    dst.zero_()
    res[order] = run(order, coff[perm].contiguous(), clen[perm].contiguous(), doff[perm].contiguous(),
                     dcap[perm].contiguous(), n, True)
# subsets by compressed length (runs blocks: ratio ~54, ~1.2 KB each)
for sub in [x for x in os.environ.get("SUBSETS", "").split(",") if x]:
    lo, hi = (int(v) for v in sub.split(":"))
    sel = torch.nonzero((clen >= lo) & (clen < hi)).flatten()
    m = int(sel.numel())
    res[f"len_{sub}"] = run(f"len_{sub}", coff[sel].contiguous(), clen[sel].contiguous(), doff[sel].contiguous(),
                            dcap[sel].contiguous(), m, False)
print(json.dumps(res))
