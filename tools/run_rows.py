"""Dev driver for counter passes: one row-decoder launch over NB silesia-like
blocks (rocprofv3 --pmc target; tools/pmc_run.sh OUT rows_exec tools/run_rows.py)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "python-lz4_amd"))
sys.path.insert(0, ROOT)
import bench as B  # noqa: E402
from lz4 import _native as N  # noqa: E402

dev = torch.device("cuda", 0)
nb = int(os.environ.get("NB", "262144"))
src = B.make_batch(nb, min(4096, nb), os.environ.get("KIND", "silesia"), 7, dev)
so, sl, slots, soff, scap, olen = B.compress_all(src, nb, 0, dev)
N.launch_compress(src, so, sl, slots, soff, scap, olen, nb, N.TABLE_U16_HASH4, 1)
dst = torch.zeros(nb * 65536, dtype=torch.uint8, device=dev)
doff = torch.arange(nb, dtype=torch.int64, device=dev) * 65536
dcap = torch.full((nb,), 65536, dtype=torch.int32, device=dev)
st = torch.empty(nb, dtype=torch.int32, device=dev)
for _ in range(int(os.environ.get("REPS", "2"))):
    N.launch_decompress(slots, soff, olen, dst, doff, dcap, st, nb, decoder=os.environ.get("DEC", "rows"))
torch.cuda.synchronize()
print("ok", bool((st == 65536).all()) and torch.equal(dst, src))
