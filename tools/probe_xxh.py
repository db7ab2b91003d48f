"""Dev probe: XXH32 long-kernel throughput."""
import os, sys, time
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "python-lz4_amd"))
from lz4 import _native as N
dev = torch.device("cuda", 0)
L = 4 << 30
buf = torch.randint(0, 255, (L + 4,), dtype=torch.uint8, device=dev)
out = torch.empty(1, dtype=torch.int32, device=dev)
for sh in (0, 1):
    b = buf[sh:sh + L]
    N.launch_xxh32_long(b, L, 0, out); torch.cuda.synchronize()
    t = time.perf_counter(); N.launch_xxh32_long(b, L, 0, out); torch.cuda.synchronize()
    print(f"xxh32_long shift {sh}: {L/(time.perf_counter()-t)/1e9:.3f} GB/s", flush=True)
