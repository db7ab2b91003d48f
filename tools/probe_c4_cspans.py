"""Dev probe: how config 4's exact compression of 4 MiB independent blocks
(8 GiB, device-resident) behaves when split into block-ordered launches --
on one stream, and alternating over two streams -- to judge pipelining the
drop-in lz4.frame.compress (upload / compress / download overlapped): when
does each launch end?"""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "python-lz4_amd"))
sys.path.insert(0, ROOT)
import bench as B  # noqa: E402
from lz4 import _native as N  # noqa: E402

dev = torch.device("cuda", 0)
L = int(os.environ.get("GIB", "8")) << 30
FB = 4 << 20
src = B.make_batch(L // 65536, 4096, "silesia", 77, dev).view(-1)[:L]
nb = L // FB
raw_off = torch.arange(nb, dtype=torch.int64, device=dev) * FB
raw_len = torch.full((nb,), FB, dtype=torch.int32, device=dev)
slot = N.compress_bound(FB)
cmp = torch.empty(nb * slot, dtype=torch.uint8, device=dev)
cmp_off = torch.arange(nb, dtype=torch.int64, device=dev) * slot
cap = raw_len - 1
cmp_len = torch.empty(nb, dtype=torch.int32, device=dev)
streams = [torch.cuda.current_stream(dev), torch.cuda.Stream(dev)]
N.launch_compress(src, raw_off, raw_len, cmp, cmp_off, cap, cmp_len, nb, N.TABLE_AUTO, 1)
torch.cuda.synchronize()
for bounds in ([0, nb], [0, nb // 2, nb], [0, nb // 16, nb // 4, nb], [0, nb // 4, nb // 2, 3 * nb // 4, nb]):
    for two in (False, True):
        if two and len(bounds) == 2:
            continue
        torch.cuda.synchronize()
        e0 = torch.cuda.Event(enable_timing=True)
        e0.record()
        evs = []
        for k in range(len(bounds) - 1):
            s = streams[k & 1] if two else streams[0]
            s.wait_event(e0)
            a, z = bounds[k], bounds[k + 1]
            with torch.cuda.stream(s):
                N.launch_compress(src, raw_off[a:z], raw_len[a:z], cmp, cmp_off[a:z], cap[a:z], cmp_len[a:z], z - a,
                                  N.TABLE_AUTO, 1, s)
                e = torch.cuda.Event(enable_timing=True)
                e.record(s)
                evs.append(e)
        torch.cuda.synchronize()
        ends = [e0.elapsed_time(e) for e in evs]
        print(f"spans {[b * 16 // nb for b in bounds]}/16 {'two streams' if two else 'one stream'}: launch ends "
              + " ".join(f"{x:.1f}" for x in ends) + f" ms; {L / max(ends) * 1e3 / 2**30:.2f} GiB/s", flush=True)
