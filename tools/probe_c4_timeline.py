"""Dev probe: timeline of config 4's hash-following frame decode (8 GiB,
4 MiB independent blocks, content checksum): when each block-ordered decode
launch ends (HIP events) and when the host hash gets to each 64 MiB piece,
relative to the call's start.  Shows whether the hash waits for the decode
(the decode launches must stay ahead of ~13.8 GB/s of hashing).
FOLLOW_CHUNKS=<k> overrides the launch count, DECODER=<name> forces the
decoder of the launches (lz4._native.DECODERS); LZ4M_FOLLOW_SPLIT=0 the
round-5 layout of equal launches on one stream."""
import os
import sys
import threading
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "python-lz4_amd"))
sys.path.insert(0, ROOT)
import bench as B  # noqa: E402
import lz4.frame  # noqa: E402
from lz4 import _native as N  # noqa: E402
from lz4.frame import _frame as F  # noqa: E402

dev = torch.device("cuda", 0)
L = int(os.environ.get("GIB", "8")) << 30
src = B.make_batch(L // 65536, 4096, "silesia", 2026, dev).view(-1)[:L]
frame = lz4.frame.compress_device(src, L, block_size=7, content_checksum=True, block_linked=False, parse="parallel")
torch.cuda.synchronize()
print(f"frame {frame.numel() / 2**30:.2f} GiB", flush=True)
if "FOLLOW_CHUNKS" in os.environ:
    F._FOLLOW_CHUNKS = int(os.environ["FOLLOW_CHUNKS"])

# wrap the piece loop: log when each piece is hashed
marks = []
orig_update = N.HostXXH32.update_ptr


def update_ptr(self, p, n):
    orig_update(self, p, n)
    marks.append((time.perf_counter(), n))


N.HostXXH32.update_ptr = update_ptr

# the decode launches: time each span's event against a start event
orig_launch = N.launch_decompress
launch_evs = []


DEC = os.environ.get("DECODER")


def launch(*a, **k):
    if DEC:
        k["decoder"] = DEC
    orig_launch(*a, **k)
    e = torch.cuda.Event(enable_timing=True)
    e.record(k.get("stream"))
    launch_evs.append((time.perf_counter(), e))


N.launch_decompress = launch
for rep in range(3):
    marks.clear()
    launch_evs.clear()
    torch.cuda.synchronize()
    e0 = torch.cuda.Event(enable_timing=True)
    e0.record()
    t0 = time.perf_counter()
    out = lz4.frame.decompress_device(frame)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    ok = torch.equal(out, src)
    del out
    print(f"rep {rep}: {dt * 1e3:.1f} ms = {L / dt / 2**30:.2f} GiB/s ok={ok} launches={len(launch_evs)}", flush=True)
    if rep == 0:
        continue
    ends = [e0.elapsed_time(e) for _, e in launch_evs]
    enq = [(t - t0) * 1e3 for t, _ in launch_evs]
    print("  launch enqueued (host ms): " + " ".join(f"{x:.1f}" for x in enq), flush=True)
    print("  launch done (device ms):   " + " ".join(f"{x:.1f}" for x in ends), flush=True)
    hs = [(t - t0) * 1e3 for t, _ in marks]
    if hs:
        gaps = [b - a for a, b in zip(hs, hs[1:])]
        print(f"  hash pieces: {len(hs)}, first done {hs[0]:.1f} ms, last {hs[-1]:.1f} ms, "
              f"median gap {sorted(gaps)[len(gaps) // 2] if gaps else 0:.2f} ms, max gap {max(gaps) if gaps else 0:.2f}",
              flush=True)
        print("  hash done at (ms): " + " ".join(f"{x:.0f}" for x in hs[:: max(1, len(hs) // 32)]), flush=True)
