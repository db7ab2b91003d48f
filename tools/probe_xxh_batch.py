"""Dev probe: lz4m_xxh32_batch throughput on config-5-like
pages -- 4 096 items of a compressed silesia-like length mix (~34 KiB mean),
and 2 048 x 4 MiB items (block checksums of config 4's frame blocks).
Times with HIP events on the launch stream; prints GB/s hashed."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "python-lz4_amd"))
from lz4 import _native as N  # noqa: E402

dev = torch.device("cuda", 0)
rng = np.random.default_rng(1)


def run(name, lens, reps=20):
    lens = np.asarray(lens, dtype=np.int64)
    offs = np.concatenate([[0], np.cumsum(lens)[:-1]])
    total = int(lens.sum())
    buf = torch.randint(0, 255, (total + 16,), dtype=torch.uint8, device=dev)
    d_off = torch.tensor(offs, device=dev)
    d_len = torch.tensor(lens, device=dev)
    out = torch.empty(len(lens), dtype=torch.int32, device=dev)
    N.launch_xxh32_batch(buf, d_off, d_len, 0, out, len(lens))
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        N.launch_xxh32_batch(buf, d_off, d_len, 0, out, len(lens))
    b.record()
    torch.cuda.synchronize()
    ms = a.elapsed_time(b) / reps
    print(f"{name}: items {len(lens)} bytes {total / 1e6:.1f} MB  {ms:.3f} ms/launch  {total / ms / 1e6:.1f} GB/s",
          flush=True)


# compressed 64 KiB silesia-like blocks: ratio ~1.96 -> ~34 KiB, spread 0.3-64 KiB
page = np.clip(rng.normal(34000, 9000, 4096), 300, 65809).astype(np.int64)
run("page 4096 x ~34 KiB", page)
run("page 4096 x 34 KiB uniform", np.full(4096, 34000))
run("256 x 34 KiB", np.full(256, 34000))
run("65536 x ~34 KiB", np.clip(rng.normal(34000, 9000, 65536), 300, 65809).astype(np.int64), reps=5)
run("2048 x 4 MiB", np.full(2048, 4 << 20), reps=3)
