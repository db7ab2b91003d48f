"""Dev probe: where a default (64 KiB linked) lz4.frame.decompress of a
256 MiB silesia-like frame spends its time (warm call, cProfile)."""
import cProfile
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "python-lz4_amd"))
import torch  # noqa: E402
import lz4.frame as F  # noqa: E402
from lz4 import _synth  # noqa: E402

data = _synth.blocks(int(os.environ.get("NB", "4096")), "silesia", seed=3).tobytes()
f = F.compress(data)
for _ in range(2):
    t = time.perf_counter()
    out = F.decompress(f)
    torch.cuda.synchronize()
    print("warm decode", round(time.perf_counter() - t, 4), "s", out == data, flush=True)
pr = cProfile.Profile()
pr.enable()
out = F.decompress(f)
pr.disable()
pstats.Stats(pr).sort_stats("cumulative").print_stats(18)
