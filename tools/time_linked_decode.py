import sys, time
sys.path.insert(0, "python-lz4_amd")
import torch, lz4.frame as F, lz4._native as N
from lz4 import _synth
data = _synth.blocks(4096, "silesia", seed=3).tobytes()
f = F.compress(data)
t = time.perf_counter(); out = F.decompress(f); dt = time.perf_counter() - t
print("linked 64K frame decode 256MiB:", round(dt, 3), "s", out == data, flush=True)
f4 = F.compress(data, block_size=7)
t = time.perf_counter(); out = F.decompress(f4); dt = time.perf_counter() - t
print("linked 4M frame decode 256MiB:", round(dt, 3), "s", out == data, flush=True)
