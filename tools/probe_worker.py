"""Dev probe: single-call compress / decompress through the persistent
workers, with the mailbox state printed (tools/gpu/r04*.sh)."""
import ctypes as C
import os
import random
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "python-lz4_amd"))
import lz4._native as N  # noqa: E402

lib = N.lib()
st = (C.c_uint32 * 16)()


def show(tag):
    f = lib.lz4m_single_call_worker_state(st)
    print(tag, "dec seq/served/quit", list(st[0:3]), "comp", list(st[3:6]), "launched", list(st[6:8]),
          "count/exit dec", list(st[8:10]), "comp", list(st[10:12]),
          "failures", f, "mode", lib.lz4m_single_call_worker(-1), flush=True)


rng = random.Random(1)
data = bytes(range(256)) * 64
out = C.create_string_buffer(70000)
dec = C.create_string_buffer(70000)
show("start")
t = time.perf_counter()
r = lib.lz4m_compress_default(data, out, len(data), 70000)
print("compress ->", r, f"{(time.perf_counter() - t) * 1e6:.0f} us", flush=True)
show("after compress")
comp = out.raw[:r]
t = time.perf_counter()
r2 = lib.lz4m_decompress_safe(comp, dec, len(comp), len(data))
print("decompress ->", r2, dec.raw[:len(data)] == data, f"{(time.perf_counter() - t) * 1e6:.0f} us", flush=True)
show("after decompress")
bad = 0
for i in range(12):
    n = rng.choice([0, 1, 100, 4096, 16384, 65536])
    src = bytes(rng.choice(b"abcdefgh") for _ in range(n // 8)) * 8 + b"x" * (n % 8)
    t = time.perf_counter()
    r = lib.lz4m_compress_default(src, out, len(src), 70000)
    t1 = time.perf_counter()
    r2 = lib.lz4m_decompress_safe(out.raw[:r], dec, r, len(src)) if r > 0 else -99
    t2 = time.perf_counter()
    ok = r2 == len(src) and dec.raw[:len(src)] == src
    bad += not ok
    print(f"pair {i}: n={n} c={r} d={r2} ok={ok} {(t1 - t) * 1e6:.0f}+{(t2 - t1) * 1e6:.0f} us", flush=True)
    if i % 4 == 3:
        time.sleep(0.01)   # the workers go idle and exit; the next call starts them again
        show(f"after idle {i}")
show("end")
sys.exit(1 if bad else 0)
