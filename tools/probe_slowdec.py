"""Dev probe: per-call times of one random 64 KiB block's decode through the
staged C call and lz4.block, worker on and off (r04m)."""
import ctypes as C
import os
import random
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "python-lz4_amd"))
import lz4._native as N  # noqa: E402
import lz4.block as B  # noqa: E402

lib = N.lib()
rand = random.Random(7).randbytes(65536)
out = C.create_string_buffer(70000)
p = C.c_void_p()
r = lib.lz4m_compress_default(rand, out, 65536, 70000)   # the call before out.raw is read
cr = out.raw[:r]
cb = B.compress(rand)
print("compress_default", len(cr), "block api", len(cb) - 4, "same", cr == cb[4:], flush=True)


def t(f, k=6):
    r = []
    for _ in range(k):
        s = time.perf_counter()
        v = f()
        r.append((time.perf_counter() - s) * 1e6)
    return v, " ".join(f"{x:.0f}" for x in r)


for mode in (1, 0):
    lib.lz4m_single_call_worker(mode)
    v, s = t(lambda: lib.lz4m_decompress_safe_staged(cr, len(cr), 65536, C.byref(p)))
    print(f"worker={mode} staged(cr): r={v} us: {s}", flush=True)
    ok = C.string_at(p.value, 65536) == rand
    v, s = t(lambda: B.decompress(cb))
    print(f"worker={mode} B.decompress(cb): ok={v == rand} us: {s}; staged ok={ok}", flush=True)
    v, s = t(lambda: lib.lz4m_decompress_safe_staged(cb[4:], len(cb) - 4, 65536, C.byref(p)))
    print(f"worker={mode} staged(cb[4:]): r={v} us: {s}", flush=True)
    v, s = t(lambda: lib.lz4m_decompress_safe_staged(cr, len(cr), 65536, C.byref(p)))
    print(f"worker={mode} staged(cr) again: r={v} us: {s}", flush=True)
