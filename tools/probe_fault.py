"""Dev probe: what bounds the drop-in download (lz4._native.to_host_bytes):
copying 8 GiB from pinned staging into a fresh result bytes object (first
touch: page faults and kernel zeroing) against the same copy into memory
already touched, with transparent huge pages requested (madvise) on the
fresh buffer, and with more copy threads.  Host only (pinned buffers need
the GPU runtime)."""
import ctypes as C
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "python-lz4_amd"))
from lz4 import _native as N  # noqa: E402

for f in ("enabled", "defrag"):
    try:
        print(f"THP {f}: {open('/sys/kernel/mm/transparent_hugepage/' + f).read().strip()}", flush=True)
    except OSError as e:
        print(f"THP {f}: {e}", flush=True)
libc = C.CDLL("libc.so.6", use_errno=True)
libc.madvise.argtypes = [C.c_void_p, C.c_size_t, C.c_int]
MADV_HUGEPAGE = 14
n = int(os.environ.get("GIB", "8")) << 30
ch = 64 << 20
bufs = N._pinned_pair(ch)
bufs[0].fill_(7)
bufs[1].fill_(9)
src = bufs[0].data_ptr()
print(f"copy threads default {N._copy_threads()}", flush=True)


def run(label, dst, thr, hash_=False):
    st = N.HostXXH32(0) if hash_ else None
    t = time.perf_counter()
    for lo in range(0, n, ch):
        N.lib().lz4m_host_copy(dst + lo, src, min(ch, n - lo), thr, None if st is None else st._st)
    dt = time.perf_counter() - t
    print(f"{label}: {n / dt / 1e9:.2f} GB/s ({dt * 1e3:.0f} ms)", flush=True)


def fresh(huge):
    b, dst = N._new_host_buffer(n, False)
    if huge:
        a = (dst + (2 << 20) - 1) & ~((2 << 20) - 1)
        r = libc.madvise(a, (dst + n - a) & ~((2 << 20) - 1), MADV_HUGEPAGE)
        if r != 0:
            print(f"madvise failed errno {C.get_errno()}", flush=True)
    return b, dst


thr = N._copy_threads()
b, dst = fresh(False)
run(f"fresh bytes, {thr} threads", dst, thr)
run(f"same bytes again (touched), {thr} threads", dst, thr)
run(f"touched, {thr} threads + hash riding", dst, thr, True)
del b
b, dst = fresh(False)
run(f"fresh bytes, {thr} threads + hash riding", dst, thr, True)
del b
b, dst = fresh(True)
run(f"fresh bytes + MADV_HUGEPAGE, {thr} threads", dst, thr)
del b
b, dst = fresh(True)
run(f"fresh bytes + MADV_HUGEPAGE, {thr} threads + hash riding", dst, thr, True)
del b
b, dst = fresh(False)
run("fresh bytes, 15 threads", dst, 15)
del b
b, dst = fresh(True)
run("fresh bytes + MADV_HUGEPAGE, 15 threads", dst, 15)
del b
N._pinned_release(ch, bufs)
