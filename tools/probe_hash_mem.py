"""Dev probe: the host XXH32 rate over the same 64 MiB hashed 128 times (8 GiB),
by where the bytes sit -- a pinned staging buffer (torch pin_memory), a
buffer with transparent huge pages (madvise), plain 4 KiB pages -- and the
same hashed from a pinned buffer registered from a THP-backed allocation."""
import ctypes as C
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "python-lz4_amd"))
from lz4 import _native as N  # noqa: E402

CH = 64 << 20
REPS = int(os.environ.get("REPS", "128"))


def rate(label, addr):
    st = N.HostXXH32(0)
    st.update_ptr(addr, CH)   # warm
    t = time.perf_counter()
    st = N.HostXXH32(0)
    for _ in range(REPS):
        st.update_ptr(addr, CH)
    dt = time.perf_counter() - t
    print(f"{label:36s} {REPS * CH / dt / 1e9:.2f} GB/s", flush=True)


pin = torch.empty(CH, dtype=torch.uint8, pin_memory=True)
pin.random_(0, 255)
rate("pinned (torch pin_memory)", pin.data_ptr())
os.environ["LZ4M_HUGEPAGES"] = "1"
b, a = N._new_host_buffer(CH, False)
C.memmove(a, pin.data_ptr(), CH)
rate("huge pages (madvise)", a)
os.environ["LZ4M_HUGEPAGES"] = "0"
b2, a2 = N._new_host_buffer(CH, False)
C.memmove(a2, pin.data_ptr(), CH)
rate("4 KiB pages", a2)
# THP-backed allocation registered as pinned memory
hip = C.CDLL("libamdhip64.so")
hip.hipHostRegister.argtypes = [C.c_void_p, C.c_size_t, C.c_uint]
os.environ["LZ4M_HUGEPAGES"] = "1"
b3, a3 = N._new_host_buffer(CH + (2 << 20), False)
al = (a3 + (2 << 20) - 1) & ~((2 << 20) - 1)
C.memmove(al, pin.data_ptr(), CH)
rc = hip.hipHostRegister(al, CH, 0)
print("hipHostRegister rc", rc, flush=True)
rate("registered THP buffer", al)
d = torch.empty(CH, dtype=torch.uint8, device="cuda")
reg = torch.frombuffer((C.c_char * CH).from_address(al), dtype=torch.uint8)
torch.cuda.synchronize()
t = time.perf_counter()
for _ in range(16):
    reg.copy_(d, non_blocking=True)
torch.cuda.synchronize()
print(f"D2H into the registered THP buffer: {16 * CH / (time.perf_counter() - t) / 1e9:.1f} GB/s", flush=True)
t = time.perf_counter()
for _ in range(16):
    pin.copy_(d, non_blocking=True)
torch.cuda.synchronize()
print(f"D2H into torch pinned: {16 * CH / (time.perf_counter() - t) / 1e9:.1f} GB/s", flush=True)
