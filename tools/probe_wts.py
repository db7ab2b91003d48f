"""Dev probe (LZ4M_WORKER_TS build, tools/abv_build.sh wts -DLZ4M_WORKER_TS=1):
where a lone-block call's time goes.  Per case, the mean of the device stages
(100 MHz real-time clock, from the worker's poll to its done flag) and the
host's wall time around the C call."""
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
rng = random.Random(7)
rand = rng.randbytes(65536)
zeros = bytes(65536)
out = C.create_string_buffer(70000)
r = lib.lz4m_compress_default(rand, out, 65536, 70000)   # the call before out.raw is read
cr = out.raw[:r]
r = lib.lz4m_compress_default(zeros, out, 65536, 70000)
cz = out.raw[:r]
p = C.c_void_p()


def dec(src, cap):
    return lambda: lib.lz4m_decompress_safe_staged(src, len(src), cap, C.byref(p))


def comp(src):
    return lambda: lib.lz4m_compress_block_api_staged(src, len(src), len(src) + len(src) // 255 + 16, 1, 0,
                                                      C.byref(p))


cases = [("decompress random 64 KiB", 0, dec(cr, 65536)), ("decompress zeros 64 KiB", 0, dec(cz, 65536)),
         ("decompress empty", 0, dec(b"\x00", 0)), ("compress random 64 KiB", 1, comp(rand)),
         ("compress 16 zero bytes", 1, comp(bytes(16)))]
names = ["poll->fields", "fields->body", "stage in", "compute", "copy out+fence"]
for name, kind, f in cases:
    for _ in range(20):
        f()
    acc = [0.0] * 5
    sub = [0.0] * 3
    wall = 0.0
    reps = 300
    for _ in range(reps):
        t = time.perf_counter()
        f()
        wall += time.perf_counter() - t
        lib.lz4m_single_call_worker_state(st)
        w = (C.c_uint32 * 8).from_address(p.value - 256 + 32)
        seen, fields = st[12 + 2 * kind], st[13 + 2 * kind]
        marks = [seen, fields, w[0], w[1], w[2], w[3]]
        for i in range(5):
            acc[i] += ((marks[i + 1] - marks[i]) & 0xFFFFFFFF) / 100.0   # 100 MHz ticks -> us
        if kind == 0 and w[5] and w[6]:   # decoder: rounds / flush / exact tail inside "compute"
            sub[0] += ((w[4] - w[1]) & 0xFFFFFFFF) / 100.0
            sub[1] += ((w[5] - w[4]) & 0xFFFFFFFF) / 100.0
            sub[2] += ((w[6] - w[5]) & 0xFFFFFFFF) / 100.0
    dev = sum(acc) / reps
    print(f"{name}: wall {wall / reps * 1e6:.1f} us, device poll->done {dev:.1f} us: " +
          ", ".join(f"{n} {a / reps:.2f}" for n, a in zip(names, acc)) +
          (f" [rounds {sub[0] / reps:.2f}, flush {sub[1] / reps:.2f}, exact tail {sub[2] / reps:.2f}]" if sub[2] else ""),
          flush=True)
