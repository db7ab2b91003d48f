"""Dev probe: lz4m_compress_default on one random 64 KiB block at capacities
around LZ4_compressBound, worker on and off, against the oracle (r04n)."""
import ctypes as C
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "python-lz4_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import lz4._native as N  # noqa: E402
import oracle as O  # noqa: E402

lib = N.lib()
orc = O.Oracle()
for seed, n in ((7, 65536), (3, 65535), (5, 4096)):
    data = random.Random(seed).randbytes(n)
    want = orc.compress(data)
    for mode in (1, 0):
        lib.lz4m_single_call_worker(mode)
        for cap in (O.compress_bound(n), O.compress_bound(n) + 1, O.compress_bound(n) + 64, 70000, 200000):
            out = C.create_string_buffer(cap + 64)
            r = lib.lz4m_compress_default(data, out, n, cap)
            got = out.raw[:r]
            diff = next((i for i in range(min(len(got), len(want))) if got[i] != want[i]), None)
            r2 = lib.lz4m_compress_block_api(data, out, n, cap, 1)
            g2 = out.raw[:r2]
            print(f"n={n} worker={mode} cap={cap}: default r={r} same={got == want} first diff={diff} "
                  f"got[{diff}:+8]={got[diff:diff + 8].hex() if diff is not None else ''} "
                  f"want={want[diff:diff + 8].hex() if diff is not None else ''}; block_api r={r2} "
                  f"same={g2 == orc.compress(data, variant=O.TABLE_U32_HASH5)}", flush=True)
