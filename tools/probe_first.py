"""Dev probe: the first single-call compress of a fresh process (argv: buffer
size, capacity, 'torch' to import lz4.block first), repeated, against the
oracle (r04o)."""
import ctypes as C
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "python-lz4_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import lz4._native as N  # noqa: E402
if "torch" in sys.argv:
    import lz4.block  # noqa: F401,E402
import oracle as O  # noqa: E402

buf, cap = int(sys.argv[1]), int(sys.argv[2])
lib = N.lib()
rand = random.Random(7).randbytes(65536)
want = O.Oracle().compress(rand)
for i in range(4):
    out = C.create_string_buffer(buf)
    r = lib.lz4m_compress_default(rand, out, 65536, cap)
    got = out.raw[:r]
    diffs = [k for k in range(min(len(got), len(want))) if got[k] != want[k]]
    print(f"buf={buf} cap={cap} {sys.argv[3:]} call {i}: r={r} same={got == want} ndiff={len(diffs)} "
          f"first={diffs[:4]} got={got[diffs[0]:diffs[0] + 8].hex() if diffs else ''} "
          f"want={want[diffs[0]:diffs[0] + 8].hex() if diffs else ''}", flush=True)
