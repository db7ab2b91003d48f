"""Dev tool: sequences per block of config 2's synthetic silesia-like data
(bench.py's pool, seed 2026), compressed by the oracle's LZ4_compress_default,
and how many of them the rows parse records as good (every sequence before
the block's last 5 literal bytes and the reference's fast-loop margins) --
the denominator of DESIGN §3.1's cycles-per-sequence table."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "python-lz4_amd"))
sys.path.insert(0, ROOT)
from lz4 import _synth  # noqa: E402
from oracle.oracle import Oracle  # noqa: E402

n = int(os.environ.get("N", "256"))
blocks = _synth.blocks(n, "silesia", seed=2026)
o = Oracle()
tot = lits = mls = comp = 0
for b in blocks:
    c = o.compress(bytes(b))
    comp += len(c)
    i, seqs = 0, 0
    while i < len(c):
        t = c[i]
        i += 1
        L = t >> 4
        if L == 15:
            while True:
                x = c[i]
                i += 1
                L += x
                if x != 255:
                    break
        i += L
        lits += L
        if i >= len(c):
            break
        i += 2
        M = t & 15
        if M == 15:
            while True:
                x = c[i]
                i += 1
                M += x
                if x != 255:
                    break
        mls += M + 4
        seqs += 1
    tot += seqs
print(f"{n} blocks: {tot / n:.1f} sequences per block, ratio {n * 65536 / comp:.3f}, "
      f"{lits / tot:.2f} literal and {mls / tot:.2f} match bytes per sequence, "
      f"{comp / tot:.2f} compressed bytes per sequence")
