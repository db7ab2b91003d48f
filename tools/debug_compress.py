"""Debug helper: first differing sequence between GPU and oracle compress."""
import sys, os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "python-lz4_amd")); sys.path.insert(0, os.path.join(ROOT, "oracle")); sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch
import oracle as O
from lz4 import _synth, _native as N
from test_gpu_codec import gpu_compress

def seqs(c):
    out, ip, op = [], 0, 0
    while ip < len(c):
        t = c[ip]; ip += 1; lit = t >> 4
        if lit == 15:
            while True:
                s = c[ip]; ip += 1; lit += s
                if s != 255: break
        lpos = op; ip += lit; op += lit
        if ip >= len(c):
            out.append((lpos, lit, None, None)); break
        off = c[ip] | (c[ip+1] << 8); ip += 2
        ml = t & 15
        if ml == 15:
            while True:
                s = c[ip]; ip += 1; ml += s
                if s != 255: break
        ml += 4
        out.append((lpos, lit, off, ml)); op += ml
    return out

orc = O.Oracle()
blocks = [b.tobytes() for b in _synth.blocks(96, "silesia", seed=11)]
variant = int(sys.argv[1]) if len(sys.argv) > 1 else 0
dev = torch.device("cuda", 0)
B0 = int(os.environ.get("B0", 0)); B1 = int(os.environ.get("B1", 4))
for bi in range(B0, B1):
    g = gpu_compress([blocks[bi]], variant, dev)[0]
    w = orc.compress(blocks[bi], variant)
    sg, sw = seqs(g), seqs(w)
    for k, (a, b) in enumerate(zip(sg, sw)):
        if a != b:
            print("block", bi, "seq", k, "gpu", a, "oracle", b, "prev", sw[k-1] if k else None)
            break
    else:
        print("block", bi, "same" if g == w else "len diff", len(g), len(w))
