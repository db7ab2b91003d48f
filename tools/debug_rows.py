"""Dev: check the row decoder's parse records (meta + lengths) against a
Python parse, and locate the first wrong output byte by sequence."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "python-lz4_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
from lz4 import _native as N, _synth  # noqa: E402
import oracle as O  # noqa: E402

orc = O.Oracle()
dev = torch.device("cuda", 0)


def pyparse(c, cap):
    i, op, seqs = 0, 0, []
    n = len(c)
    while i < n:
        t = c[i]
        st = i
        i += 1
        lit = t >> 4
        if lit == 15:
            while True:
                b = c[i]; i += 1; lit += b
                if b != 255:
                    break
        i += lit
        if i >= n:
            break
        off = c[i] | (c[i + 1] << 8); i += 2
        ml = t & 15
        if ml == 15:
            while True:
                b = c[i]; i += 1; ml += b
                if b != 255:
                    break
        ml += 4
        seqs.append((st, i - st, op, lit, off, ml))
        op += lit + ml
    return seqs


blocks = [b.tobytes() for b in _synth.blocks(96, "silesia", seed=11)]
for bi in range(int(os.environ.get("NB", "4"))):
    raw = blocks[bi]
    comp = orc.compress(raw)
    d_src = N.to_device(comp, dev)
    dst = torch.zeros(65536, dtype=torch.uint8, device=dev)
    st = torch.empty(1, dtype=torch.int32, device=dev)
    args = (d_src, torch.zeros(1, dtype=torch.int64, device=dev), torch.tensor([len(comp)], dtype=torch.int32, device=dev),
            dst, torch.zeros(1, dtype=torch.int64, device=dev), torch.tensor([65536], dtype=torch.int32, device=dev), st, 1)
    N.launch_decompress(*args, decoder="rows")
    torch.cuda.synchronize()
    w = list(N._WORK.values())[0]
    meta = w[64:96].cpu().numpy().view(np.int32)
    loff = int(meta[0]) | (int(meta[1]) << 32)
    nseq, ip, op = int(meta[2]), int(meta[3]), int(meta[4])
    seqs = pyparse(comp, 65536)
    fixed = 64 + 32
    lens = w[fixed + loff: fixed + loff + nseq].cpu().numpy()
    want = np.array([min(s[1], 255) for s in seqs[:nseq]], dtype=np.uint8)
    out = dst.cpu().numpy().tobytes()
    diff = next((i for i in range(65536) if out[i] != raw[i]), None)
    print(f"block {bi}: status {int(st.item())} nseq {nseq} (python total {len(seqs)}) ip {ip} op {op} "
          f"lens_match {bool((lens == want).all())} first_len_diff "
          f"{next((i for i in range(nseq) if lens[i] != want[i]), None)} out_diff {diff}")
    if diff is not None:
        k = max(i for i, s in enumerate(seqs) if s[2] <= diff)
        print("  seq", k, seqs[k], "round", k // 16, "lane", k % 16, "prev", seqs[k - 1] if k else None)
        print("  got", out[diff - 8:diff + 8], "want", raw[diff - 8:diff + 8])
