"""Dev probe for the quad executor (lz4m_rows.hip quad_exec_kernel): runs the
test corpus of tests/test_gpu_codec.py::test_decompress_matches_oracle with an
iteration bound (lz4m_quad_debug) and prints the state of any wave that hit
it, then the blocks whose bytes or statuses differ from the oracle's."""
import ctypes
import os
import random
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "python-lz4_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
from lz4 import _native as N, _synth  # noqa: E402
import oracle as O  # noqa: E402

dev = torch.device("cuda", 0)
orc = O.Oracle()
blocks = [b.tobytes() for b in _synth.blocks(int(os.environ.get("NB", 96)), "silesia", seed=11)]
rng = random.Random(5)
sizes = [0, 1, 4, 5, 11, 12, 13, 14, 15, 16, 17, 31, 32, 63, 64, 65, 100, 255, 256, 1000, 4095, 4096, 65535, 65536]
src = blocks + [blocks[rng.randrange(len(blocks))][:s] for s in sizes] + [bytes(65536), bytes([7]) * 65536, b"ab" * 32768]
comp = [orc.compress(b) for b in src]
L = N.lib()
L.lz4m_quad_debug.argtypes = [ctypes.c_void_p, ctypes.c_uint32]
dbg = torch.zeros(64 * 64 * 16, dtype=torch.int32, device=dev)
L.lz4m_quad_debug(dbg.data_ptr(), int(os.environ.get("MAXIT", 200000)))
offs, acc = [], 0
for c in comp:
    offs.append(acc)
    acc += len(c)
d_src = N.to_device(b"".join(comp) + bytes(64), dev)
caps = [len(b) for b in src]
doff = np.cumsum([0] + caps[:-1]).tolist()
d_dst = torch.zeros(sum(caps) + 64, dtype=torch.uint8, device=dev)
st = torch.empty(len(src), dtype=torch.int32, device=dev)
N.launch_decompress(d_src, torch.tensor(offs, dtype=torch.int64, device=dev),
                    torch.tensor([len(c) for c in comp], dtype=torch.int32, device=dev), d_dst,
                    torch.tensor(doff, dtype=torch.int64, device=dev), torch.tensor(caps, dtype=torch.int32, device=dev),
                    st, len(src), decoder=os.environ.get("DEC", "quad"))
torch.cuda.synchronize()
D = dbg.cpu().numpy().reshape(64, 64, 16)
for w in range(64):
    for ln in range(0, 64, 4):
        if D[w, ln, 15] == 0x5A5A:
            print("wave", D[w, ln, 14], "quad", ln // 4, "flags", bin(D[w, ln, 0]), "nseq kF ipF oF base F kL kI kE useE iend",
                  D[w, ln, 1:12].tolist(), "lenL", D[w, ln:ln + 4, 12].tolist(), "lenI", D[w, ln:ln + 4, 13].tolist())
F = dbg.cpu().numpy()
print("bad decodes:", F[-1])
for e in range(min(32, F[-1])):
    w = F[-1 - 16 * (e + 1): -1 - 16 * e]
    print("  wg lane k ip len lit off ml oF o wa0 wa1 nseq iend base", w.tolist())
host = d_dst.cpu().numpy()
bad = 0
for i, s in enumerate(st.cpu().tolist()):
    out = host[doff[i]:doff[i] + max(s, 0)].tobytes()
    if s != len(src[i]) or out != src[i]:
        bad += 1
        if bad <= 10:
            j = next((k for k in range(min(len(out), len(src[i]))) if out[k] != src[i][k]), None)
            print("block", i, "status", s, "want", len(src[i]), "first diff", j)
            if j is not None and bad <= 3:   # the sequences around it
                c, ip, op, k = comp[i], 0, 0, 0
                while ip < len(c):
                    tk = c[ip]; ip0 = ip; ip += 1; L = tk >> 4
                    if L == 15:
                        while True:
                            x = c[ip]; ip += 1; L += x
                            if x != 255: break
                    ip += L
                    if ip >= len(c): break
                    off = c[ip] | (c[ip + 1] << 8); ip += 2; M = tk & 15
                    if M == 15:
                        while True:
                            x = c[ip]; ip += 1; M += x
                            if x != 255: break
                    M += 4
                    if op + L + M > j - 40 and op < j + 20:
                        print(f"   seq {k} (round {k // 4} lane {k % 4}) ip {ip0} o {op} lit {L} off {off} ml {M} src {op + L - off}")
                    op += L + M; k += 1
                    if op > j + 20: break
                print("   got ", out[max(0, j - 8):j + 24])
                print("   want", src[i][max(0, j - 8):j + 24])
print("bad blocks:", bad, "of", len(src))
