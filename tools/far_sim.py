"""Dev tool (CPU): far-source line fills of the row executor per history rule.
Replays config 2's synthetic silesia-like blocks (oracle LZ4_compress_default),
in rounds of 16 sequences per row with the executor's rebase rule (history
H, keep, room) or a ring history, and counts the sources below the history
(far) and the 128-byte lines their 16-byte pieces touch.  DESIGN §3.1
"far-source line fills".  env: N (blocks, default 48)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "python-lz4_amd")); sys.path.insert(0, ROOT)
from lz4 import _synth
from oracle.oracle import Oracle
n=int(os.environ.get("N","48"))
blocks=_synth.blocks(n,"silesia",seed=2026); o=Oracle()
def seqs(c):
    i=0; op=0; out=[]
    while i<len(c):
        t=c[i]; i+=1; L=t>>4
        if L==15:
            while True:
                x=c[i]; i+=1; L+=x
                if x!=255: break
        i+=L
        if i>=len(c): break
        off=c[i]|(c[i+1]<<8); i+=2; M=t&15
        if M==15:
            while True:
                x=c[i]; i+=1; M+=x
                if x!=255: break
        M+=4; m=op+L; out.append((m, off, M)); op=m+M
    return out
S=[seqs(o.compress(bytes(b))) for b in blocks]
def lines(a, b):  # 128-B lines touched by [a, b)
    return (b-1)//128 - a//128 + 1
def run(H, keep, room, ring):
    nseq=far=lf=0; offs=[]
    for sq in S:
        base=0; k=0; op=0
        while k < len(sq):
            rnd=sq[k:k+16]
            if not ring:
                if op-base > H-room: base=(op-keep)&~15
                b=base
            # round end
            use=len(rnd)
            for j,(m,off,M) in enumerate(rnd):
                if (not ring and m+M > b+H) or (ring and m+M - op > H - 64):
                    use=j; break
            if use==0: use=1
            rnd=rnd[:use]
            end=rnd[-1][0]+rnd[-1][2]
            for (m,off,M) in rnd:
                s0=m-off
                f = s0 < b if not ring else s0 < end - H
                nseq+=1
                if f:
                    far+=1
                    lf+=lines(s0, s0+16)
                    if M>16: lf+=lines(s0+16, s0+32) - (1 if (s0+16)//128==(s0+15)//128 else 0)
                    if M>32: lf+=lines(s0+32, s0+M) - (1 if (s0+32)//128==(s0+31)//128 else 0)
            op=end; k+=use
    return nseq, far, lf
for cfg in [(1024,512,512,False),(1280,768,512,False),(1536,1024,512,False),(2048,1536,512,False),(1024,0,0,True),(1280,0,0,True),(1536,0,0,True)]:
    a,f,l=run(*cfg)
    print(cfg, f"far {f/a:.3f} lines/seq {l/a:.3f}")
