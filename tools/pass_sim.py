"""Dev tool (CPU): readiness passes of the row executor per round (the
kernel's rule: a match is ready once every earlier pending match of the round
ends at or before its source or starts at or after its source's end), with far
copies as now, held out of pass 1, or held until no near lane is ready; the
wave's count is the max over 4 rows (4 consecutive rounds of a block stand in
for the 4 blocks of a wave).  1280-byte histories.  env: N, SEED."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__))); sys.path.insert(0, os.path.join(ROOT, "python-lz4_amd")); sys.path.insert(0, ROOT)
from lz4 import _synth
from oracle.oracle import Oracle
n=int(os.environ.get("N","32")); seed=int(os.environ.get("SEED","2026"))
blocks=_synth.blocks(n,"silesia",seed=seed); o=Oracle()
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
H,KEEP,ROOM=1280,768,512
def passes(rnd, base, defer):
    # rnd: list of (m, off, ml); returns number of passes
    pend=[True]*len(rnd); far=[(m-off)<base for (m,off,ml) in rnd]
    p=0
    while any(pend):
        p+=1
        ready=[]
        for j,(m,off,ml) in enumerate(rnd):
            if not pend[j]: continue
            s0=m-off; se=s0+min(off,ml)
            below=[rnd[i] for i in range(j) if pend[i]]
            x=max([mi+mli for (mi,oi,mli) in below], default=-1)
            y=min([mi for (mi,oi,mli) in below], default=1<<30)
            if x<=s0 or y>=se: ready.append(j)
        if defer == "all" or (defer == "pass1" and p == 1):
            nr=[j for j in ready if not far[j]]
            if nr: ready=nr
        for j in ready: pend[j]=False
    return p
MODES=(False, "pass1", "all")
tot={d:0 for d in MODES}; rounds=0; wave={d:0 for d in MODES}
for b in blocks:
    sq=seqs(o.compress(bytes(b))); base=0; op=0; k=0; rows=[]
    while k<len(sq):
        if op-base>H-ROOM: base=(op-KEEP)&~15
        rnd=[]
        for (m,off,ml) in sq[k:k+16]:
            if m+ml>base+H: break
            rnd.append((m,off,ml))
        if not rnd: rnd=[sq[k]]
        for d in MODES: tot[d]+=passes(rnd, base, d)
        rows.append(tuple(passes(rnd, base, d) for d in MODES))
        rounds+=1; k+=len(rnd); op=rnd[-1][0]+rnd[-1][2]
    # waves: 4 rows of different blocks run together; approximate with 4 consecutive rounds of this block
    for i in range(0,len(rows)-3,4):
        for di,d in enumerate(MODES): wave[d]+=max(r[di] for r in rows[i:i+4])
for d in MODES:
    print(f"far copies deferred: {d}: passes per row-round {tot[d]/rounds:.3f}, max over 4 rows {wave[d]/(rounds/4):.3f} ({rounds} rounds)")
