"""Dev tool (CPU): the rows parse kernel's wave schedule, one lane per block --
fast-loop iterations (MA: the go-lane threshold, UNR: steps per exit test),
general steps and ring loads per 64 sequences, and the lane use of the fast
steps, with a VALU cost model (fast step ~32.5 new / ~65 old, general step
~168).  DESIGN §3.1 "the parse kernel".  env: N, MA, UNR."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "python-lz4_amd")); sys.path.insert(0, ROOT)
from lz4 import _synth
from oracle.oracle import Oracle
n=int(os.environ.get("N","128"))
blocks=_synth.blocks(n,"silesia",seed=2026); o=Oracle()
def seqs(c, oend=65536):
    i=0; op=0; out=[]
    iend=len(c)
    while i<len(c):
        ip=i; t=c[i]; i+=1; L=t>>4
        if L==15:
            while True:
                x=c[i]; i+=1; L+=x
                if x!=255: break
        i+=L
        if i>=len(c): break
        off=c[i]|(c[i+1]<<8); i+=2; M=t&15; mx=0
        if M==15:
            while True:
                x=c[i]; i+=1; M+=x; mx+=1
                if x!=255: break
        M+=4
        lit0=t>>4
        fast = lit0<=12 and mx<=1 and (M-4-15)<255 if (t&15)==15 else lit0<=12
        fast = fast and ip <= iend-20 and op+L+M < oend-64
        out.append((ip, i-ip, fast))   # start, adv, fast
        op+=L+M
    return out
S=[seqs(o.compress(bytes(b))) for b in blocks]
KPW=128; MINACT=int(os.environ.get("MA","40")); UNR=int(os.environ.get("UNR","2"))
def wave(blks):
    # lanes: dict per lane
    L=[dict(live=True, q=0, ip=0, wb=-4*KPW, pfv=False, need=True, stall=False, k=0, kf=0, sq=b) for b in blks]
    fl=0; gs=0; loads=0; steps_active=0; nseq=sum(len(b) for b in blks)
    while any(l['live'] for l in L):
        gs+=1
        for l in L:
            if not l['live']: continue
            if l['pfv'] and l['ip']>=l['wb']+64: l['wb']+=64; l['pfv']=False
        for l in L:
            if l['live'] and l['stall'] and not l['need'] and l['ip']+16>l['wb']+KPW: l['need']=True
            l['stall']=False
        for l in L:
            if l['live'] and l['need']:
                l['need']=False
                if l['ip']+32>l['wb']+KPW: l['wb']=l['ip']&~63; l['pfv']=False; loads+=1
                if l['q']>=len(l['sq']): l['live']=False; continue
                ip,adv,f=l['sq'][l['q']]; l['q']+=1; l['ip']=ip+adv; l['k']+=1
        for l in L:
            if l['live'] and l['k']-l['kf']>=16: l['kf']+=16
        for l in L:
            if l['live'] and not l['pfv']: l['pfv']=True
        thr=min(MINACT, sum(l['live'] for l in L))
        while True:
            for u in range(UNR):
                for l in L:
                    go=l['live'] and not l['need'] and not l['stall']
                    if not go: continue
                    steps_active+=1
                    if l['q']>=len(l['sq']): l['need']=True; continue
                    ip,adv,f=l['sq'][l['q']]
                    inw= l['ip']+16<=l['wb']+KPW; room=l['k']-l['kf']<31
                    if inw and room and f:
                        l['ip']+=adv; l['q']+=1; l['k']+=1
                    else:
                        l['stall']=True
                        if inw and room and not f: l['need']=True
            fl+=1
            if sum(l['live'] and not l['need'] and not l['stall'] for l in L) < max(thr,1): break
    return fl, gs, loads, nseq, steps_active
tot=[0]*5
for w in range(0, n, 64):
    r=wave(S[w:w+64])
    tot=[a+b for a,b in zip(tot,r)]
fl,gs,loads,nseq,sa=tot
print(f"MA {MINACT} cost new {(fl*UNR*32.5+gs*168)*64/nseq:.1f} old {(fl*UNR*65+gs*168)*64/nseq:.1f} UNR {UNR}: fast iters {fl}, general steps {gs}, ring loads {loads}, seqs {nseq}; per 64 seqs: fast iters {fl*64/nseq:.2f}, general {gs*64/nseq:.3f}; lane util in fast steps {sa/(fl*UNR*64):.2f}")
