#!/usr/bin/env python3
"""Model of the Bloom blocks k_nb_build touches per wave instruction (random
sequence, k = 31, minimizer 15-mers of a random order): one window per lane
and one substituted offset j per step (k_nb_build pass 0) vs the windows'
(window, substituted position) pairs in position order, 64 per step
(k_nb_first).  Distinct blocks ~ memory requests.

    python scripts/nb_model.py
"""
import numpy as np

rng=np.random.default_rng(1)
k=31; m=15; L=64*40+k
seq=rng.integers(0,4,L)
def order(x): # x: int code of 15-mer
    return (x*0x9E3779B1 + 12345) & 0xFFFFFFFF
def minim(s):
    best=None
    for i in range(len(s)-m+1):
        v=0
        for c in s[i:i+m]: v=v*4+int(c)
        o=order(v)
        if best is None or o<best[0]: best=(o,v)
    return best[1]
nb={}  # (t,j,b) -> minimizer
for t in range(64*8):
    w=seq[t:t+k].copy()
    for j in range(k):
        for b in range(3):
            w2=w.copy(); w2[j]=(w[j]+1+b)&3
            nb[(t,j,b)]=minim(w2)
# current: instruction = (tile, j, b), lanes t in tile
cur=[]
for tile in range(8):
    for j in range(k):
        for b in range(3):
            cur.append(len({nb[(tile*64+l,j,b)] for l in range(64)}))
print('current: distinct blocks per instruction avg %.1f, total per tile %.0f'%(np.mean(cur), np.sum(cur)/8))
# p-major: pairs ordered by p then t, 64 per step
new=[]
for tile in range(8):
    pairs=sorted([(t+j,t,j) for t in range(tile*64,tile*64+64) for j in range(k)])
    for s in range(0,len(pairs),64):
        for b in range(3):
            new.append(len({nb[(t,j,b)] for p,t,j in pairs[s:s+64]}))
print('p-major: distinct blocks per instruction avg %.1f, total per tile %.0f'%(np.mean(new), np.sum(new)/8))
