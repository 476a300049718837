"""Where k_find_sorted's below-chunk broadcast steps go: positions of 8 MB of the
benchmark text in 64 KiB blocks sorted by (first 4 bytes, position) as the finder sorts them, cut into
64-slot chunks; for every chunk, the candidates of the group that began before it are the broadcast
steps, weighted by how many of the chunk's lanes belong to that group.  CPU only.

    python tools/group_stats.py
"""
import sys, numpy as np
sys.path.insert(0, __import__('os').path.dirname(__import__('os').path.dirname(__import__('os').path.abspath(__file__))))
from smallz4_amd import synth
data = np.frombuffer(synth.enwik8_like(8 << 20, seed=1), dtype=np.uint8)
B=65536
tot_steps=0; hist=np.zeros(65); shift_steps=0
for o in range(0, len(data)-B+1, B):
    blk=data[o:o+B].astype(np.uint32)
    n=B-3
    key=blk[:n] | (blk[1:n+1]<<8) | (blk[2:n+2]<<16) | (blk[3:n+3]<<24)
    order=np.lexsort((np.arange(n), key))
    sk=key[order]
    # group start index for each sorted element
    newg=np.ones(n,bool); newg[1:]=sk[1:]!=sk[:-1]
    gstart=np.maximum.accumulate(np.where(newg, np.arange(n), 0))
    for c0 in range(0, n, 64):
        c1=min(c0+64,n)
        gs0=gstart[c0]
        below=c0-gs0            # candidates of the first group below the chunk
        if below>0:
            g=int(np.sum(gstart[c0:c1]==gs0))
            tot_steps+=below; hist[g]+=below
print('broadcast steps per position %.3f'%(tot_steps/ (len(data))))
cum=np.cumsum(hist)/hist.sum()
for g in (4,8,16,32,48,63,64): print(g, '%.3f'%cum[g])
