#!/usr/bin/env python3
"""Model check of the data-parallel dictionary mode (smallz4_amd/csrc/sz4_dict.hip)
against the in-order replay (k_dict_matches), in pure Python at small block sizes (multiples of 65536 keep
the dictionary's 65535 mod 65536 alignment): match arrays and final chain tables must be identical.
Diagnostic, CPU only: python tools/dict_model.py (about a minute)."""
import sys, random
sys.path.insert(0, __import__('os').path.dirname(__import__('os').path.dirname(__import__('os').path.abspath(__file__))))
from smallz4_amd import synth
W = 65535
SAME = 19 + 255 * 256  # MaxSameLetter
def h32(f): return ((f * 48271) & 0xFFFFFFFF) >> 12
def lcp(d, x, y, cap):
    """common prefix of d[x:] and d[y:], at most cap (findLongestMatch's phase 2 byte loops)"""
    if cap <= 0: return 0
    if d[x:x + cap] == d[y:y + cap]: return cap
    lo, hi = 0, cap  # d[x:x+lo] == d[y:y+lo], d[x:x+hi] != d[y:y+hi]
    while hi - lo > 1:
        m = (lo + hi) // 2
        if d[x:x + m] == d[y:y + m]: lo = m
        else: hi = m
    return lo
def ld4(d, p): return int.from_bytes(d[p:p+4].ljust(4, b'\0'), 'little')

def serial(data, blocks, dictBack, maxChain):
    last = {}; prevH = [0]*65536; prevX = [0]*65536
    mlen = {}; mdist = {}; low = 0; withDict = True
    for (start, end) in blocks:
        size = end - start; stop = end - 5
        back = -dictBack if withDict else -12
        i = back
        while i + 12 <= size:
            pos = start + i
            # self-matching (smallz4.h:631-643): copy the predecessor's long distance-1 match, no insertion
            if i > 0 and data[pos] == data[pos - 1] and mdist.get(pos - 1) == 1 and mlen[pos - 1] > SAME:
                mlen[pos] = mlen[pos - 1] - 1; mdist[pos] = 1
                i += 1
                continue
            slot = i & W
            four = ld4(data, pos); h = h32(four)
            cand = last.get(h); last[h] = pos
            linked = False
            if cand is None or pos - cand > W:
                prevH[slot] = 0; prevX[slot] = 0
            else:
                dist = pos - cand; prevH[slot] = dist; ok = True
                while True:
                    if cand < low: ok = False; break
                    seen = ld4(data, cand)
                    if seen == four: break
                    if h32(seen) != h: ok = False; break
                    step = prevH[cand & W]
                    if step == 0: ok = False; break
                    dist += step
                    if dist > W: ok = False; break
                    cand -= step
                    if cand < low: ok = False; break
                prevX[slot] = dist if ok else 0
                linked = ok and dist != 0
            if linked and i >= 0:
                bestLen, bestDist, steps = 1, 0, maxChain
                hop = prevX[pos & W]; bd = 0; room = stop - pos
                while hop:
                    bd += hop
                    if bd > W: break
                    hop = prevX[(pos - bd) & W]
                    need = bestLen + 1
                    if need > room: break
                    c = pos - bd
                    lo = need - 4
                    while lo > 0 and ld4(data, pos+lo) == ld4(data, c+lo): lo -= 4
                    if lo > 0: continue
                    hi = need + lcp(data, pos + need, c + need, room - need)
                    bestLen, bestDist = hi, bd
                    steps -= 1
                    if steps == 0: break
                mlen[pos] = bestLen; mdist[pos] = bestDist
            i += 1
        withDict = False
        if end - low > W: low = end - W
    return mlen, mdist, prevH, prevX

def parallel(data, blocks, dictBack, maxChain, X=None):
    """One round of the data-parallel algorithm under an assumed set of same-letter shortcut positions
    X (position -> inherited match length; those positions are neither inserted nor searched)."""
    X = X or {}
    nb = len(blocks); cont = 0
    def back(b): return -dictBack if (b == 0 and not cont) else -12
    def dup(b): return b != 0 or cont
    def own_lo(b): return blocks[b][0] + (-11 if dup(b) else back(b))
    def own_hi(b): return blocks[b][1] - 12
    def lowb(b): return 0 if b == 0 else max(0, blocks[b-1][1] - W)
    ph = {}; pe = {}; last = {}
    p0 = own_lo(0)
    for b in range(nb):
        lo, hi = own_lo(b), own_hi(b)
        if hi < lo: continue
        # a block's own insertions suffice: an earlier one is found through the hash table `last`
        keys = sorted((h32(ld4(data, p)), p) for p in range(lo, hi + 1) if p not in X)
        for j, (h, p) in enumerate(keys):
            if p < lo: continue
            d = None
            if j > 0 and keys[j-1][0] == h: d = p - keys[j-1][1]
            else:
                q = last.get(h)
                if q is not None and q < p: d = p - q
            ph[p] = d if d is not None and d <= W else 0
        for j, (h, p) in enumerate(keys):
            if p >= lo and (j + 1 == len(keys) or keys[j+1][0] != h): last[h] = p
    def read_slot(tab, s, b, it):
        # the latest insertion at or before step it whose block-relative index is s mod 65536; shortcut
        # positions were never inserted, so their slot keeps the value of 65536 indices earlier
        start = blocks[b][0]
        iw = it - ((it - s) & W)
        while iw >= back(b) and start + iw in X: iw -= 65536
        if iw >= back(b):
            if iw == -12 and dup(b): return 0
            return tab[start + iw]
        for bb in range(b - 1, -1, -1):
            st, en = blocks[bb]; hi = en - st - 12
            iw = hi - ((hi - s) & W)
            while iw >= back(bb) and st + iw in X: iw -= 65536
            if iw >= back(bb):
                if iw == -12 and dup(bb): return 0
                return tab[st + iw]
        return 0
    for b in range(nb):
        start = blocks[b][0]; low = lowb(b)
        for p in range(own_lo(b), own_hi(b) + 1):
            it = p - start; first = ph.get(p, 0) if p not in X else 0; exact = 0
            if first:
                four = ld4(data, p); h = h32(four); cand = p - first; dist = first; ok = True
                while True:
                    if cand < low: ok = False; break
                    seen = ld4(data, cand)
                    if seen == four: break
                    if h32(seen) != h: ok = False; break
                    step = read_slot(ph, cand & W, b, it)
                    if not step: ok = False; break
                    dist += step
                    if dist > W: ok = False; break
                    cand -= step
                exact = dist if ok else 0
            pe[p] = exact
    mlen = {}; mdist = {}
    for b in range(nb):
        start, end = blocks[b]; size = end - start; stop = end - 5
        for i in range(0, size - 12 + 1):
            pos = start + i
            if pos in X:
                mlen[pos] = X[pos]; mdist[pos] = 1
                continue
            if pe[pos] == 0: continue
            bestLen, bestDist, steps = 1, 0, maxChain
            hop = read_slot(pe, pos & W, b, i); bd = 0; room = stop - pos
            while hop:
                bd += hop
                if bd > W: break
                hop = read_slot(pe, (pos - bd) & W, b, i)
                need = bestLen + 1
                if need > room: break
                c = pos - bd
                lo = need - 4
                while lo > 0 and ld4(data, pos+lo) == ld4(data, c+lo): lo -= 4
                if lo > 0: continue
                hi = need + lcp(data, pos + need, c + need, room - need)
                bestLen, bestDist = hi, bd
                steps -= 1
                if steps == 0: break
            mlen[pos] = bestLen; mdist[pos] = bestDist
    b = nb - 1; it = blocks[b][1] - blocks[b][0] - 12
    cH = [read_slot(ph, s, b, it) for s in range(65536)]
    cX = [read_slot(pe, s, b, it) for s in range(65536)]
    return mlen, mdist, cH, cX


def observed_shortcuts(blocks, X, mlen, mdist):
    """The shortcut positions the reference's loop would take given this round's results: a searched
    position a (not assumed skipped) with a distance-1 match longer than MaxSameLetter starts
    a + 1 .. a + La - MaxSameLetter (smallz4.h:631-643); positions assumed skipped but not confirmed have
    no search result, so they start nothing (the next round searches them)."""
    Y = {}
    for (start, end) in blocks:
        size = end - start
        i = 1
        while i + 12 <= size:
            a = start + i - 1
            if a in Y: L = Y[a]
            elif a in X: L = 0
            else: L = mlen.get(a, 0) if mdist.get(a) == 1 else 0
            if L > SAME:
                Y[a + 1] = L - 1
            i += 1
    return Y


def parallel_sc(data, blocks, dictBack, maxChain, rounds=None):
    """Rounds of parallel() until the assumed shortcut positions are the ones the results imply; every
    round settles at least the prefix up to its first disagreement (k_dict_sc_check)."""
    X = {}
    for r in range(100):
        res = parallel(data, blocks, dictBack, maxChain, X)
        Y = observed_shortcuts(blocks, X, res[0], res[1])
        if Y == X:
            if rounds is not None: rounds.append(r + 1)
            return res
        X = Y
    raise RuntimeError("shortcut positions did not settle")


# ---- greedy/lazy bookkeeping (k_dict_lz_walk / _fix / _clear): the speculative per-sub-segment walk
# against the reference's serial skip loop (smallz4.h:726-744), on linked flags and lengths
def lz_serial(linked, L):
    kept=set(); skip=0; lazy=False
    for q in range(len(L)):
        if not linked[q]: continue
        if skip>0:
            skip-=1
            if not lazy: continue
            lazy=False
        kept.add(q)
        if L[q]!=1:
            lazy = skip==0; skip=L[q]
    return kept
def lz_next(linked, pos, need):
    while pos < len(linked):
        if linked[pos]:
            if need==0: return pos
            need-=1
        pos+=1
    return 10**9
def lz_step(linked,L,q,md,carry):
    if md==0:
        if L[q]!=1: carry=L[q]-1; md=1
        return lz_next(linked,q+1,0),md,carry
    return lz_next(linked,q+1,L[q] if L[q]!=1 else carry),0,carry
def lz_spec(linked, L, SEG=64):
    n=len(L); segs=[]
    for a in range(0,n,SEG):
        an=min(a+SEG,n); fresh=set(); kept=set(); md=0; carry=0
        q=lz_next(linked,a,0)
        while q<an:
            kept.add(q)
            if md==0: fresh.add(q)
            q,md,carry=lz_step(linked,L,q,md,carry)
        segs.append([fresh,kept,(q,md,carry)])
    ex=segs[0][2]
    for k in range(1,len(segs)):
        a=k*SEG; an=min(a+SEG,n); fresh,kept,sp=segs[k]
        q,md,carry=ex
        if q>=an: segs[k][1]=set(); continue
        merged = md==0 and q in fresh; rep=set()
        if not merged:
            while q<an:
                if md==0 and q in fresh: merged=True; break
                rep.add(q); q,md,carry=lz_step(linked,L,q,md,carry)
        frm = q if merged else an
        segs[k][1]=rep|{x for x in kept if x>=frm}
        ex = sp if merged else (q,md,carry)
    out=set()
    for s in segs: out|=s[1]
    return out


def make_case(bs, n, dl, seed):
    dic = synth.enwik8_like(dl, seed=seed)
    body = synth.enwik8_like(n, seed=seed + 10)
    dictBack = min(dl, W)
    prefix = (b'\0' * W + dic)[-W:]
    data = prefix + body + b'\0' * 16
    blocks = []
    s = W
    while s < W + n:
        blocks.append((s, min(s + bs, W + n)))
        s += bs
    return data, blocks, dictBack


if __name__ == "__main__":
    import random
    random.seed(1)
    for t in range(3000):
        n = random.randint(1, 700)
        p = random.random()
        linked = [random.random() < p for _ in range(n)]
        L = [random.choice([1, 1, 2, 3, 4, 5, 6, 9, 20, 100]) for _ in range(n)]
        assert lz_serial(linked, L) == lz_spec(linked, L), (t, n)
    print("lazy walk: 3000 random cases equal")
    for (bs, n, dl, chain, seed) in [(131072, 300000, 20000, 65535, 1), (65536 * 2, 280000, 65535, 5, 2),
                                     (65536 * 3, 200000, 3000, 65535, 3)]:
        data, blocks, dictBack = make_case(bs, n, dl, seed)
        a = serial(data, blocks, dictBack, chain)
        b = parallel(data, blocks, dictBack, chain)
        print(bs, n, dl, chain, 'mlen', a[0] == b[0], 'mdist', a[1] == b[1], 'prevH', a[2] == b[2], 'prevX', a[3] == b[3],
              len(a[0]))
