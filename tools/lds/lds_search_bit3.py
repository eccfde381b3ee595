#!/usr/bin/env python3
"""Exhaustive search of additive LDS maps WITH a bit-3 weight (design aid): slot(p) = p +
sum_{i>=3} bit_i(p) W_i over small weights and row pads, scored by the mean conflict degree
of every access pattern of tools/lds/lds_sim.py (pass-1 write-back as ds_write_b64, LDS-pass
reads as ds_read_b64 and as ds_read2_b64, natural-order write); only injective maps.  The
SF7 map of lora_demod_fast.hip (W3 = 1, W = {1, 2, 4}, rowc 136) is its first result.
usage: lds_search_bit3.py [SF]   (SF 7: 9^4 maps, seconds; larger SF grow as 9^(SF-3))"""
import itertools, sys
sys.path.insert(0, __file__.rsplit('/', 1)[0])
from lds_sim import geo, patterns

def deg(slots, gsz, nb):
    tot = 0
    for i in range(0, 64, gsz):
        grp = slots[i:i+gsz]
        banks = {}
        for s in set(grp):
            for d in (2*s, 2*s+1):
                banks.setdefault(d % nb, set()).add(d)
        tot += max(len(v) for v in banks.values())
    return tot / (64 // gsz)

SF = int(sys.argv[1]) if len(sys.argv) > 1 else 7
G = geo(SF); N = G['N']
pats = patterns(SF)
nbits = SF - 3
best = []
for W in itertools.product(range(0, 9), repeat=nbits):
    def slot(p):
        return p + sum(((p >> (3 + i)) & 1) * W[i] for i in range(nbits))
    sl = [slot(p) for p in range(N)]
    if len(set(sl)) != N: continue
    # linearity over disjoint bits holds by construction
    width = max(sl) + 1
    for pad in range(0, 12):
        rowc = width + pad
        res = {}
        for name, pat in pats:
            s = [g * rowc + slot(p) for g, p in pat]
            if name[0] == 'w':
                res.setdefault('w', []).append(deg(s, 16, 32))
            elif name[0] == 'r':
                res.setdefault('r64', []).append(deg(s, 32, 64))
                res.setdefault('r2', []).append(deg(s, 16, 32))
            else:
                res.setdefault('keep', []).append(deg(s, 16, 32))
        r = {k: sum(v)/len(v) for k, v in res.items()}
        key = (r['w'] + r['r2'] + r['r64'], rowc)
        best.append((key, W, pad, rowc, r))
best.sort(key=lambda x: x[0])
for b in best[:8]: print(b)
