#!/usr/bin/env python3
"""Search an ADDITIVE padding map for the k_demod_fast LDS rows (design aid).

slot(g, p) = g*rowc + p + sum_{i>=4} bit_i(p) * w_i,  rowc = N + sum w + pad, with
w_i = sum_{j<i} w_j + d_i, 0 <= d_i < 32: the offset of each 16-position block is then
monotone in the block index, so blocks never overlap and the map is injective.
Being linear over the bits of p, the map splits into a per-lane part plus a compile-time
part for every access pattern (positions = lane base | unrolled offset, disjoint bits),
so the offsets fold into the ds_read/ds_write immediate: no VALU per access.
"""
import random
import sys

import numpy as np

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from lds_sim import geo, patterns  # noqa: E402


def build(SF):
    G = geo(SF)
    pats = patterns(SF)
    arr = np.array([[p for g, p in pat] for _, pat in pats], np.int64)
    rows = np.array([[g for g, p in pat] for _, pat in pats], np.int64)
    wr = np.array([name[0] in "wk" for name, _ in pats])
    return G, arr, rows, wr


def slots(G, arr, rows, w, pad):
    extra = np.zeros_like(arr)
    for i, wi in enumerate(w):
        extra += ((arr >> (4 + i)) & 1) * wi
    rowc = G["N"] + sum(w) + pad
    return rows * rowc + arr + extra


def cost(G, arr, rows, wr, w, pad):
    s = slots(G, arr, rows, w, pad)
    tot, n = 0.0, 0
    for is_w, gsz, nb in ((True, 16, 32), (False, 32, 64)):
        sel = s[wr == is_w]
        for inst in sel:
            for grp in inst.reshape(64 // gsz, gsz):
                u = np.unique(grp)
                b = np.bincount((2 * u) % nb, minlength=nb) + np.bincount((2 * u + 1) % nb, minlength=nb)
                tot += b.max()
                n += 1
    return tot / max(n, 1)


def weights(d):
    w, acc = [], 0
    for di in d:
        w.append(acc + di)
        acc += w[-1]
    return w


def search(SF, iters=3000, seed=1):
    G, arr, rows, wr = build(SF)
    nb = SF - 4
    rnd = random.Random(seed)
    cur_d = [1] + [0] * (nb - 1)  # w = 1, 1, 2, 4, ... (the p + p/16 map)
    cur_pad = 0
    cur_w = weights(cur_d)
    cur = cost(G, arr, rows, wr, cur_w, cur_pad)
    best = (cur, list(cur_w), cur_pad)
    for it in range(iters):
        d, pad = list(cur_d), cur_pad
        if G["T"] < 64 and rnd.random() < 0.25:
            pad = rnd.randrange(0, 32)
        else:
            d[rnd.randrange(nb)] = rnd.randrange(32) if rnd.random() < 0.5 else rnd.randrange(4)
        w = weights(d)
        c = cost(G, arr, rows, wr, w, pad)
        # prefer smaller rows on ties
        key = (c, sum(w) + pad)
        if key <= (cur, sum(cur_w) + cur_pad) or rnd.random() < 0.02:
            cur, cur_d, cur_w, cur_pad = c, d, w, pad
            if key < (best[0], sum(best[1]) + best[2]):
                best = (c, list(w), pad)
        if best[0] <= 1.0 and it > 300:
            break
    return best, G


if __name__ == "__main__":
    for SF in [int(a) for a in sys.argv[1:]] or range(6, 13):
        (c, w, pad), G = search(SF)
        print(f"SF{SF}: mean degree {c:.3f}  w={w} pad={pad} rowc={G['N'] + sum(w) + pad}", flush=True)
