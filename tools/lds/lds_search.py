#!/usr/bin/env python3
"""Search an XOR swizzle for the k_demod_fast LDS rows (design aid, see lds_sim.py).

slot(g, p) = g*N + (p ^ sum_i bit_i(p >> 5) * V[i] ^ sum_j bit_j(g) * W[j])  (5-bit V, W)
Objective: mean conflict degree over every LDS access of one symbol transform.
Prints the best vectors per SF as C++ initialisers.
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


def cost(G, arr, rows, wr, V, W):
    N = G["N"]
    hi = arr >> 5
    x = np.zeros_like(arr)
    for i, v in enumerate(V):
        x ^= ((hi >> i) & 1) * v
    for j, w in enumerate(W):
        x ^= ((rows >> j) & 1) * w
    slot = rows * N + (arr ^ x)
    total = 0.0
    for is_w, gsz, nb in ((True, 16, 32), (False, 32, 64)):
        sel = slot[wr == is_w]
        if sel.size == 0:
            continue
        g = sel.reshape(sel.shape[0], 64 // gsz, gsz)
        d0 = (2 * g) % nb  # each b64 touches banks d0, d0+1; distinct slots -> conflicts
        # degree = max multiplicity of (bank) among distinct dword addresses
        deg = []
        for inst in range(g.shape[0]):
            for grp in range(g.shape[1]):
                s = np.unique(g[inst, grp])
                b = np.bincount((2 * s) % nb, minlength=nb) + np.bincount((2 * s + 1) % nb, minlength=nb)
                deg.append(b.max())
        total += float(np.sum(deg))
    n_groups = int(wr.sum()) * 4 + int((~wr).sum()) * 2
    return total / n_groups


def search(SF, iters=4000, seed=0):
    G, arr, rows, wr = build(SF)
    nv = max(0, SF - 5)
    nw = max(0, (G["SPW"] - 1).bit_length()) if G["T"] < 64 else 0
    rnd = random.Random(seed)
    best_V = [0] * nv
    best_W = [0] * nw
    best = cost(G, arr, rows, wr, best_V, best_W)
    cur_V, cur_W, cur = list(best_V), list(best_W), best
    for it in range(iters):
        V, W = list(cur_V), list(cur_W)
        k = rnd.randrange(nv + nw) if nv + nw else 0
        if nv + nw == 0:
            break
        if k < nv:
            V[k] = rnd.randrange(32)
        else:
            W[k - nv] = rnd.randrange(32)
        c = cost(G, arr, rows, wr, V, W)
        if c <= cur or rnd.random() < 0.02:
            cur_V, cur_W, cur = V, W, c
            if c < best:
                best_V, best_W, best = list(V), list(W), c
        if best <= 1.0:
            break
    return best, best_V, best_W


if __name__ == "__main__":
    for SF in [int(a) for a in sys.argv[1:]] or range(6, 13):
        b, V, W = search(SF)
        print(f"SF{SF}: mean degree {b:.3f}  V={V} W={W}", flush=True)
