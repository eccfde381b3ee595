#!/usr/bin/env python3
"""SF7 whole-line pass (PL): which 16-byte chunk of a symbol's 128-byte line lane l loads
(chunk pi(l), pi a permutation of 0..7) decides the residues it holds, (2 pi(l) + h - d)
mod 16, hence its pass-1 write-back positions.  Search every pi for the one whose write-back
is conflict-free under the current LdsMap<7> for every line offset d (16-lane groups of two
symbols, 32 banks: ds_write_b64, lds_sim.py's rules)."""
import itertools

import numpy as np

import lds_sim as L

N, T, R1, ROWC = 128, 8, 8, 136
rev = L.leaf_rev(N)
cpos = np.array([rev[r] >> 3 for r in range(16)])


def slot(p):
    return p + ((p >> 3) & 1) * 1 + ((p >> 4) & 1) * 1 + ((p >> 5) & 1) * 2 + ((p >> 6) & 1) * 4


perms = np.array(list(itertools.permutations(range(8))))  # [40320, 8]
lane = np.arange(16)
g, l = lane // T, lane % T
worst = np.zeros(len(perms))
total = np.zeros(len(perms))
for d in range(16):
    for h in range(2):
        r = (2 * perms[:, l] + h - d) % 16  # [P, 16]
        for u in range(R1):
            p = cpos[r] * R1 + u
            s = g * ROWC + slot(p)  # [P, 16]
            dw = np.concatenate([2 * s, 2 * s + 1], axis=1) % 32
            cnt = np.zeros((len(perms), 32), int)
            for k in range(32):
                np.add.at(cnt, (np.arange(len(perms)), dw[:, k]), 1)
            deg = cnt.max(axis=1)
            worst = np.maximum(worst, deg)
            total += deg
idx = np.argsort(total)[:10]
for i in idx:
    print(list(perms[i]), "mean degree", total[i] / (16 * 2 * R1), "worst", worst[i])
