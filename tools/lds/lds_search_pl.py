#!/usr/bin/env python3
"""SF7 LDS slot-map search for k_spec_demod's whole-line pass (PL, round 6): every access
pattern of the SF7 transforms at once - the PL pass-1 write-back (lane l writes residues
(2l + h - d) mod 16, every line offset d), the role layout's write-back (residues l, l + 8:
sync blocks, exact kernels), the pass-A reads and the natural-order write (KEEP) - under
the MI355X banking rules of lds_sim.py, over additive maps slot = p + bit3 W3 + sum
bit_{4+i} W[i] (superincreasing: injective) with rows of at most 150 slots (four
workgroups per CU).  Prints the best maps by total mean conflict degree (1.0 = none)."""
import itertools

import numpy as np

import lds_sim as L

SF = 7
G = L.geo(SF)
N, T, R1, P = G["N"], G["T"], G["R1"], G["P"]
rev = L.leaf_rev(N)
lanes = np.arange(64)
g, l = lanes // T, lanes % T
pats = []  # (name, rows, positions, write)
for h in range(2):
    for u in range(R1):
        pats.append(("w_role", g, np.array([(rev[x + T * h] >> 3) * R1 + u for x in l]), True))
for d in range(16):
    for h in range(2):
        for u in range(R1):
            pats.append(("w_pl", g, np.array([(rev[(2 * x + h - d) % 16] >> 3) * R1 + u for x in l]), True))
RA, MA = G["RA"], G["MA_A"]
for gg in range(P // RA):
    for u in range(RA):
        gi = l + T * gg
        pats.append(("r_A", g, (gi // MA) * MA * RA + gi % MA + MA * u, False))
        pats.append(("keep", g, gi + MA * u, True))
names = sorted(set(p[0] for p in pats))


def degrees(slots, write):
    gsz, nb = (16, 32) if write else (32, 64)
    s = slots.reshape(-1, gsz)
    out = []
    for grp in s:
        u = np.unique(grp)
        d = np.concatenate([2 * u, 2 * u + 1])
        cnt = np.bincount(d % nb, minlength=nb)
        out.append(cnt.max())
    return np.mean(out)


def evaluate(W3, W, pad):
    rowc = N + W3 + sum(W) + pad
    res = {n: [] for n in names}
    for name, rows, pos, wr in pats:
        slot = pos + ((pos >> 3) & 1) * W3 + sum(((pos >> (4 + i)) & 1) * W[i] for i in range(3))
        res[name].append(degrees(rows * rowc + slot, wr))
    return {n: float(np.mean(v)) for n, v in res.items()}, rowc


if __name__ == "__main__":
    cur, rc = evaluate(1, [1, 2, 4], 0)
    print("current", cur, "rowc", rc, flush=True)
    best = []
    for W3 in range(0, 3):
        for w0 in range(W3, 9):
            for w1 in range(W3 + w0, 13):
                for w2 in range(W3 + w0 + w1, 23):
                    for pad in range(0, 4):
                        if N + W3 + w0 + w1 + w2 + pad > 150:
                            continue
                        r, rowc = evaluate(W3, [w0, w1, w2], pad)
                        best.append((sum(r.values()), rowc, W3, (w0, w1, w2), pad, r))
    best.sort(key=lambda x: (x[0], x[1]))
    for b in best[:10]:
        print(b)
