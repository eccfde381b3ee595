#!/usr/bin/env python3
"""Bank-conflict model of the k_demod_fast LDS transposes (design aid).

Replays, per SF, every ds_read_b64 / ds_write_b64 address pattern of the pass-1
write-back, the LDS passes (read, and write-back between passes) and the natural-order
write (KEEP), for a candidate LDS address map, and reports the average conflict degree
per access (1.0 = conflict-free).  Banking per MI355X_MICROARCH.md section LDS:
ds_read_b64 = 2 groups of 32 lanes, bank (a/4) mod 64; ds_write_b64 = 4 groups of 16
contiguous lanes, bank (a/4) mod 32; identical dwords broadcast.
"""
import itertools
import sys


def radices(N):
    r, n = [], N
    while n > 1:
        p = 4 if n % 4 == 0 else 2
        r.append(p)
        n //= p
    return r


def leaf_rev(N):
    rad = radices(N)
    rev = [0] * N

    def rec(stage, out_pos, in_idx, fstride, length):
        p = rad[stage]
        m = length // p
        if m == 1:
            for j in range(p):
                rev[in_idx + j * fstride] = out_pos + j
            return
        for q in range(p):
            rec(stage + 1, out_pos + q * m, in_idx + q * fstride, fstride * p, m)

    rec(0, 0, 0, 1, N)
    return rev


def geo(SF):
    N = 1 << SF
    small = SF <= 5
    P = N if small else 16
    T = N // P
    R1 = N if small else (8 if SF & 1 else 16)
    LOGR1 = {2: 2, 3: 3, 4: 4, 5: 5}.get(SF, 3 if SF & 1 else 4) if small else (3 if SF & 1 else 4)
    X = N // R1
    RA = 16 if X >= 16 else X
    RB = X // 16 if X > 16 else 1
    npass = 1 + (X > 1) + (X > 16)
    return dict(N=N, P=P, T=T, R1=R1, LOGR1=LOGR1, G1=P // R1, RA=RA, RB=RB, MA_A=R1, MA_B=R1 * RA,
                NPASS=npass, SPW=256 // T)


def patterns(SF):
    """Yield lists of (row g, position p) per instruction for one 64-lane wave (wave 0
    and, for T > 64, every wave)."""
    G = geo(SF)
    N, P, T, R1 = G["N"], G["P"], G["T"], G["R1"]
    rev = leaf_rev(N)
    waves = range(max(1, T // 64)) if T > 64 else [0]
    pats = []
    for w in waves:
        lanes = [(64 * w + t) for t in range(64)]
        gl = [(tid // T, tid % T) for tid in lanes]
        # pass-1 write-back
        for h in range(G["G1"]):
            for u in range(R1):
                pats.append(("w1", [(g, (rev[l + T * h] >> G["LOGR1"]) * R1 + u) for g, l in gl]))
        passes = []
        if G["NPASS"] >= 2:
            passes.append((G["RA"], G["MA_A"]))
        if G["NPASS"] == 3:
            passes.append((G["RB"], G["MA_B"]))
        for (R, MA) in passes:
            NG = P // R
            for gg in range(NG):
                for u in range(R):
                    pos = [(g, ((l + T * gg) // MA) * MA * R + (l + T * gg) % MA + MA * u) for g, l in gl]
                    pats.append((f"r{R}x{MA}", pos))
                    if (R, MA) != passes[-1]:
                        pats.append((f"w{R}x{MA}", pos))
        if G["NPASS"] >= 2:
            RL, ML = passes[-1]
            for gg in range(P // RL):
                for u in range(RL):
                    pats.append(("keep", [(g, l + T * gg + ML * u) for g, l in gl]))
    return pats


def degree(slots, write):
    """slots: complex-element indices of 64 lanes -> mean conflict degree over groups."""
    gsz, nb = (16, 32) if write else (32, 64)
    tot = 0
    groups = [slots[i:i + gsz] for i in range(0, 64, gsz)]
    for grp in groups:
        banks = {}
        for s in set(grp):
            for d in (2 * s, 2 * s + 1):
                banks.setdefault(d % nb, set()).add(d)
        tot += max(len(v) for v in banks.values())
    return tot / len(groups)


def evaluate(SF, addr, rowc):
    res = {}
    for name, pat in patterns(SF):
        slots = [g * rowc + addr(p) for g, p in pat]
        res.setdefault(name, []).append(degree(slots, name[0] in "wk"))
    return {k: sum(v) / len(v) for k, v in res.items()}


if __name__ == "__main__":
    for SF in range(6, 13):
        G = geo(SF)
        lg = G["LOGR1"]
        cur_rowc = G["N"] + (G["N"] >> lg)
        while cur_rowc % 32 != 8:
            cur_rowc += 1
        cur = evaluate(SF, lambda p: p + (p >> lg), cur_rowc)
        print(SF, "current", {k: round(v, 2) for k, v in cur.items()}, "rowc", cur_rowc)
