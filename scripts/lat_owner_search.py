"""Block -> wave ownership of the latency kernel (csrc/chol_lat.hip LAT_MAP).

chol_lat_kernel gives each (pulsar, sample) one 4-wave workgroup; block (i, j)
of the upper block triangle lives in the registers of wave own[i][j].  Panel
bb costs (measured stamps, profiles/r03f/lat_stamps_b1.log, fitted below)
    M * max_w rowV_w  +  max_w (M * trail_w + [w owns (bb+1, bb+1)] (4 M + F))  +  ov
with rowV_w / trail_w the MFMAs wave w issues for V = E^T A of block row bb
and for the trailing updates, F the diagonal-block factorisation that only the
owner of (bb+1, bb+1) runs (lookahead), M ~ 130 cycles per MFMA with its LDS
operand traffic.  The round-3 map (i + j) mod 4 gives the next diagonal's
owner a full share of the trailing work (fit: 40.4 k cycles for the 7
panels vs 40.6 k measured).  This anneals a map per NB that unloads that
owner and prints the C++ table.

    python scripts/lat_owner_search.py
"""
import math
import random

M, F, OV = 130.0, 2500.0, 600.0
UNEXT = 0.0     # --unext: cycles per panel when U (bb, bb+1) is formed by another wave than the lookahead owner


def cost(nb, own):
    tot = 0.0
    for bb in range(nb - 1):
        rv = [0] * 4
        tr = [0] * 4
        for j in range(bb + 1, nb):
            rv[own[(bb, j)]] += 4
        for i in range(bb + 1, nb):
            for j in range(i, nb):
                if (i, j) != (bb + 1, bb + 1):
                    tr[own[(i, j)]] += 4
        o = own[(bb + 1, bb + 1)]
        tot += M * max(rv) + max(tr[w] * M + ((4 * M + F) if w == o else 0.0) for w in range(4)) + OV
        if own[(bb, bb + 1)] != o:
            tot += UNEXT
    return tot


def search(nb, seed=1, restarts=24, iters=20000):
    blocks = [(i, j) for i in range(nb) for j in range(i, nb)]
    rng = random.Random(seed)
    best = None
    for _ in range(restarts):
        own = {b: rng.randrange(4) for b in blocks}
        c = cost(nb, own)
        t = 2000.0
        for _ in range(iters):
            b = rng.choice(blocks)
            old = own[b]
            own[b] = rng.randrange(4)
            c2 = cost(nb, own)
            if c2 <= c or rng.random() < math.exp(-(c2 - c) / t):
                c = c2
            else:
                own[b] = old
            t *= 0.9995
        if best is None or c < best[0]:
            best = (c, dict(own))
    return best


def main():
    import argparse
    global UNEXT
    ap = argparse.ArgumentParser()
    ap.add_argument("--unext", type=float, default=0.0,
                    help="penalty (cycles) per panel whose U (bb, bb+1) another wave than the lookahead owner forms "
                         "(its LDS publish / wait; round 4 A/B)")
    ap.add_argument("--nb", type=int, default=0, help="only this NB")
    args = ap.parse_args()
    UNEXT = args.unext
    rows = []
    for nb in range(1, 9):
        if args.nb and nb != args.nb:
            rows.append([[0] * 8 for _ in range(8)])
            continue
        base = {(i, j): (i + j) & 3 for i in range(nb) for j in range(i, nb)}
        if nb == 1:
            c, own = cost(nb, base), base
        else:
            c, own = search(nb)
        print(f"// NB={nb}: model {cost(nb, base):.0f} -> {c:.0f} cycles")
        rows.append([[own.get((i, j), 0) for j in range(8)] for i in range(8)])
    print("constexpr unsigned char LAT_MAP[9][8][8] = {{},")
    for nb, t in enumerate(rows, 1):
        print("  {" + ", ".join("{" + ",".join(str(v) for v in r) + "}" for r in t) + "},")
    print("};")


if __name__ == "__main__":
    main()
