#!/usr/bin/env python3
"""Search the v4 transform's middle/output layouts and relayout scratch
positions (fhe-icp_amd/csrc/br_v4.h: LAYS, RC).

A scratch position is p(j) = j + sum_k c_k * bit_{4+k}(j) with superincreasing
c (injective, additive in the lane and slot parts of j). For each relayout
(source layout A written with ds_write_b128, target layout B read with
ds_read_b128) it must be bank-conflict-free on gfx950 (MI355X_MICROARCH.md
§LDS): the 8 lanes of a write group hit 8 distinct 16-B quads mod 8, the 16
lanes of a read group ({0-3,12-15,20-27}, {4-11,16-19,28-31}, +32) 16 distinct
quads mod 16. Layout LA (natural) is fixed; LB holds index bits 3,4,5 in its
slots, LC bits 0,1,2. Prints the smallest-scratch solution.

--lb a,b,c,d,e,f fixes LB's lane bits (the kernel now reaches LB from LA in
registers: slot bits <-> lane bits 3..5, so LB lanes = 0,1,2,6,7,8) and
searches only LC and the LB <-> LC offsets.
"""
import sys
import itertools

BASES = [(0, 0, 0, 0), (1, 2, 4, 8), (0, 1, 2, 4), (1, 1, 2, 4), (2, 4, 8, 16), (0, 2, 4, 8), (1, 2, 4, 7)]


def injective(c):
    return len({j + sum(c[k] * ((j >> (4 + k)) & 1) for k in range(5)) for j in range(512)}) == 512


cands = [b + (c8,) for b in BASES for c8 in range(sum(b), sum(b) + 24) if injective(b + (c8,))]
W = {c: [(1 << k) + (c[k - 4] if k >= 4 else 0) for k in range(9)] for c in cands}


def wok(c, lanes):  # write groups vary lane bits 0..2
    w = W[c]
    return len({(x * w[lanes[0]] + y * w[lanes[1]] + z * w[lanes[2]]) % 8
                for x in (0, 1) for y in (0, 1) for z in (0, 1)}) == 8


def rok(c, lanes):  # read groups: lane bits 0,1 free, bits 2,3,4 in a parity class
    w = W[c]
    for par in (0, 1):
        s = {(x * w[lanes[0]] + y * w[lanes[1]] + a * w[lanes[2]] + b * w[lanes[3]] + d * w[lanes[4]]) % 16
             for x in (0, 1) for y in (0, 1) for a in (0, 1) for b in (0, 1) for d in (0, 1)
             if (a + b + d) % 2 == par}
        if len(s) != 16:
            return False
    return True


def size(c):
    return 511 + sum(c) + 1


def best_func(A, B):
    f = [c for c in cands if wok(c, A) and rok(c, B)]
    return min(f, key=size) if f else None


LA = (0, 1, 2, 3, 4, 5)
if "--lb" in sys.argv:
    l2 = tuple(int(x) for x in sys.argv[sys.argv.index("--lb") + 1].split(","))
    res = []
    for l3 in itertools.permutations((3, 4, 5, 6, 7, 8)):
        f2 = best_func(l2, l3)
        g2 = best_func(l3, l2) if f2 else None
        if g2:
            res.append((max(size(f2), size(g2)), l3, f2, g2))
    sz, l3, f2, g2 = min(res)
    print("scratch", sz, "LC lanes", l3)
    print("R2F", f2, "R2I", g2)
    sys.exit(0)
best = None
for l2 in itertools.permutations((0, 1, 2, 6, 7, 8)):
    f1, g1 = best_func(LA, l2), best_func(l2, LA)
    if not (f1 and g1):
        continue
    for l3 in itertools.permutations((3, 4, 5, 6, 7, 8)):
        f2 = best_func(l2, l3)
        g2 = best_func(l3, l2) if f2 else None
        if not g2:
            continue
        sz = max(map(size, (f1, g1, f2, g2)))
        if best is None or sz < best[0]:
            best = (sz, l2, l3, f1, g1, f2, g2)
print("scratch", best[0], "LB lanes", best[1], "LC lanes", best[2])
print("R1F", best[3], "R1I", best[4], "R2F", best[5], "R2I", best[6])
