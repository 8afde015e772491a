"""LDS bank model of the multi-bit product phase under the lane -> frequency
remap (k_blind_rotate.h, mb::jq): consumer lane l of slot quarter g, slot t,
works on frequency j with j bits 0-3 = l bits 0-3 (so each ds_read_b128 lane
group spans the frequencies whose exponents differ in bits 7-10 only), j bits
6, 7 = the lane group (l2 ^ l3 ^ l4, l5), j bit 4 = t, j bits 5, 8 = g.

Checks, against MI355X_MICROARCH.md's LDS table (ds_read_b128: four 16-lane
groups, banks (a/4) mod 64; ds_write_b128: 8 x 8 contiguous lanes, (a/4) mod 32):
  - psi gathers at entry ((x & 127) << 4) | (x >> 7), x = a e mod 2N, every a;
  - the F reads and the products' hand-off at u * 65 + L (pitch 65);
  - the old mapping (slot quarter {2g, 2g+1}, table x ^ ((x >> 4) & 15)).
Prints LDS cycles per instruction (4 = conflict-free for b128 reads)."""
import numpy as np

LC = [0, 1, 2, 4, 5, 8, 3, 6, 7]  # br_v4.h jof(LC): slot bits, then lane bits
GROUPS = [[*range(0, 4), *range(12, 16), *range(20, 28)], [*range(4, 12), *range(16, 20), *range(28, 32)]]
GROUPS += [[x + 32 for x in g] for g in GROUPS]


def jof_lc(lane, u):
    j = 0
    for b in range(3):
        j |= ((u >> b) & 1) << LC[b]
    for b in range(6):
        j |= ((lane >> b) & 1) << LC[3 + b]
    return j


def lc_pos(j):  # (u, owner lane) of frequency j
    u = sum(((j >> LC[b]) & 1) << b for b in range(3))
    L = sum(((j >> LC[3 + b]) & 1) << b for b in range(6))
    return u, L


def br9(j):
    return int(f"{j:09b}"[::-1], 2)


def jq(g, l, t):
    b = lambda v, i: (v >> i) & 1
    return ((l & 15) | (t << 4) | (b(g, 0) << 5) | ((b(l, 2) ^ b(l, 3) ^ b(l, 4)) << 6) | (b(l, 5) << 7) |
            (b(g, 1) << 8))


def read_cycles(pos):  # ds_read_b128, pos in 16-B entries, one per lane
    c = 0
    for grp in GROUPS:
        addrs = np.unique(pos[grp])
        c += np.bincount(addrs % 16, minlength=16).max()
    return c


def write_cycles(pos):  # ds_write_b128: 8 groups of 8 contiguous lanes, 32 banks
    return sum(np.bincount(pos[8 * k:8 * k + 8] % 8, minlength=8).max() for k in range(8))


def main():
    # bijection
    js = sorted(jq(g, l, t) for g in range(4) for l in range(64) for t in range(2))
    assert js == list(range(512))
    psi_new = lambda x: ((x & 127) << 4) | (x >> 7)
    psi_old = lambda x: x ^ ((x >> 4) & 15)
    assert sorted(psi_new(x) for x in range(2048)) == list(range(2048))
    lanes = np.arange(64)
    for name, jmap, psi in (("old", lambda g, l, t: jof_lc(l, 2 * g + t), psi_old), ("new", jq, psi_new)):
        e = {(g, t): np.array([(4 * br9(jmap(g, l, t)) + 1) & 2047 for l in lanes]) for g in range(4) for t in range(2)}
        tot = n = 0
        for a in range(2048):
            for (g, t), ev in e.items():
                tot += read_cycles(np.array([psi(x) for x in (a * ev) & 2047]))
                n += 1
        pitch = 64 if name == "old" else 65
        fr = hw = 0
        for g in range(4):
            for t in range(2):
                pos = np.array([(lambda uL: uL[0] * pitch + uL[1])(lc_pos(jmap(g, l, t))) for l in lanes])
                fr += read_cycles(pos)
                hw += write_cycles(pos)
        own = np.array([u * pitch + l for u in range(8) for l in lanes]).reshape(8, 64)
        print(f"{name}: psi gather {tot / n:.2f} cycles/read (4 = conflict-free); F read {fr / 8:.2f}; "
              f"hand-off write {hw / 8:.2f} (8 = conflict-free); owner store {np.mean([write_cycles(p) for p in own]):.2f}, "
              f"owner read {np.mean([read_cycles(p) for p in own]):.2f}")


if __name__ == "__main__":
    main()
