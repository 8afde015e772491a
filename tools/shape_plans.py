#!/usr/bin/env python3
"""Sign-extraction plans at the two GLWE shapes with kN = 2048 (VERDICT r04
item 6): the shipped k = 2, N = 1024 and tfhe-rs's k = 1, N = 2048, under the
same noise model (fheicp.params._variances / _ms_var / sign_rounds), over
key-switch (base, level) choices and sign-digit widths d = 4..6.

Every plan is the cheapest monotone gadget ladder (the first, most amplified
rounds on the most precise gadget) that keeps every decision at 9.2 sigma,
found by exhaustive search over the gadget multiset. Costs: the measured
BR_COST (ms per 1024 bootstraps relative to L = 2 classic) for k = 2, N = 1024;
for k = 1, N = 2048 the same entries times the ratio of counted f64 work per
LWE coefficient (transforms: (k+1)(L+1) complex transforms of M = N/2 points at
~45 flops per point for M = 512 and 50 for M = 1024 (one more radix-2 level);
products: (k+1)^2 L complex MACs per point classic, 3 (k+1)^2 L + 3 (k+1) per
pair multi-bit, 8 flops each). A key-switch cost is added per bootstrap:
0.017 x (level / 5) of the L = 2 classic rotation (k_keyswitch_mfma).
No GPU; prints a markdown table.
With --probe FILE (the output of tools/shape_probe.hip) the k = 1 costs come
from the measured ns per transform point and per complex MAC instead of the
counted flops (--probe-waves 2 or 3: the occupancy the k = 1 kernel is priced
at).
Usage: tools/shape_plans.py [--probe FILE [--probe-waves W]] [P ...]"""
from __future__ import annotations

import itertools
import math
import sys
from dataclasses import replace
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "fhe-icp_amd"))
from fheicp.params import (BR_COST, PBS_GADGETS, SIGMA_BAR, SchemeParams, _ms_var,  # noqa: E402
                           _variances, sign_rounds)

SHAPES = ((2, 1024), (1, 2048))
KS_CHOICES = ((3, 5), (4, 4), (3, 6), (2, 7), (4, 5), (2, 8), (2, 9), (3, 7))
KS_COST = 0.017


def flops_per_coef(k: int, N: int, L: int, grp: int) -> float:
    M = N // 2
    ct = 45.0 if M == 512 else 50.0
    if grp == 1:
        return (k + 1) * (L + 1) * M * ct + (k + 1) ** 2 * L * M * 8
    return ((k + 1) * (L + 1) * M * ct + (3 * (k + 1) ** 2 * L + 3 * (k + 1)) * M * 8) / 2


# measured per-point costs (tools/shape_probe.hip, ns per point per SIMD):
# set by --probe FILE; None = the counted flops above
PROBE = None


def parse_probe(path: str) -> dict:
    """ns per transform point (fwd + inv pair) at M = 512 / 1024 and per
    complex MAC, at 3 and 2 waves per SIMD, from the probe's output."""
    import re
    out = {}
    for ln in open(path):
        m = re.match(r"(\d+)-pt fwd\+inv, (\d) waves/SIMD.*?([\d.]+) ns per pt", ln)
        if m:
            out[("T", int(m.group(1)), int(m.group(2)))] = float(m.group(3))
        m = re.match(r"cmac .*?(\d) w/SIMD.*?([\d.]+) ns per cmac", ln)
        if m:
            out[("mac", int(m.group(1)))] = float(m.group(2))
    return out


def cost_per_pair_measured(k: int, N: int, L: int, grp: int, waves: int) -> float:
    """Probe-priced work per LWE coefficient: (k+1)(L+1) forward + inverse
    transform halves of M points at the measured ns per point, and the
    products' complex MACs at the measured ns per MAC (multi-bit: per pair,
    halved per coefficient)."""
    M = N // 2
    t_T = PROBE[("T", M, waves)] / 2.0      # the probe prices a forward + inverse pair
    t_mac = PROBE[("mac", waves)]
    if grp == 1:
        return (k + 1) * (L + 1) * M * t_T + (k + 1) ** 2 * L * M * t_mac
    return ((k + 1) * (L + 1) * M * t_T + (3 * (k + 1) ** 2 * L + 3 * (k + 1)) * M * t_mac) / 2


# the occupancy a k = 1, N = 2048 kernel is priced at (--probe-waves)
K1_WAVES = 2


def br_cost(k: int, N: int, L: int, grp: int) -> float:
    base = BR_COST[(L, grp)]
    if (k, N) == (2, 1024):
        return base
    if PROBE:
        return base * cost_per_pair_measured(k, N, L, grp, K1_WAVES) / cost_per_pair_measured(2, 1024, L, grp, 3)
    return base * flops_per_coef(k, N, L, grp) / flops_per_coef(2, 1024, L, grp)


def gadgets():
    """(base_log, level, group): the PBS table on both rotations (multi-bit
    L * beta <= 47) and the fast gadgets."""
    out = {(b, lv, 1) for _, b, lv in PBS_GADGETS} | {(b, lv, 2) for _, b, lv in PBS_GADGETS if lv * b <= 47}
    out |= {(15, 2, 1), (23, 1, 1), (15, 2, 2), (23, 1, 2), (12, 3, 2), (10, 4, 2), (8, 5, 2)}
    return sorted(out)


def best_plan(p: SchemeParams, d: int):
    """Cheapest ladder for digit width d: (cost, pbs count, gadget list) or None."""
    rounds = sign_rounds(p.msg_bits, d)
    R = len(rounds)
    _, v_ks, _ = _variances(p)
    gs = gadgets()
    var = {g: _variances(replace(p, pbs_base_log=g[0], pbs_level=g[1]), group=g[2])[0] for g in gs}
    vms = {g: _ms_var(p, g[2]) for g in gs}
    cost = {g: br_cost(p.k, p.N, g[1], g[2]) + KS_COST * p.ks_level / 5 for g in gs}
    # a ladder never takes a gadget both noisier and costlier than another
    cand = [g for g in gs if not any(var[h] <= var[g] and cost[h] < cost[g] - 1e-12 for h in gs)]
    cand.sort(key=lambda g: var[g])
    best = None
    for combo in itertools.combinations_with_replacement(range(len(cand)), R):
        sched = [cand[i] for i in combo]           # precise first
        c = sum(cost[g] for g in sched)
        if best and c >= best[0] - 1e-12:
            continue
        acc, ok = 0.0, True
        for r, (sh, ml) in enumerate(rounds):
            if 2.0 ** ml / math.sqrt(acc * 4.0 ** sh + v_ks + vms[sched[r]]) < SIGMA_BAR:
                ok = False
                break
            acc += var[sched[r]]
        if ok and 0.25 / math.sqrt(var[sched[-1]]) >= SIGMA_BAR:
            best = (c, R, sched)
    return best


def main():
    global PROBE, K1_WAVES
    args = sys.argv[1:]
    if "--probe" in args:
        i = args.index("--probe")
        PROBE = parse_probe(args[i + 1])
        del args[i:i + 2]
    if "--probe-waves" in args:
        i = args.index("--probe-waves")
        K1_WAVES = int(args[i + 1])
        del args[i:i + 2]
    Ps = [int(x) for x in args] or [16, 21, 26]
    if PROBE:
        print(f"costs: measured (tools/shape_probe.hip), k = 1 priced at {K1_WAVES} waves/SIMD; "
              f"probe: " + ", ".join(f"{k}: {v}" for k, v in sorted(PROBE.items(), key=str)))
        for L in (1, 2, 3, 5, 8):
            print(f"  L = {L} multi-bit: k=1,N=2048 / k=2,N=1024 work per coefficient = "
                  f"{br_cost(1, 2048, L, 2) / BR_COST[(L, 2)]:.3f} (counted flops: "
                  f"{flops_per_coef(1, 2048, L, 2) / flops_per_coef(2, 1024, L, 2):.3f})")
        print()
    print("| P | shape (k, N) | key switch | d | PBS | plan (base_log, level, group) | relative cost |")
    print("|---|---|---|---|---|---|---|")
    summary = {}
    for P in Ps:
        for k, N in SHAPES:
            rows = []
            for bks, lks in KS_CHOICES:
                if lks * (bks + 1) + P > 64:
                    continue
                p = SchemeParams(k=k, N=N, ks_base_log=bks, ks_level=lks, msg_bits=P)
                for d in (4, 5, 6):
                    if d > P:
                        continue
                    b = best_plan(p, d)
                    if b:
                        rows.append((b[0], (bks, lks), d, b[1], b[2]))
            rows.sort(key=lambda r: r[0])
            summary[(P, k, N)] = rows[0] if rows else None
            for c, ks, d, n, sched in rows[:3]:
                plan = " ".join(f"{g[0]},{g[1]}{'mb' if g[2] == 2 else ''}" for g in sched)
                print(f"| {P} | ({k}, {N}) | {ks} | {d} | {n} | {plan} | {c:.3f} |")
            if not rows:
                print(f"| {P} | ({k}, {N}) | — | — | — | no plan keeps 9.2 sigma | — |")
    print()
    for P in Ps:
        a, b = summary.get((P, 2, 1024)), summary.get((P, 1, 2048))
        if a and b:
            print(f"P = {P}: k=1,N=2048 best / k=2,N=1024 best = {b[0] / a[0]:.3f} "
                  f"({b[3]} vs {a[3]} bootstraps, d = {b[2]} vs {a[2]})")


if __name__ == "__main__":
    main()
