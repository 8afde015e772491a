"""Parameter sets and the noise model that selects them.

The reference delegates parameter choice to Concrete's optimizer inside
``model.compile`` (fhe_similarity.py:120), sized from a 10-sample inputset.
Here parameters are chosen from the WORST-CASE accumulator width P (every
representable quantized input), so no input can overflow the encoding.

Security anchors (not re-estimated here; no lattice estimator offline):
  * small LWE (n = 887, TUniform(46)) and
  * GLWE with k*N = 2048 and TUniform(17)
are the pairs tfhe-rs publishes as 128-bit secure for its TUniform
parameter sets; this build uses k = 2, N = 1024 (same k*N).
"""
from __future__ import annotations

import math
from dataclasses import asdict, dataclass, replace


@dataclass(frozen=True)
class SchemeParams:
    n: int = 887
    k: int = 2
    N: int = 1024
    pbs_base_log: int = 15
    pbs_level: int = 2
    # key switch: 5 levels of base 2^3 (15 bits). The modulus switch is the
    # largest fixed noise term of a sign round (2^-8.39); the key switch
    # comes next, and at (3, 5) it is 2^-10.72 against 2^-10.06 at (4, 4):
    # enough margin that the P = 16 plan needs no classic main round (all
    # multi-bit) and the P = 26 plan goes from 3- to 4-bit digits (17 -> 13
    # bootstraps) for 1.25x the key-switch work
    ks_base_log: int = 3
    ks_level: int = 5
    lwe_noise_bits: int = 46
    glwe_noise_bits: int = 17
    msg_bits: int = 16
    # digit width of the sign extraction; 0 = sign_digit_bits(): the widest
    # meeting the noise bar (fhe_params.sign_digit_bits)
    sign_digit_bits: int = 0
    # second, faster bootstrap gadget (same keys, its own bootstrapping key)
    # for the sign-extraction rounds whose noise is not amplified much; 0, 0 =
    # none (fhe_params.pbs_fast_base_log / pbs_fast_level, sign_plan())
    pbs_fast_base_log: int = 0
    pbs_fast_level: int = 0
    # third, cheapest gadget for the last rounds (needs the fast one; 0, 0 = none)
    pbs_fast2_base_log: int = 0
    pbs_fast2_level: int = 0
    # grouping factor of the fast / fast2 gadget's blind rotation: 0 or 1 =
    # one LWE coefficient per step, 2 = pairs (multi-bit key)
    pbs_fast_group: int = 0
    pbs_fast2_group: int = 0
    # up to two gadgets between the main and the fast one (classic rotation;
    # 0, 0 = none; mid needs the fast gadget, mid2 needs mid): the sign plan
    # runs main -> mid -> mid2 -> fast -> fast2 (sign_schedule)
    pbs_mid_base_log: int = 0
    pbs_mid_level: int = 0
    pbs_mid2_base_log: int = 0
    pbs_mid2_level: int = 0
    # grouping factor of the mid / mid2 gadget's blind rotation (as
    # pbs_fast_group; 2 = multi-bit, 48-bit accumulators past level 2)
    pbs_mid_group: int = 0
    pbs_mid2_group: int = 0
    # a sixth gadget between the main and the mid one (0, 0 = none; needs
    # mid): the ladder is main -> mid0 -> mid -> mid2 -> fast -> fast2, so a
    # plan's most amplified round can run on a multi-bit gadget as precise as
    # the classic main one (P = 26: (5,8) multi-bit)
    pbs_mid0_base_log: int = 0
    pbs_mid0_level: int = 0
    pbs_mid0_group: int = 0

    def as_dict(self) -> dict:
        return asdict(self)

    def with_msg_bits(self, P: int) -> "SchemeParams":
        return replace(self, msg_bits=int(P))


# Bootstrap gadget by message width (checked by noise_report()): the widest
# P each (base_log, level) supports with >= 9.2 sigma at the decision margin
# of the 3-bit digit sign extraction (fhe_sign_batch), whose worst round is
# the low-bits bootstrap of the first digit: margin 2^-4, the first bootstrap's
# noise amplified by 2^(P-3). The single-bit extraction (fhe_bit_extract_batch:
# margin 2^-2, amplification 2^(P-2)) is looser at every entry. Wider digits
# (sign_digit_bits) are used where they too keep 9.2 sigma.
PBS_GADGETS = ((17, 15, 2), (21, 12, 3), (23, 10, 4), (24, 8, 5), (25, 7, 6), (26, 6, 7), (27, 5, 8))
SIGMA_BAR = 9.2
# candidate fast gadgets for the low-amplification sign rounds, each with
# the classic (1) or the multi-bit (2) blind rotation, and the blind-rotation
# time per bootstrap by (level, group) relative to L = 2 classic, measured on
# MI355X at 4096 ciphertexts (tests/test_gpu_noise.py timing lines,
# profiles/r03e_noise.log), ms per 1024: classic v4 (32-bit accumulators)
# L = 1, 2: 6.38 / 9.87; key-stationary v4s (64-bit) L = 3..8: 13.9 / 18.0 /
# 21.0 / 24.4 / 27.4 / 31.1; multi-bit L = 1, 2 (32-bit): 4.32 / 7.09; multi-bit
# L = 3..8 (48-bit, mb64): 10.5 / 13.0 / 15.9 / 18.6 / 21.4 / 24.2. Only the
# ranking matters.
FAST_GADGETS = ((15, 2, 1), (23, 1, 1), (15, 2, 2), (23, 1, 2))
BR_COST = {(1, 1): 0.647, (2, 1): 1.0, (3, 1): 1.413, (4, 1): 1.824, (5, 1): 2.125, (6, 1): 2.476,
           (7, 1): 2.781, (8, 1): 3.147, (1, 2): 0.438, (2, 2): 0.718, (3, 2): 1.059, (4, 2): 1.313,
           (5, 2): 1.612, (6, 2): 1.884, (7, 2): 2.164, (8, 2): 2.454}


def sign_rounds(P: int, d: int):
    """The bootstraps of fhe_sign_batch in order as (shift, log2 margin): the
    round decides on v << shift, so every earlier bootstrap's output noise is
    amplified by 2^shift (fheicp.hip sign_rounds)."""
    out, b, m = [], 0, P - d
    while b + d <= m:
        out += [(P - b - d, -(d + 1))] * 2
        b += d
    if m - b >= 3:
        c = m - b
        out += [(P - b - c, -(c + 1))] * 2
        b = m
    while b < m:
        out.append((P - b - 1, -2))
        b += 1
    out.append((0, -(d + 1)))
    return out


def sign_round_ops(P: int, d: int, N: int):
    """Every round of fhe_sign_batch as the library issues it (fheicp.hip
    sign_extract), for measuring it: the key switch of v << shift centred by
    `add`, the bootstrap's test vector (base, step, tv_shift) and mode, and
    the bits of v already cleared when the round runs: the round decides on
    v_cur = v with bits [0, lo) and the bit `hi` (if not None) cleared."""
    logN = N.bit_length() - 1
    ops = []
    if P < 4:
        for i in range(P):
            ops.append(dict(shift=P - 1 - i, add=1 << 62, tv=(1 << (63 - P + i), 0, 0), mode=1, lo=i, hi=None))
        return ops
    m = P - d

    def digit(b, c):
        ops.append(dict(shift=P - b - c, add=1 << (63 - c), tv=(1 << (62 - P + b + c), 0, 0), mode=1, lo=b, hi=None))
        ops.append(dict(shift=P - b - c, add=1 << (63 - c), tv=(0, 1 << (64 - P + b), logN - (c - 1)), mode=2,
                        lo=b, hi=b + c - 1))
    b = 0
    while b + d <= m:
        digit(b, d)
        b += d
    if m - b >= 3:
        digit(b, m - b)
        b = m
    while b < m:
        ops.append(dict(shift=P - b - 1, add=1 << 62, tv=(1 << (63 - P + b), 0, 0), mode=1, lo=b, hi=None))
        b += 1
    ops.append(dict(shift=0, add=1 << (63 - d), tv=(1 << 62, 0, 0), mode=1, lo=m, hi=None))
    return ops


def sign_round_sigmas(p: "SchemeParams", sched=None):
    """The noise model of every decision of the sign extraction, round by
    round (the terms of _sched_worst): [(shift, log2 margin, sigma)], sigma
    relative to the torus, on the plan's schedule or an explicit one. The
    input ciphertext's own noise is not in it (the caller adds it)."""
    d, plan = sign_schedule(p)
    sched = list(plan if sched is None else sched)
    rounds = sign_rounds(p.msg_bits, d)
    if len(sched) != len(rounds):
        raise ValueError(f"schedule has {len(sched)} rounds, the plan {len(rounds)}")
    vs = {g: _gadget_var(p, g) for g in set(sched)}
    vms = {g: _ms_var(p, gadget_of(p, g)[2]) for g in set(sched)}
    _, v_ks, _ = _variances(p)
    acc, out = 0.0, []
    for r, (sh, ml) in enumerate(rounds):
        out.append((sh, ml, math.sqrt(acc * 4.0 ** sh + v_ks + vms[sched[r]])))
        acc += vs[sched[r]]
    return out


# gadget ids (fhe_pbs_gadget_batch): 0 main, 1 fast, 2 fast2, 3 mid, 4 mid2, 5 mid0
GADGET_IDS = (0, 1, 2, 3, 4, 5)


def gadget_level(p: "SchemeParams", g: int) -> int:
    return (p.pbs_level, p.pbs_fast_level, p.pbs_fast2_level, p.pbs_mid_level, p.pbs_mid2_level,
            p.pbs_mid0_level)[g]


def gadget_of(p: "SchemeParams", g: int):
    """(base_log, level, group) of gadget g: 0 main, 1 fast, 2 fast2, 3 mid,
    4 mid2, 5 mid0 (an absent fast2 falls back to the fast one, an absent
    fast, mid, mid2 or mid0 gadget to the main one)."""
    if g == 2 and p.pbs_fast2_level:
        return p.pbs_fast2_base_log, p.pbs_fast2_level, max(p.pbs_fast2_group, 1)
    if g in (1, 2) and p.pbs_fast_level:
        return p.pbs_fast_base_log, p.pbs_fast_level, max(p.pbs_fast_group, 1)
    if g == 3 and p.pbs_mid_level:
        return p.pbs_mid_base_log, p.pbs_mid_level, max(p.pbs_mid_group, 1)
    if g == 4 and p.pbs_mid2_level:
        return p.pbs_mid2_base_log, p.pbs_mid2_level, max(p.pbs_mid2_group, 1)
    if g == 5 and p.pbs_mid0_level:
        return p.pbs_mid0_base_log, p.pbs_mid0_level, max(p.pbs_mid0_group, 1)
    return p.pbs_base_log, p.pbs_level, 1


def _gadget_var(p: "SchemeParams", g: int) -> float:
    bl, lv, grp = gadget_of(p, g)
    return _variances(replace(p, pbs_base_log=bl, pbs_level=lv), group=grp)[0]


def table_gadget(p: "SchemeParams") -> int:
    """The gadget fhe_pbs_table_batch runs on (fheicp.hip table_gadget): the
    multi-bit gadget of the set with the smallest bootstrap noise (first on a
    tie, in gadget order), 0 (the classic main gadget) when it has none."""
    groups = (p.pbs_fast_group, p.pbs_fast2_group, p.pbs_mid_group, p.pbs_mid2_group, p.pbs_mid0_group)
    best, v = 0, 0.0
    for g in range(1, 6):
        if not gadget_level(p, g) or groups[g - 1] != 2:
            continue
        vg = _gadget_var(p, g)
        if not best or vg < v:
            best, v = g, vg
    return best


def _sched_worst(p: "SchemeParams", d: int, sched) -> float:
    """Worst decision margin (sigmas) when bootstrap r runs on gadget
    sched[r] (fheicp.hip plan_worst); round r's modulus switch is that of its
    own gadget's rotation (classic or multi-bit)."""
    vs = {g: _gadget_var(p, g) for g in set(sched)}
    vms = {g: _ms_var(p, gadget_of(p, g)[2]) for g in set(sched)}
    _, v_ks, _ = _variances(p)
    acc, worst = 0.0, math.inf
    for r, (sh, ml) in enumerate(sign_rounds(p.msg_bits, d)):
        worst = min(worst, 2.0 ** ml / math.sqrt(acc * 4.0 ** sh + v_ks + vms[sched[r]]))
        acc += vs[sched[r]]
    # the last bootstrap's output is the sign ciphertext: decryptable at 1/4
    return min(worst, 0.25 / math.sqrt(vs[sched[-1]]))


def _plan_worst(p: "SchemeParams", d: int, j1: int, j2: int | None = None) -> float:
    """Worst decision margin (sigmas) when bootstraps [0, j1) use the main
    gadget, [j1, j2) the fast one and the rest the fast2 one (j2 = None: all
    the rest on the fast one)."""
    R = len(sign_rounds(p.msg_bits, d))
    if j2 is None:
        j2 = R
    return _sched_worst(p, d, [0 if r < j1 else 1 if r < j2 else 2 for r in range(R)])


def _ladder(p: "SchemeParams"):
    """The gadgets the sign plan walks through, in order: main, mid0, mid,
    mid2, fast, fast2 (those present)."""
    return [0] + [g for g in (5, 3, 4, 1, 2) if gadget_level(p, g)]


def sign_schedule(p: "SchemeParams"):
    """(d, sched) of fhe_sign_batch (fhe_sign_schedule): digit width d and
    the gadget of every bootstrap. Without a fast gadget: d = the explicit
    p.sign_digit_bits, else 4 if its worst round keeps SIGMA_BAR sigmas, else
    3, and every round on the main gadget. With fast gadgets: the widest d (or
    the explicit one); then along the ladder main, mid, mid2, fast, fast2 each
    gadget takes the fewest leading rounds for which the next gadget on all the
    remaining ones keeps every round at SIGMA_BAR (the ladder's variances grow,
    so that is the best the rest can do); the last one takes the rest.
    (0, [0] * P) when P < 4 (single-bit rounds)."""
    P = p.msg_bits
    if P < 4:
        return 0, [0] * max(P, 0)
    if p.sign_digit_bits not in (0, 3, 4):
        raise ValueError("sign_digit_bits must be 0 (auto), 3 or 4")
    if not p.pbs_fast_level:
        if p.sign_digit_bits:
            d = min(p.sign_digit_bits, P)
        else:
            d = min(4, P) if _digit_margin(p, min(4, P)) >= SIGMA_BAR else 3
        return d, [0] * len(sign_rounds(P, d))
    lad = _ladder(p)
    first = min(p.sign_digit_bits, P) if p.sign_digit_bits else min(4, P)
    last = first if p.sign_digit_bits else 3
    for d in range(first, last - 1, -1):
        R = len(sign_rounds(P, d))
        sched, start, ok = [0] * R, 0, True
        for i in range(len(lad) - 1):
            for c in range(start, R + 1):
                sched[start:] = [lad[i]] * (c - start) + [lad[i + 1]] * (R - c)
                if _sched_worst(p, d, sched) >= SIGMA_BAR:
                    break
            else:
                ok = False  # the main gadget alone cannot: a narrower d
                break
            start = c
        if ok:
            return d, sched
    return last, [0] * len(sign_rounds(P, last))


def sign_plan(p: "SchemeParams"):
    """(d, j1, j2) of fhe_sign_batch (fhe_sign_plan): digit width d, the
    leading bootstraps [0, j1) on the main gadget and the first fast2 one j2
    (R without one) of sign_schedule; without mid gadgets, [j1, j2) is the
    fast gadget's. (0, P, P) when P < 4."""
    d, sched = sign_schedule(p)
    R = len(sched)
    j1 = next((r for r, g in enumerate(sched) if g != 0), R)
    j2 = R
    while j2 > 0 and sched[j2 - 1] == 2:
        j2 -= 1
    return d, j1, j2


def sign_digit_bits(p: "SchemeParams") -> int:
    """Digit width of fhe_sign_batch (fhe_sign_digit_bits), from sign_plan."""
    return sign_plan(p)[0]


def sign_precise_rounds(p: "SchemeParams") -> int:
    """Bootstraps of fhe_sign_batch on the main gadget (fhe_sign_precise_rounds)."""
    return sign_plan(p)[1]


def plan_levels(p: SchemeParams) -> list:
    """Gadget level of every bootstrap of the sign extraction, in order."""
    return [gadget_of(p, g)[1] for g in sign_schedule(p)[1]]


def sign_pbs_count(p) -> int:
    """Key switches + bootstraps per sign extraction (fhe_sign_pbs_count);
    an int P means params_for_bits(P)."""
    if not isinstance(p, SchemeParams):
        p = params_for_bits(int(p)) if int(p) >= 1 else SchemeParams(msg_bits=int(p))
    P = p.msg_bits
    if P < 4:
        return max(P, 0)
    d = sign_digit_bits(p)
    m = P - d
    r = m % d
    return 2 * (m // d) + (2 if r >= 3 else r) + 1


def plan_gadgets(p: SchemeParams) -> list:
    """(base_log, level, group) of every bootstrap of the sign extraction."""
    return [gadget_of(p, g) for g in sign_schedule(p)[1]]


def plan_cost(p: SchemeParams) -> float:
    """Relative time of one sign extraction: its bootstraps weighted by
    BR_COST of the gadget and rotation each runs on (sign_plan)."""
    return sum(BR_COST[(lv, grp)] for _, lv, grp in plan_gadgets(p))


def _cheapest_plan(p: SchemeParams) -> SchemeParams:
    """p (main gadget set) with the cheapest fast / fast2 choice of
    FAST_GADGETS, then the cheapest mid / mid2 choice (by plan_cost)."""
    beta, lvl = p.pbs_base_log, p.pbs_level
    cands = [g for g in FAST_GADGETS if g != (beta, lvl, 1)]
    choices = [(g,) for g in cands] + [(a, b) for a in cands for b in cands if a[:2] != b[:2]]
    best = plan_cost(p)
    for ch in choices:
        kw = {"pbs_fast_base_log": ch[0][0], "pbs_fast_level": ch[0][1], "pbs_fast_group": ch[0][2]}
        if len(ch) > 1:
            kw.update(pbs_fast2_base_log=ch[1][0], pbs_fast2_level=ch[1][1], pbs_fast2_group=ch[1][2])
        q = replace(p, **kw)
        c = plan_cost(q)
        if c < best - 1e-9:
            p, best = q, c
    if p.pbs_fast_level:
        # then one or two mid gadgets between the main and the fast one:
        # gadgets of PBS_GADGETS on the classic rotation below the main level,
        # or on the multi-bit one at any level up to it (a multi-bit mid at the
        # main gadget's own level can take the first rounds from it)
        mids = [(b, lv, 1) for _, b, lv in PBS_GADGETS if lv < lvl]
        mids += [(b, lv, 2) for _, b, lv in PBS_GADGETS if 3 <= lv <= lvl and (lv, 2) in BR_COST]
        q0 = p
        for ch in [(m,) for m in mids] + [(a, b) for a in mids for b in mids if a[1] > b[1]]:
            kw = {"pbs_mid_base_log": ch[0][0], "pbs_mid_level": ch[0][1], "pbs_mid_group": ch[0][2]}
            if len(ch) > 1:
                kw.update(pbs_mid2_base_log=ch[1][0], pbs_mid2_level=ch[1][1], pbs_mid2_group=ch[1][2])
            q = replace(q0, **kw)
            c = plan_cost(q)
            if c < best - 1e-9:
                p, best = q, c
    return p


def _with_mid0(p: SchemeParams) -> SchemeParams:
    """p with a sixth gadget ahead of the mids if it makes the plan cheaper:
    a multi-bit one above the mid level, up to one past the main gadget's
    (its more precise neighbour in PBS_GADGETS), with L * beta <= 47 (the
    48-bit-accumulator kernels), so the first, most amplified rounds run on
    the multi-bit rotation instead of the classic main one.
    Tried after the main gadget is chosen, so plans it does not improve stay
    as they were."""
    if not p.pbs_mid_level:
        return p
    best, q1 = plan_cost(p), p
    for b0, lv0 in sorted({(b, lv) for _, b, lv in PBS_GADGETS if p.pbs_mid_level < lv <= q1.pbs_level + 1}):
        if (lv0, 2) not in BR_COST or b0 * lv0 > 47:
            continue
        q = replace(q1, pbs_mid0_base_log=b0, pbs_mid0_level=lv0, pbs_mid0_group=2)
        c = plan_cost(q)
        if c < best - 1e-9:
            p, best = q, c
    return p


def params_for_bits(P: int, fast: bool = True) -> SchemeParams:
    """The gadget of PBS_GADGETS for width P; with fast, also up to two of
    FAST_GADGETS (other than the main gadget, in their order: fast, then
    fast2) for the sign rounds whose noise is barely amplified, the choice
    whose sign plan is cheapest by BR_COST, if it beats the single-gadget
    plan; then up to two mid gadgets (cheaper entries of PBS_GADGETS) for the
    rounds between, if they make the plan cheaper still. A more precise main
    gadget (the next entry of the table) is taken when its cheapest plan is
    cheaper: a quieter first bootstrap can allow 4-bit digits (DESIGN.md
    §3.6). Last, a multi-bit mid0 gadget for the first rounds (_with_mid0)."""
    for i, (pmax, beta, lvl) in enumerate(PBS_GADGETS):
        if P <= pmax:
            p = SchemeParams(pbs_base_log=beta, pbs_level=lvl, msg_bits=P)
            if not (fast and P >= 4):
                return p
            p = _cheapest_plan(p)
            best = plan_cost(p)
            for _, b2, l2 in PBS_GADGETS[i + 1:i + 2]:
                q = _cheapest_plan(SchemeParams(pbs_base_log=b2, pbs_level=l2, msg_bits=P))
                c = plan_cost(q)
                if c < best - 1e-9:
                    p, best = q, c
            return _with_mid0(p)
    raise ValueError(f"accumulator width P={P} exceeds the supported 27 bits")


# A tiny, INSECURE set with the same structure, for fast functional tests.
TOY = SchemeParams(n=64, k=2, N=256, pbs_base_log=15, pbs_level=2, ks_base_log=4, ks_level=4,
                   lwe_noise_bits=46, glwe_noise_bits=17, msg_bits=8)


# FFT error constant of the noise model: bounds the 11.6-13.8 measured on
# every MI355X blind-rotation instance (tests/test_gpu_noise.py)
C_FFT = 16.0


def _tuniform_var(b: int) -> float:
    """Variance of TUniform(b): (2^(2b+1) + 1) / 6."""
    return (2.0 ** (2 * b + 1) + 1.0) / 6.0


def ks_round_bits(p: SchemeParams) -> int:
    """The key switch rounds every KSK word to a multiple of 2^R (fheicp.hip
    ks_round_bits, oracle/tfhe_ref.c): R = 8 floor((lwe_noise_bits - 6) / 8),
    at most 40, so the rounding stays below 2^-7 of the KSK noise and the i8
    matrix-core key switch needs 8 - R / 8 byte planes."""
    return 0 if p.lwe_noise_bits < 14 else 8 * min((p.lwe_noise_bits - 6) // 8, 5)


def _variances(p: SchemeParams, group: int = 1):
    """(bootstrap, key switch, modulus switch) output variances, relative to
    the 2^64 torus, for the main gadget of p on the classic
    (group 1) or the multi-bit (group 2) blind rotation: per pair, three GGSWs
    times (X^a - 1) (3x the key noise), one gadget rounding whose error is
    multiplied by X^e - 1 (the same total as n classic steps), three subsets'
    products at |psi^(a e) - 1|^2 ~ 2 (3x the FFT error) and half the 2^32
    output roundings."""
    q2 = 2.0 ** 128
    s2_bsk = _tuniform_var(p.glwe_noise_bits) / q2
    R = ks_round_bits(p)
    s2_ksk = (_tuniform_var(p.lwe_noise_bits) + (2.0 ** (2 * R) / 12.0 if R else 0.0)) / q2
    B = 2.0 ** p.pbs_base_log
    rows = p.pbs_level * (p.k + 1) * p.N
    steps = p.n * (1 + p.k * p.N / 2)
    br_key = p.n * rows * (B * B + 2) / 12.0 * s2_bsk
    br_round = steps / (12.0 * B ** (2 * p.pbs_level))
    # f64 FFT arithmetic error per step and output coefficient (the product's
    # variance rows * N * (B^2/12) * (1/12) times the unit roundoff 2^-106,
    # times C_FFT) and the 2^32 output rounding of the 32-bit-accumulator
    # kernels; key-weighted like the gadget rounding
    arith = C_FFT * rows * B * B / 144.0 * 2.0 ** -106
    if p.pbs_base_log * p.pbs_level <= 31:
        arith += 2.0 ** -64 / 12.0
    if group == 2:
        fft = C_FFT * rows * B * B / 144.0 * 2.0 ** -106
        br_key *= 3.0
        arith = 3.0 * fft + (arith - fft) * 0.5
    v_pbs = br_key + br_round + steps * arith
    Bk = 2.0 ** p.ks_base_log
    v_ks = p.k * p.N * p.ks_level * (Bk * Bk + 2) / 12.0 * s2_ksk
    v_ks += p.k * p.N / 2 * (2.0 ** (-2 * p.ks_level * p.ks_base_log)) / 12.0
    v_ms = _ms_var(p, group)
    return v_pbs, v_ks, v_ms


def _ms_var(p: SchemeParams, group: int = 1) -> float:
    """Modulus-switch variance of a bootstrap's input phase (relative to the
    torus). Classic rotation: each of the ~n/2 set key bits and the body
    carry one rounding to 1/(2N), 1/12 each. Multi-bit (group 2, DESIGN.md
    §4.5): the rotation by sum_i a_i s_i uses the exponent of the ACTIVE
    subset, rounded from the exact sum (round(a1 + a2) for s = (1, 1)), so a
    pair carries one rounding if any bit is set: 3/4 x 1/12 per full pair,
    1/2 x 1/12 for a lone last coefficient, plus the body's."""
    if group == 2:
        per = (p.n // 2) * 0.75 / 12.0 + (p.n % 2) * 0.5 / 12.0 + 1.0 / 12.0
    else:
        per = (p.n / 2 + 1) / 12.0
    return per / (2.0 * p.N) ** 2


def _digit_margin(p: SchemeParams, d: int) -> float:
    v_pbs, v_ks, v_ms = _variances(p)
    return 2.0 ** -(d + 1) / math.sqrt(v_pbs * 4.0 ** (p.msg_bits - d) + v_ks + v_ms)


def noise_report(p: SchemeParams, method: str = "digits") -> dict:
    """Variance model (relative to the 2^64 torus) of the worst extraction round.

    method "bits" (fhe_bit_extract_batch): round i = 1, the PBS output noise of
    bit 0 amplified by 2^(P-2), decision margin 1/4 of the torus.
    method "digits" (fhe_sign_batch, P >= 4) with d = sign_digit_bits(p): the
    staircase bootstrap of the first d-bit digit, the digit-MSB bootstrap's
    noise amplified by 2^(P-d), margin 2^-(d+1); with a fast
    gadget, the worst round of sign_plan's main/fast schedule.
    """
    if method not in ("bits", "digits"):
        raise ValueError(method)
    d = sign_digit_bits(p) if method == "digits" and p.msg_bits >= 4 else 1
    v_pbs, v_ks, v_ms = _variances(p)
    v_amp = v_pbs * 4.0 ** (p.msg_bits - (d if d > 1 else 2))
    v_total = v_amp + v_ks + v_ms
    sigma = math.sqrt(v_total)
    margin_sigmas = (2.0 ** -(d + 1) if d > 1 else 0.25) / sigma
    if d > 1 and p.pbs_fast_level:
        # several gadgets: the worst round of sign_plan's schedule
        margin_sigmas = _sched_worst(p, d, sign_schedule(p)[1])
        sigma = 2.0 ** -(d + 1) / margin_sigmas
    return {
        "digit_bits": d if d > 1 else 1,
        "log2_sigma_pbs": 0.5 * math.log2(v_pbs),
        "log2_sigma_ks": 0.5 * math.log2(v_ks),
        "log2_sigma_ms": 0.5 * math.log2(v_ms),
        "log2_sigma_total": math.log2(sigma),
        "margin_sigmas": margin_sigmas,
        # two-sided Gaussian tail at the decision margin
        "log2_pfail_per_pbs": math.log2(max(math.erfc(margin_sigmas / math.sqrt(2)), 1e-300)),
    }
