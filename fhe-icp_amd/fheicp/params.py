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
    ks_base_log: int = 4
    ks_level: int = 4
    lwe_noise_bits: int = 46
    glwe_noise_bits: int = 17
    msg_bits: int = 16
    # digit width of the sign extraction; 0 = sign_digit_bits(): the widest
    # meeting the noise bar (fhe_params.sign_digit_bits)
    sign_digit_bits: int = 0

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
PBS_GADGETS = ((17, 15, 2), (21, 12, 3), (23, 10, 4), (25, 8, 5), (26, 7, 6), (27, 6, 7))
SIGMA_BAR = 9.2


def sign_digit_bits(p: "SchemeParams") -> int:
    """Digit width of fhe_sign_batch (fhe_sign_digit_bits): the explicit
    p.sign_digit_bits (3 or 4), else 4 if its worst round keeps SIGMA_BAR
    sigmas (noise_report), else 3; 0 when P < 4 (single-bit rounds)."""
    P = p.msg_bits
    if P < 4:
        return 0
    if p.sign_digit_bits not in (0, 3, 4):
        raise ValueError("sign_digit_bits must be 0 (auto), 3 or 4")
    if p.sign_digit_bits:
        return min(p.sign_digit_bits, P)
    for d in range(min(4, P), 3, -1):
        if _digit_margin(p, d) >= SIGMA_BAR:
            return d
    return 3


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


def params_for_bits(P: int) -> SchemeParams:
    for pmax, beta, lvl in PBS_GADGETS:
        if P <= pmax:
            return SchemeParams(pbs_base_log=beta, pbs_level=lvl, msg_bits=P)
    raise ValueError(f"accumulator width P={P} exceeds the supported 27 bits")


# A tiny, INSECURE set with the same structure, for fast functional tests.
TOY = SchemeParams(n=64, k=2, N=256, pbs_base_log=15, pbs_level=2, ks_base_log=4, ks_level=4,
                   lwe_noise_bits=46, glwe_noise_bits=17, msg_bits=8)


def _tuniform_var(b: int) -> float:
    """Variance of TUniform(b): (2^(2b+1) + 1) / 6."""
    return (2.0 ** (2 * b + 1) + 1.0) / 6.0


def _variances(p: SchemeParams):
    """(bootstrap, key switch, modulus switch) output variances, relative to
    the 2^64 torus."""
    q2 = 2.0 ** 128
    s2_bsk = _tuniform_var(p.glwe_noise_bits) / q2
    s2_ksk = _tuniform_var(p.lwe_noise_bits) / q2
    B = 2.0 ** p.pbs_base_log
    rows = p.pbs_level * (p.k + 1) * p.N
    br_key = p.n * rows * (B * B + 2) / 12.0 * s2_bsk
    br_round = p.n * (1 + p.k * p.N / 2) / (12.0 * B ** (2 * p.pbs_level))
    v_pbs = br_key + br_round
    Bk = 2.0 ** p.ks_base_log
    v_ks = p.k * p.N * p.ks_level * (Bk * Bk + 2) / 12.0 * s2_ksk
    v_ks += p.k * p.N / 2 * (2.0 ** (-2 * p.ks_level * p.ks_base_log)) / 12.0
    v_ms = (p.n / 2 + 1) / 12.0 / (2.0 * p.N) ** 2
    return v_pbs, v_ks, v_ms


def _digit_margin(p: SchemeParams, d: int) -> float:
    v_pbs, v_ks, v_ms = _variances(p)
    return 2.0 ** -(d + 1) / math.sqrt(v_pbs * 4.0 ** (p.msg_bits - d) + v_ks + v_ms)


def noise_report(p: SchemeParams, method: str = "digits") -> dict:
    """Variance model (relative to the 2^64 torus) of the worst extraction round.

    method "bits" (fhe_bit_extract_batch): round i = 1, the PBS output noise of
    bit 0 amplified by 2^(P-2), decision margin 1/4 of the torus.
    method "digits" (fhe_sign_batch, P >= 4) with d = sign_digit_bits(p): the
    staircase bootstrap of the first d-bit digit, the digit-MSB bootstrap's
    noise amplified by 2^(P-d), margin 2^-(d+1).
    """
    if method not in ("bits", "digits"):
        raise ValueError(method)
    d = sign_digit_bits(p) if method == "digits" and p.msg_bits >= 4 else 1
    v_pbs, v_ks, v_ms = _variances(p)
    v_amp = v_pbs * 4.0 ** (p.msg_bits - (d if d > 1 else 2))
    v_total = v_amp + v_ks + v_ms
    sigma = math.sqrt(v_total)
    margin_sigmas = (2.0 ** -(d + 1) if d > 1 else 0.25) / sigma
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
