"""Test helpers (no tests here): the exact rounds of a sign extraction, in
numpy, against which tests/test_gpu_decision_noise.py measures the decision
noise the library's bootstraps see (fhe_sign_trace_batch), and the CPU test
of the round bookkeeping (tests/test_params_and_search.py).

A round of fhe_sign_batch (fheicp.params.sign_round_ops, fheicp.hip
sign_extract) key-switches v_cur << shift, adds `add`, and the blind rotation
reads the test vector at the rotation exponent phi (the phase modulus-switched
to 2N). The exact exponent is ideal = ((v_cur << (64 - P + shift)) + add) / 2^53
(for 2N = 2048), the centre of v_cur's slot, and the decision noise of the
round is phi - ideal: every earlier bootstrap's output noise amplified by
2^shift, the input's noise likewise, plus the key switch and the modulus
switch. The decision is wrong exactly when the test vector reads differently
at phi than at ideal.
"""
from __future__ import annotations

import math

import numpy as np

U64 = np.uint64


def v_cur(v: np.ndarray, op: dict) -> np.ndarray:
    """v with the bits the earlier rounds cleared (op['lo'] low bits, and the
    digit's top bit op['hi'] for a staircase round), two's complement."""
    out = np.asarray(v, dtype=np.int64) & ~np.int64((1 << op["lo"]) - 1)
    if op["hi"] is not None:
        out = out & ~np.int64(1 << op["hi"])
    return out


def ideal_index(v: np.ndarray, op: dict, P: int, N: int) -> np.ndarray:
    """Exact rotation exponent of the round for values v (int64 array)."""
    lg = int(2 * N).bit_length() - 1
    with np.errstate(over="ignore"):
        ph = (v_cur(v, op).astype(np.int64).view(U64) << U64(64 - P + op["shift"])) + U64(op["add"])
    if np.any(ph & U64((1 << (64 - lg)) - 1)):
        raise AssertionError("the exact phase is not on the 2N grid")
    return (ph >> U64(64 - lg)).astype(np.int64)


def tv_decode(idx: np.ndarray, op: dict, N: int) -> np.ndarray:
    """The test-vector word the rotation selects at exponent idx (common.h
    tv_rot, negacyclic): base + (j >> tv_shift) * step, negated from N on."""
    base, step, sh = op["tv"]
    idx = np.asarray(idx, dtype=np.int64)
    j = (idx & (N - 1)).astype(U64)
    with np.errstate(over="ignore"):
        val = U64(base) + (j >> U64(sh)) * U64(step)
        return np.where(idx < N, val, U64(0) - val)


def boundary_distances(op: dict, N: int):
    """(d_lo, d_hi) per exponent x in [0, 2N): the smallest k > 0 with a
    different test-vector word at x - k, resp. x + k (mod 2N)."""
    M = 2 * N
    x = np.arange(M)
    dec = tv_decode(x, op, N)
    d_lo = np.zeros(M, np.int64)
    d_hi = np.zeros(M, np.int64)
    for k in range(1, M):
        hi = (d_hi == 0) & (tv_decode((x + k) % M, op, N) != dec)
        d_hi[hi] = k
        lo = (d_lo == 0) & (tv_decode((x - k) % M, op, N) != dec)
        d_lo[lo] = k
        if (d_lo > 0).all() and (d_hi > 0).all():
            break
    return d_lo, d_hi


def centred(phi: np.ndarray, ideal: np.ndarray, N: int) -> np.ndarray:
    """phi - ideal in (-N, N] of the 2N grid (signed decision noise in grid units)."""
    M = 2 * N
    return (np.asarray(phi, np.int64) - ideal + N) % M - N


def qfunc(x):
    """Gaussian upper tail Q(x), elementwise."""
    x = np.asarray(x, dtype=np.float64)
    from scipy.special import erfc
    return 0.5 * erfc(x / math.sqrt(2.0))


def flip_probability(ideal: np.ndarray, op: dict, N: int, mu: float, sd: float, dist=None) -> np.ndarray:
    """Probability that a Gaussian decision noise N(mu, sd^2) (grid units)
    moves the round's exponent off its test-vector word: the integer noise
    reaches d_hi (>= d_hi - 1/2 continuous) or -d_lo."""
    d_lo, d_hi = dist if dist is not None else boundary_distances(op, N)
    lo, hi = d_lo[ideal], d_hi[ideal]
    return qfunc((hi - 0.5 - mu) / sd) + qfunc((lo - 0.5 + mu) / sd)


def ms_phase_numpy(small: np.ndarray, s: np.ndarray, N: int, group: int) -> np.ndarray:
    """k_ms_phase restated from the oracle's rounding (tfhe_ref.c modswitch,
    pbs1g / pbs1_mb): b~ - sum over set key bits of a~_i (classic) or of the
    active subset's exponent per pair (multi-bit: a~_1, a~_2, or the switch of
    the exact sum a_1 + a_2 when both bits are set), mod 2N."""
    lg = int(2 * N).bit_length() - 1
    M = 1 << lg

    def ms(a):
        return (((a >> U64(63 - lg)) + U64(1)) >> U64(1)).astype(np.int64) & (M - 1)

    small = np.asarray(small, dtype=U64)
    n = small.shape[1] - 1
    s = np.asarray(s, dtype=U64).astype(bool)
    acc = np.zeros(small.shape[0], np.int64)
    if group == 2:
        for j in range(0, n, 2):
            s1, s2 = s[j], (j + 1 < n and s[j + 1])
            if s1 and s2:
                with np.errstate(over="ignore"):
                    acc += ms(small[:, j] + small[:, j + 1])
            elif s1:
                acc += ms(small[:, j])
            elif s2:
                acc += ms(small[:, j + 1])
    else:
        for i in range(n):
            if s[i]:
                acc += ms(small[:, i])
    return (ms(small[:, n]) - acc) % M
