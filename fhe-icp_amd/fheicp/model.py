"""Quantized linear similarity model executed under TFHE on the GPU.

This is the engine behind the drop-in estimator (fheicp.sklearn). It owns
 * the post-training quantisation Concrete-ML 1.9 applies to a linear model
   (input: per-tensor asymmetric signed n_bits uniform quantizer; weights:
   symmetric signed; bias at the accumulator scale s_x*s_w) — calibration is
   fit-time host arithmetic, the per-input quantisation runs in the
   k_pair_quantize kernel;
 * the accumulator width P derived from the worst case over every
   representable input (fhe_similarity.py:120 lets Concrete size it from 10
   samples instead), which selects the TFHE parameter set;
 * the encrypted path: quantize -> encrypt -> linear (q_w, -zp*sum(q_w)+q_b-T)
   -> P-round bit extraction -> decrypt, all HIP kernels through libfheicp.
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass

import numpy as np

from .params import SchemeParams, params_for_bits


@dataclass
class QuantParams:
    n_bits: int
    coef: np.ndarray
    intercept: float
    s_x: float
    zp_x: int
    s_w: float
    q_w: np.ndarray
    q_b: int

    @property
    def out_scale(self) -> float:
        return float(np.float64(self.s_x) * np.float64(self.s_w))

    @property
    def qmin(self) -> int:
        return -(2 ** (self.n_bits - 1))

    @property
    def qmax(self) -> int:
        return 2 ** (self.n_bits - 1) - 1

    @property
    def cst(self) -> int:
        """Clear part of Concrete-ML's _inference: -zp_x * sum(q_w) + q_b."""
        return int(-int(self.zp_x) * int(np.asarray(self.q_w, dtype=np.int64).sum()) + int(self.q_b))

    def acc_range(self):
        qw = np.asarray(self.q_w, dtype=np.int64)
        lo = np.minimum(qw * self.qmin, qw * self.qmax).sum() + self.cst
        hi = np.maximum(qw * self.qmin, qw * self.qmax).sum() + self.cst
        return int(lo), int(hi)

    def msg_bits(self) -> int:
        lo, hi = self.acc_range()
        return int(math.ceil(math.log2(hi - lo + 2))) + 1

    def to_dict(self) -> dict:
        return {"n_bits": int(self.n_bits), "coef": [float(c) for c in self.coef], "intercept": float(self.intercept),
                "s_x": float(self.s_x), "zp_x": int(self.zp_x), "s_w": float(self.s_w),
                "q_w": [int(v) for v in self.q_w], "q_b": int(self.q_b)}

    @classmethod
    def from_dict(cls, d: dict) -> "QuantParams":
        return cls(int(d["n_bits"]), np.asarray(d["coef"], dtype=np.float64), float(d["intercept"]), float(d["s_x"]),
                   int(d["zp_x"]), float(d["s_w"]), np.asarray(d["q_w"], dtype=np.int64), int(d["q_b"]))


def _asym_signed(values: np.ndarray, n_bits: int):
    """Concrete-ML UniformQuantizer, is_signed=True, is_symmetric=False."""
    rmin, rmax = float(np.min(values)), float(np.max(values))
    offset = 2 ** (n_bits - 1)
    nlev = 2 ** n_bits - 1
    if rmax == rmin:
        return 1.0, 0
    scale = (rmax - rmin) / nlev
    zp = int(np.round((rmax * (-offset) - rmin * (nlev - offset)) / (rmax - rmin)))
    return scale, zp


def quantize_linear(X: np.ndarray, coef, intercept: float, n_bits: int) -> QuantParams:
    coef = np.asarray(coef, dtype=np.float64).reshape(-1)
    s_x, zp_x = _asym_signed(np.asarray(X, dtype=np.float64), n_bits)
    wmax = float(np.max(np.abs(coef)))
    s_w = wmax / float(2 ** (n_bits - 1) - 1) if wmax > 0 else 1.0
    q_w = np.clip(np.rint(coef / s_w), -(2 ** (n_bits - 1)), 2 ** (n_bits - 1) - 1).astype(np.int64)
    q_b = int(np.rint(np.float64(intercept) / (np.float64(s_x) * np.float64(s_w))))
    return QuantParams(n_bits, coef, float(intercept), s_x, zp_x, s_w, q_w, q_b)


def threshold_int(qp: QuantParams, t: float) -> int:
    """Smallest integer a in [lo, hi+1] with float64(out_scale * a) >= t
    (dequantisation is monotone, so score >= t <=> acc >= T)."""
    lo, hi = qp.acc_range()
    s = np.float64(qp.out_scale)
    ok = lambda a: bool(s * np.float64(a) >= np.float64(t))  # noqa: E731
    if ok(lo):
        return lo
    if not ok(hi):
        return hi + 1
    a = min(max(int(math.ceil(t / float(s))), lo), hi)
    while a > lo and ok(a - 1):
        a -= 1
    while not ok(a):
        a += 1
    return a


class FheLinearModel:
    """Quantized linear regression evaluated under TFHE on one MI355X."""

    def __init__(self, qparams: QuantParams):
        self.qparams = qparams
        self.msg_bits = qparams.msg_bits()
        self.scheme: SchemeParams = params_for_bits(self.msg_bits)
        self.engine = None
        self._w_dev = None
        self._enc_counter = 0
        self.enc_seed = None     # session stream key (32 bytes), or an int seed in tests

    # ------------------------------------------------------------- fitting --
    @classmethod
    def fit(cls, X, y, n_bits: int) -> "FheLinearModel":
        from sklearn.linear_model import LinearRegression as SkLR
        X = np.asarray(X)
        sk = SkLR().fit(X, np.asarray(y))
        coef = np.asarray(sk.coef_, dtype=np.float64).reshape(-1)
        intercept = float(np.asarray(sk.intercept_).reshape(-1)[0])
        return cls(quantize_linear(X, coef, intercept, n_bits))

    # ------------------------------------------------------------- compile --
    def compile(self, key_seed: int | None = None, device: int = 0, enc_seed: int | None = None,
                keys: dict | None = None):
        """Create the device context and generate (or import) the keys.

        Keys: imported (``keys``), or generated from 32 bytes of os.urandom
        through fhe_keygen_key; an explicit ``key_seed`` selects the 64-bit
        seed form (fhe_keygen, reproducible tests and benches only).
        Encryption: every compile starts a session with its own 256-bit stream
        key from os.urandom, never derived from the key material, and a random
        64-bit start for the stream ids, so two sessions (two processes with
        the same configured key_seed included) never share masks or noise.
        Nothing persisted lets the stream key be recomputed. ``enc_seed``
        (tests only) replaces it with a seeded stream starting at id 0."""
        from .engine import Engine
        self.engine = Engine(self.scheme, device)
        if keys is not None:
            self.engine.import_keys(keys)
        elif key_seed is not None:
            self.engine.keygen(seed=int(key_seed))
        else:
            self.engine.keygen(key=os.urandom(32))
        self._w_dev = self.engine.to_dev(np.asarray(self.qparams.q_w, dtype=np.int64))
        if enc_seed is None:
            self.enc_seed = os.urandom(32)
            self._enc_counter = int.from_bytes(os.urandom(8), "little")
        else:
            self.enc_seed = int(enc_seed)
            self._enc_counter = 0
        return self

    @property
    def compiled(self) -> bool:
        return self.engine is not None

    # ------------------------------------------------------------- predict --
    def quantize_dev(self, docs_dev, query_dev=None):
        """Device: q_x = quantize(query (.) docs) (or quantize(docs) when
        query_dev is None), int64 [B, D]; f32/f64 inputs, numpy promotion."""
        import ctypes as C
        import torch
        from . import _lib
        from .engine import _ptr, _stream
        eng = self.engine
        B, D = docs_dev.shape
        qx = torch.empty((B, D), dtype=torch.int64, device=eng.device)
        qp = self.qparams
        q64 = 1 if (query_dev is not None and query_dev.dtype == torch.float64) else 0
        d64 = 1 if docs_dev.dtype == torch.float64 else 0
        _lib.check(eng._L.fhe_quantize_pairs(eng._ctx, _ptr(query_dev), q64, _ptr(docs_dev), d64, B, D,
                                             C.c_double(qp.s_x), qp.zp_x, qp.qmin, qp.qmax, _ptr(qx),
                                             _stream(eng.device)), eng._ctx)
        return qx

    def next_id0(self, count: int) -> int:
        """Stream ids [id0, id0 + count) of the next batch (mod 2^64: the
        kernels add per-row offsets to a u64 id0)."""
        id0 = self._enc_counter
        self._enc_counter = (self._enc_counter + count) & 0xFFFFFFFFFFFFFFFF
        return id0

    def encrypt_linear(self, qx_dev, T: int = 0):
        """The client encryption + leveled dot product alone, under this
        session's stream key: big LWEs [B, kN + 1] of acc - T (device)."""
        if self.engine is None:
            raise RuntimeError("Model not compiled. Call compile() first.")
        B, D = qx_dev.shape
        return self.engine.encrypt_linear(qx_dev, self._w_dev, self.qparams.cst - int(T), self.enc_seed,
                                          self.next_id0(B * D))

    def encrypted_acc(self, qx_dev, T: int = 0):
        """Run the fused encrypted compare on quantized inputs (device)."""
        if self.engine is None:
            raise RuntimeError("Model not compiled. Call compile() first.")
        B = qx_dev.shape[0]
        lo, hi = self.qparams.acc_range()
        T = min(max(int(T), lo), hi + 1)
        return self.engine.compare(qx_dev, self._w_dev, self.qparams.cst, T, self.enc_seed, self.next_id0(B * qx_dev.shape[1]))

    def encrypted_score(self, qx_dev):
        """The reference's encrypted predict as it is (fhe_similarity.py:142-160):
        the leveled circuit only (fhe_score_batch, no PBS). Returns acc int64[B]
        (device)."""
        if self.engine is None:
            raise RuntimeError("Model not compiled. Call compile() first.")
        B = qx_dev.shape[0]
        lo, hi = self.qparams.acc_range()
        centre = (lo + hi) // 2      # |acc - centre| <= (hi - lo) / 2 + 1 fits msg_bits
        return self.engine.score(qx_dev, self._w_dev, self.qparams.cst, centre, self.enc_seed,
                                 self.next_id0(B * qx_dev.shape[1]))

    def predict_encrypted(self, X, threshold: float | None = None):
        """Encrypted predict for features X [B, D] (numpy). Returns float64
        scores and, if a threshold is given, below[b] = score < threshold
        decided under encryption by the bootstrapped sign extraction. Without
        a threshold only the leveled circuit runs (no key switch or bootstrap),
        as in the reference, and below is all zeros."""
        import torch
        X = np.asarray(X)
        if X.ndim == 1:
            X = X.reshape(1, -1)
        Xd = torch.from_numpy(np.ascontiguousarray(X)).to(self.engine.device)
        qx = self.quantize_dev(Xd)
        if threshold is None:
            acc = self.encrypted_score(qx)
            below = None
        else:
            acc, below = self.encrypted_acc(qx, threshold_int(self.qparams, threshold))
        scores = np.float64(self.qparams.out_scale) * acc.cpu().numpy().astype(np.float64)
        b = below.cpu().numpy() if below is not None else np.zeros(len(scores), np.int64)
        return scores, b

    def clear_acc(self, X) -> np.ndarray:
        """Quantized integer accumulators in the clear (host): Concrete's
        _inference on quantize(X), q_x @ q_w - zp * sum(q_w) + q_b."""
        X = np.atleast_2d(np.asarray(X))
        qp = self.qparams
        q = np.clip(np.rint(X.astype(np.float64) / qp.s_x + qp.zp_x), qp.qmin, qp.qmax).astype(np.int64)
        return q @ np.asarray(qp.q_w, dtype=np.int64) + np.int64(qp.cst)

    def predict_clear(self, X) -> np.ndarray:
        """Concrete's fhe="disable" path: quantized integer inference in the clear (host)."""
        return np.float64(self.qparams.out_scale) * self.clear_acc(X).astype(np.float64)
