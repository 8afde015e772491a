"""ORACLE (test infrastructure only) — CPU restatement of the reference's clear path.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this module, and only as the checker. The product path never routes through it.

What it restates
----------------
The reference's hot path ends in ``self.fhe_model.model.predict(X)`` on a
Concrete-ML ``LinearRegression(n_bits)`` (fhe_similarity.py:88-94, :151, :167;
batch_operations.py:226, :233, :273-284). The arithmetic lives in the
third-party wheel concrete-ml==1.9.0 (requirements.txt:5), which is NOT present
in /root/reference and cannot be installed offline. This file restates its
published algorithm for linear models:

* input quantizer: per-tensor, asymmetric, signed ``n_bits`` uniform quantizer
  calibrated on min/max of the full training X
  (concrete-ml ``quantization/quantizers.py`` UniformQuantizer,
  ``_compute_scale_zero_point``);
* weight quantizer: symmetric signed, ``scale = max|w| / (2^(n-1)-1)``, zp 0;
* bias: ``q_b = rint(b / (s_x * s_w))`` — no clipping;
* ``_inference``: ``acc = q_x @ q_w - zp_x * sum(q_w) + q_b`` in int64;
* dequantize: ``score = (s_x * s_w) * float64(acc)``.

Parity status: the reference's own tests pin nothing at this boundary
(SURVEY.md §8c). The only deterministic known-answer test is
/root/reference/test_fhe.py:13-60 (y = 2x, n_bits=8, x=7), which under this
restatement clips to exactly 12.0 (tests/test_oracle_quant.py). Everything else
is **parity unpinned** against a real Concrete-ML run, which is impossible here.

Search semantics follow batch_operations.py:268-284: float ``>=`` threshold,
stable sort by score descending (Python's sort is stable, so equal scores keep
index-insertion order), then ``[:top_k]``.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

import numpy as np


# --------------------------------------------------------------------------
# Synthetic data with fhe_similarity.py:34-70 semantics, but seeded.
# --------------------------------------------------------------------------
def prepare_training_data(input_dim: int, n_samples: int = 1000, similarity_type: str = "cosine",
                          seed: int = 0):
    """fhe_similarity.py:34-70 with ``np.random`` replaced by a seeded Generator.

    The reference draws from the global unseeded RNG; the call order is kept
    (randn, randn, rand, randn) so the distribution is the same.
    """
    rng = np.random.default_rng(seed)
    emb1 = rng.standard_normal((n_samples, input_dim)).astype(np.float32)
    emb1 = emb1 / np.linalg.norm(emb1, axis=1, keepdims=True)
    emb2 = rng.standard_normal((n_samples, input_dim)).astype(np.float32)
    emb2 = emb2 / np.linalg.norm(emb2, axis=1, keepdims=True)
    mask = rng.random(n_samples) > 0.5
    emb2[mask] = emb1[mask] + 0.2 * rng.standard_normal((int(mask.sum()), input_dim))
    emb2 = emb2 / np.linalg.norm(emb2, axis=1, keepdims=True)
    X = emb1 * emb2
    if similarity_type in ("cosine", "dot"):
        y = np.sum(emb1 * emb2, axis=1)
    elif similarity_type == "manhattan":
        y = -np.sum(np.abs(emb1 - emb2), axis=1)
        y = (y - y.min()) / (y.max() - y.min())
    else:
        raise ValueError(f"Unknown similarity type: {similarity_type}")
    return X, y


def make_corpus(input_dim: int, n_docs: int, seed: int, clip_set: bool = False):
    """Query + docs per SURVEY.md §8d: L2-normalised N(0,1)^D, half the docs
    correlated with the query (q + 0.2 N, renormalised). ``clip_set`` draws
    un-normalised N(0, 3^2) vectors instead, exercising input clipping like
    real PCA projections (batch_operations.py:166-178)."""
    rng = np.random.default_rng(seed)
    if clip_set:
        q = (3.0 * rng.standard_normal(input_dim)).astype(np.float32)
        docs = (3.0 * rng.standard_normal((n_docs, input_dim))).astype(np.float32)
        return q, docs
    q = rng.standard_normal(input_dim).astype(np.float32)
    q /= np.linalg.norm(q)
    docs = rng.standard_normal((n_docs, input_dim)).astype(np.float32)
    docs /= np.linalg.norm(docs, axis=1, keepdims=True)
    mask = rng.random(n_docs) > 0.5
    docs[mask] = q[None, :] + 0.2 * rng.standard_normal((int(mask.sum()), input_dim)).astype(np.float32)
    docs /= np.linalg.norm(docs, axis=1, keepdims=True)
    return q.astype(np.float32), docs.astype(np.float32)


# --------------------------------------------------------------------------
# Concrete-ML 1.9 uniform quantizer restatement.
# --------------------------------------------------------------------------
@dataclass
class UniformQuantizer:
    n_bits: int
    is_signed: bool
    is_symmetric: bool
    scale: float = 1.0
    zero_point: int = 0

    @property
    def offset(self) -> int:
        return 2 ** (self.n_bits - 1) if self.is_signed else 0

    @property
    def qmin(self) -> int:
        return -self.offset

    @property
    def qmax(self) -> int:
        return 2 ** self.n_bits - 1 - self.offset

    def calibrate(self, values: np.ndarray) -> "UniformQuantizer":
        values = np.asarray(values, dtype=np.float64)
        rmin, rmax = float(values.min()), float(values.max())
        if self.is_symmetric:
            self.zero_point = 0
            self.scale = max(abs(rmax), abs(rmin)) / float(2 ** self.n_bits - 1 - self.offset)
            if self.scale == 0.0:
                self.scale = 1.0
        else:
            if rmax - rmin == 0.0:
                self.scale = 1.0
                self.zero_point = int(round(-rmin)) if rmin != 0 else 0
            else:
                nlev = 2 ** self.n_bits - 1
                self.scale = (rmax - rmin) / nlev
                self.zero_point = int(np.round((rmax * (-self.offset) - (rmin * (nlev - self.offset)))
                                               / (rmax - rmin)))
        return self

    def quant(self, values) -> np.ndarray:
        """q = clip(rint(x / s + zp), qmin, qmax); rint is round-half-even, float64."""
        v = np.asarray(values, dtype=np.float64)
        q = np.rint(v / self.scale + self.zero_point)
        return np.clip(q, self.qmin, self.qmax).astype(np.int64)

    def dequant(self, q) -> np.ndarray:
        return self.scale * (np.asarray(q, dtype=np.float64) - np.float64(self.zero_point))


@dataclass
class QuantizedLinearParams:
    """Frozen parameters of a fitted quantized linear regressor (the fixture)."""
    n_bits: int
    coef: np.ndarray          # float64 [D]
    intercept: float
    s_x: float
    zp_x: int
    s_w: float
    q_w: np.ndarray           # int64 [D]
    q_b: int
    out_scale: float = field(init=False)

    def __post_init__(self):
        self.coef = np.asarray(self.coef, dtype=np.float64)
        self.q_w = np.asarray(self.q_w, dtype=np.int64)
        self.out_scale = float(np.float64(self.s_x) * np.float64(self.s_w))

    @property
    def qx_min(self) -> int:
        return -(2 ** (self.n_bits - 1))

    @property
    def qx_max(self) -> int:
        return 2 ** (self.n_bits - 1) - 1

    @property
    def const_term(self) -> int:
        """The clear constant -zp_x * sum(q_w) + q_b added to the encrypted dot."""
        return int(-self.zp_x * int(self.q_w.sum()) + self.q_b)

    def to_json(self) -> dict:
        return {"n_bits": self.n_bits, "coef": [float(c) for c in self.coef], "intercept": float(self.intercept),
                "s_x": float(self.s_x), "zp_x": int(self.zp_x), "s_w": float(self.s_w),
                "q_w": [int(v) for v in self.q_w], "q_b": int(self.q_b)}

    @classmethod
    def from_json(cls, d: dict) -> "QuantizedLinearParams":
        return cls(n_bits=d["n_bits"], coef=np.array(d["coef"]), intercept=d["intercept"], s_x=d["s_x"],
                   zp_x=d["zp_x"], s_w=d["s_w"], q_w=np.array(d["q_w"], dtype=np.int64), q_b=d["q_b"])


def fit_quantized_linear(X: np.ndarray, y: np.ndarray, n_bits: int) -> QuantizedLinearParams:
    """Concrete-ML LinearRegression(n_bits).fit: sklearn OLS then post-training quantisation."""
    from sklearn.linear_model import LinearRegression as SkLR
    sk = SkLR().fit(X, y)
    coef = np.asarray(sk.coef_, dtype=np.float64).reshape(-1)
    intercept = float(np.asarray(sk.intercept_).reshape(-1)[0])
    return quantize_fitted(X, coef, intercept, n_bits)


def quantize_fitted(X: np.ndarray, coef: np.ndarray, intercept: float, n_bits: int) -> QuantizedLinearParams:
    qin = UniformQuantizer(n_bits, is_signed=True, is_symmetric=False).calibrate(X)
    qw = UniformQuantizer(n_bits, is_signed=True, is_symmetric=True).calibrate(coef)
    q_w = qw.quant(coef)
    q_b = int(np.rint(np.float64(intercept) / (np.float64(qin.scale) * np.float64(qw.scale))))
    return QuantizedLinearParams(n_bits=n_bits, coef=coef, intercept=intercept, s_x=qin.scale,
                                 zp_x=qin.zero_point, s_w=qw.scale, q_w=q_w, q_b=q_b)


def quantize_input(params: QuantizedLinearParams, X) -> np.ndarray:
    q = UniformQuantizer(params.n_bits, True, False, params.s_x, params.zp_x)
    return q.quant(X)


def accumulate(params: QuantizedLinearParams, q_x: np.ndarray) -> np.ndarray:
    """Concrete-ML ``_inference``: int64 q_x @ q_w - zp * sum(q_w) + q_b."""
    q_x = np.asarray(q_x, dtype=np.int64)
    return q_x @ params.q_w + np.int64(params.const_term)


def dequantize(params: QuantizedLinearParams, acc) -> np.ndarray:
    return np.float64(params.out_scale) * np.asarray(acc, dtype=np.float64)


def predict(params: QuantizedLinearParams, X) -> np.ndarray:
    """predict(X, fhe="disable") restated: quantize -> int64 dot -> dequantize."""
    X = np.atleast_2d(np.asarray(X))
    return dequantize(params, accumulate(params, quantize_input(params, X)))


def pair_features(query: np.ndarray, docs: np.ndarray) -> np.ndarray:
    """batch_operations.py:226 / :273 — element-wise product in the inputs' dtype
    (numpy promotion: a float64 query times float32 docs is float64)."""
    return np.asarray(query)[None, :] * np.asarray(docs)


def threshold_int(params: QuantizedLinearParams, t: float, lo: int, hi: int) -> int:
    """Smallest integer a in [lo, hi+1] with float64(out_scale * a) >= t.

    Since the dequantisation is monotone in a, ``score >= t`` (batch_operations.py:278)
    is exactly ``acc >= T``."""
    s = np.float64(params.out_scale)

    def ok(a: int) -> bool:
        return bool(s * np.float64(a) >= np.float64(t))

    if ok(lo):
        return lo
    if not ok(hi):
        return hi + 1
    a = int(math.ceil(t / float(s)))
    a = min(max(a, lo), hi)
    while a > lo and ok(a - 1):
        a -= 1
    while not ok(a):
        a += 1
    return a


def search(params: QuantizedLinearParams, query, docs, top_k: int, min_similarity: float, doc_ids=None):
    """batch_operations.py:240-284 semantics over an in-memory corpus."""
    X = pair_features(query, docs)
    scores = predict(params, X)
    ids = list(range(len(docs))) if doc_ids is None else list(doc_ids)
    sims = [(ids[i], float(scores[i])) for i in range(len(ids)) if scores[i] >= min_similarity]
    sims.sort(key=lambda x: x[1], reverse=True)
    return sims[:top_k]


def acc_bounds(params: QuantizedLinearParams):
    """Worst-case accumulator range over every representable q_x."""
    lo_terms = np.minimum(params.q_w * params.qx_min, params.q_w * params.qx_max)
    hi_terms = np.maximum(params.q_w * params.qx_min, params.q_w * params.qx_max)
    c = params.const_term
    return int(lo_terms.sum()) + c, int(hi_terms.sum()) + c


def message_bits(params: QuantizedLinearParams) -> int:
    """P: two's-complement width that holds acc - T for any clamped threshold T."""
    lo, hi = acc_bounds(params)
    rng = hi - lo
    return int(math.ceil(math.log2(rng + 2))) + 1


# --------------------------------------------------------------------------
# Encrypted-corpus mode. The reference has
# no such mode — its stored "encrypted_embedding" is the plaintext vector
# (batch_operations.py:175-178) — so this is a restatement of this build's
# own spec: documents and the query are quantized separately with one
# symmetric signed n_e-bit quantizer (Concrete-ML is_symmetric=True
# calibration), the product's quantisation becomes the product of the
# quantized values, and the bias moves to the scale (s_e * s_e) * s_w.
# --------------------------------------------------------------------------
def corpus_scale(embeddings, n_e: int) -> float:
    q = UniformQuantizer(n_e, is_signed=True, is_symmetric=True).calibrate(np.asarray(embeddings).reshape(-1))
    return q.scale


def corpus_quant(s_e: float, n_e: int, v) -> np.ndarray:
    return UniformQuantizer(n_e, True, True, s_e, 0).quant(v)


def corpus_out_scale(params: QuantizedLinearParams, s_e: float) -> float:
    return float((np.float64(s_e) * np.float64(s_e)) * np.float64(params.s_w))


def corpus_qb(params: QuantizedLinearParams, s_e: float) -> int:
    return int(np.rint(np.float64(params.intercept) / np.float64(corpus_out_scale(params, s_e))))


def corpus_accumulate(params: QuantizedLinearParams, s_e: float, n_e: int, query, docs) -> np.ndarray:
    """acc[b] = sum_j q_w[j] * qq_j * dq[b, j] + q_b' in int64."""
    qq = corpus_quant(s_e, n_e, query)
    dq = corpus_quant(s_e, n_e, np.atleast_2d(docs))
    return dq @ (params.q_w * qq) + np.int64(corpus_qb(params, s_e))


def corpus_bounds(params: QuantizedLinearParams, s_e: float, n_e: int, query):
    W = params.q_w * corpus_quant(s_e, n_e, query)
    qmin, qmax = -(2 ** (n_e - 1)), 2 ** (n_e - 1) - 1
    c = corpus_qb(params, s_e)
    return int(np.minimum(W * qmin, W * qmax).sum()) + c, int(np.maximum(W * qmin, W * qmax).sum()) + c


def corpus_worst_bits(params: QuantizedLinearParams, s_e: float, n_e: int) -> int:
    bound = int(np.abs(params.q_w).sum()) * 4 ** (n_e - 1) + abs(corpus_qb(params, s_e))
    return int(math.ceil(math.log2(2 * bound + 2))) + 1


def corpus_search(params: QuantizedLinearParams, s_e: float, n_e: int, query, docs, top_k: int,
                  min_similarity: float):
    """batch_operations.py:268-284 semantics (float >=, stable sort desc,
    [:top_k]) on the encrypted-corpus scores: list of (index, score)."""
    s = np.float64(corpus_out_scale(params, s_e))
    scores = s * corpus_accumulate(params, s_e, n_e, query, docs).astype(np.float64)
    sims = [(i, float(scores[i])) for i in range(len(scores)) if scores[i] >= min_similarity]
    sims.sort(key=lambda x: x[1], reverse=True)
    return sims[:top_k]
