"""Encrypted document corpus: documents persisted as seeded LWE ciphertexts.

SURVEY.md §8f-1. In the reference, ``EncryptedDocument.encrypted_embedding``
holds the PLAINTEXT PCA vector (batch_operations.py:175-178; the
``model_version`` field, encrypted_storage.py:26, is never used) and every
compare re-quantizes the product ``q (.) d`` in the clear. This module adds the
opt-in mode where documents are encrypted once, at insert time, and never
decrypted by the search:

  * each document d is quantized on its own, ``dq = E.quant(d)`` (symmetric
    signed ``n_e``-bit uniform quantizer, Concrete-ML's ``is_symmetric=True``
    calibration), and its D values are encrypted as seeded
    LWEs (fhe_encrypt_seeded_batch): one body word per feature plus a 64-bit
    stream id, the masks regenerated from a public mask key;
  * a clear query q is quantized the same way, ``qq = E.quant(q)``, and folded
    into the model's quantized weights: ``W_j = q_w[j] * qq_j``;
  * the server computes ``acc = sum_j W_j * dq_j + q_b'`` homomorphically
    (fhe_compare_seeded_batch: masks regenerated in registers, leveled dot,
    sign extraction of ``acc - T``), ``q_b' = rint(b / s')``, and the score
    is ``s' * acc`` with ``s' = (s_e * s_e) * s_w``.

This is the bilinear quantisation of the same fitted LinearRegression: the
reference quantizes the product (a non-linear function of an encrypted d),
which no leveled circuit over encrypted documents can reproduce. Scores
therefore differ from the plaintext-store mode by quantisation error; the
parity bar for this mode is bit-exactness against its restatement
(oracle/quant_ref.py, ``corpus_*``), checked on the GPU in
tests/test_gpu_corpus.py.

Stored payload (EncryptedDocument with ``model_version == PAYLOAD_VERSION``):
``encrypted_embedding`` is a uint64 vector
    [MAGIC, 1, D, P0, id0, mask key (4 words), k*N, body_0 .. body_{D-1}]
where P0 is the encoding width the bodies were encrypted at (Delta =
2^(64 - P0)) and feature j uses stream id ``id0 + j``.
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass

import numpy as np

from .model import QuantParams
from .params import SchemeParams, params_for_bits

PAYLOAD_VERSION = "fheicp-seeded-lwe-v1"
MAGIC = int.from_bytes(b"FHEICPCT", "little")
HEADER_WORDS = 10


# ---------------------------------------------------------------- quantizer --
@dataclass
class CorpusQuant:
    """Bilinear quantisation of a fitted linear model for encrypted documents."""
    model: QuantParams
    n_e: int
    s_e: float

    @classmethod
    def calibrate(cls, model: QuantParams, embeddings, n_e: int | None = None) -> "CorpusQuant":
        """Symmetric signed n_e-bit scale from max|v| of calibration embeddings
        (concrete-ml UniformQuantizer, is_symmetric=True)."""
        n_e = int(model.n_bits if n_e is None else n_e)
        m = float(np.max(np.abs(np.asarray(embeddings, dtype=np.float64))))
        s = m / float(2 ** (n_e - 1) - 1) if m > 0 else 1.0
        return cls(model, n_e, s)

    @property
    def qmin(self) -> int:
        return -(2 ** (self.n_e - 1))

    @property
    def qmax(self) -> int:
        return 2 ** (self.n_e - 1) - 1

    @property
    def out_scale(self) -> float:
        return float((np.float64(self.s_e) * np.float64(self.s_e)) * np.float64(self.model.s_w))

    @property
    def q_b(self) -> int:
        return int(np.rint(np.float64(self.model.intercept) / np.float64(self.out_scale)))

    def quant(self, v) -> np.ndarray:
        """clip(rint(v / s_e), qmin, qmax) in float64 (host; queries)."""
        q = np.rint(np.asarray(v, dtype=np.float64) / np.float64(self.s_e))
        return np.clip(q, self.qmin, self.qmax).astype(np.int64)

    def weights(self, qq) -> np.ndarray:
        return np.asarray(self.model.q_w, dtype=np.int64) * np.asarray(qq, dtype=np.int64)

    def acc_range(self, W) -> tuple[int, int]:
        W = np.asarray(W, dtype=np.int64)
        lo = int(np.minimum(W * self.qmin, W * self.qmax).sum()) + self.q_b
        hi = int(np.maximum(W * self.qmin, W * self.qmax).sum()) + self.q_b
        return lo, hi

    @staticmethod
    def bits_for(lo: int, hi: int) -> int:
        """Two's-complement width holding acc - T for any clamped T in [lo, hi+1]."""
        return int(math.ceil(math.log2(hi - lo + 2))) + 1

    def worst_msg_bits(self) -> int:
        """P0: the width of every query's accumulator (|qq_j| <= 2^(n_e-1))."""
        qw = np.abs(np.asarray(self.model.q_w, dtype=np.int64))
        bound = int(qw.sum()) * 4 ** (self.n_e - 1) + abs(self.q_b)
        return self.bits_for(-bound, bound)

    def threshold_int(self, lo: int, hi: int, t: float) -> int:
        """Smallest a in [lo, hi+1] with float64(out_scale * a) >= t."""
        s = np.float64(self.out_scale)
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

    def to_dict(self) -> dict:
        return {"n_e": int(self.n_e), "s_e": float(self.s_e)}


# ------------------------------------------------------------------ payload --
def pack_payload(body_row, id0: int, P0: int, mask_key, big: int) -> np.ndarray:
    body_row = np.asarray(body_row, dtype=np.uint64).reshape(-1)
    mk = np.ascontiguousarray(mask_key, dtype=np.uint32).view(np.uint64)
    head = np.array([MAGIC, 1, body_row.size, P0, np.uint64(id0)], dtype=np.uint64)
    return np.concatenate([head, mk, np.array([big], np.uint64), body_row])


def unpack_payload(arr) -> dict:
    a = np.asarray(arr)
    if a.dtype != np.uint64 or a.ndim != 1 or a.size < HEADER_WORDS or int(a[0]) != MAGIC:
        raise ValueError("not an fheicp seeded-LWE payload")
    if int(a[1]) != 1:
        raise ValueError(f"unsupported payload version {int(a[1])}")
    D = int(a[2])
    if a.size != HEADER_WORDS + D:
        raise ValueError(f"payload holds {a.size - HEADER_WORDS} bodies, header says {D}")
    return {"D": D, "P0": int(a[3]), "id0": int(a[4]), "mask_key": a[5:9].copy().view(np.uint32),
            "big": int(a[9]), "body": a[HEADER_WORDS:].copy()}


# ------------------------------------------------------------------- engine --
class EncryptedCorpus:
    """GPU side of the encrypted-corpus mode: own context (parameters sized for
    P0), keys, the public mask key and the secret noise key."""

    def __init__(self, cq: CorpusQuant, scheme: SchemeParams | None = None):
        self.cq = cq
        self.P0 = cq.worst_msg_bits()
        self.scheme = scheme if scheme is not None else params_for_bits(self.P0)
        if self.scheme.msg_bits != self.P0:
            self.scheme = self.scheme.with_msg_bits(self.P0)
        self.engine = None
        self.mask_key = None
        self._noise_key = None
        self._w_cache = {}

    def compile(self, key_seed: int | None = None, device: int = 0, keys: dict | None = None,
                mask_key=None, noise_seed: int | None = None):
        """Create the context, generate (key_seed) or import (keys) the secret
        keys. mask_key (8 x u32, public) defaults to fresh OS randomness; the
        noise key is secret and session-local (noise_seed only for tests)."""
        from .engine import Engine
        self.engine = Engine(self.scheme, device)
        if keys is not None:
            self.engine.import_keys(keys)
        else:
            # 256-bit key from the OS CSPRNG; a key_seed is the 64-bit test form
            if key_seed is None:
                self.engine.keygen(key=os.urandom(32))
            else:
                self.engine.keygen(seed=int(key_seed))
        self.mask_key = (np.frombuffer(os.urandom(32), np.uint32).copy() if mask_key is None
                         else np.ascontiguousarray(mask_key, dtype=np.uint32).copy())
        self._noise_key = (np.frombuffer(os.urandom(32), np.uint32).copy() if noise_seed is None
                           else self.engine.key_from_seed(noise_seed))
        return self

    @property
    def compiled(self) -> bool:
        return self.engine is not None

    def _need(self):
        if self.engine is None:
            raise RuntimeError("Encrypted corpus not compiled. Call compile() first.")

    # ------------------------------------------------------------- client --
    def encrypt_docs(self, docs, id0=None):
        """docs f32/f64 [B, D] -> (bodies uint64 [B, D], id0 uint64 [B]) (host).
        id0 defaults to random 64-bit stream ids (features use id0 + j)."""
        import torch
        self._need()
        eng = self.engine
        docs = np.ascontiguousarray(docs)
        B, D = docs.shape
        if id0 is None:
            id0 = np.frombuffer(os.urandom(8 * B), np.uint64).copy()
        ids = np.ascontiguousarray(id0, dtype=np.uint64).reshape(B)
        dd = torch.from_numpy(docs).to(eng.device)
        eng.set_msg_bits(self.P0)
        dq = eng.quantize(dd, self.cq.s_e, 0, self.cq.qmin, self.cq.qmax)
        body = eng.encrypt_seeded(dq, self.mask_key, self._noise_key, eng.to_dev(ids))
        return body.cpu().numpy().view(np.uint64), ids

    def payloads(self, bodies, ids):
        big = self.scheme.k * self.scheme.N
        return [pack_payload(bodies[i], int(ids[i]), self.P0, self.mask_key, big) for i in range(len(ids))]

    def check_payload(self, pl: dict) -> None:
        if pl["P0"] != self.P0 or pl["big"] != self.scheme.k * self.scheme.N:
            raise ValueError("payload was encrypted under different parameters")
        if not np.array_equal(pl["mask_key"], self.mask_key):
            raise ValueError("payload was encrypted under a different mask key")

    def decrypt_docs(self, bodies, ids) -> np.ndarray:
        """Quantized document values (the key holder's view; tests and
        compare_encrypted of two stored documents)."""
        self._need()
        eng = self.engine
        bodies = np.ascontiguousarray(bodies, dtype=np.uint64)
        B, D = bodies.shape
        eng.set_msg_bits(self.P0)
        ct = eng.expand_seeded(eng.to_dev(bodies), eng.to_dev(np.asarray(ids, np.uint64)), B, D, self.mask_key)
        return eng.decrypt(ct).cpu().numpy().reshape(B, D)

    # ------------------------------------------------------------- server --
    def query_plan(self, query, min_similarity: float):
        """Clear per-query constants: (W' device, cst, T, P). P is the
        query's own accumulator width; the 2^(P0 - P) rescale of the stored
        encoding is folded into W'."""
        qq = self.cq.quant(query)
        W = self.cq.weights(qq)
        lo, hi = self.cq.acc_range(W)
        P = max(4, min(self.P0, self.cq.bits_for(lo, hi)))
        T = self.cq.threshold_int(lo, hi, min_similarity) if min_similarity is not None else lo
        Wr = (W.astype(np.uint64) << np.uint64(self.P0 - P)).view(np.int64)
        return Wr, self.cq.q_b, T, P

    def compare(self, body_dev, id_dev, query, min_similarity: float | None):
        """-> (acc int64 [B], below int64 [B]) device tensors, and P used."""
        self._need()
        eng = self.engine
        Wr, cst, T, P = self.query_plan(query, min_similarity)
        eng.set_msg_bits(P)
        acc, below = eng.compare_seeded(body_dev, id_dev, self.mask_key, eng.to_dev(Wr), cst, T)
        return acc, below, P

    def scores(self, acc) -> np.ndarray:
        return np.float64(self.cq.out_scale) * np.asarray(acc, dtype=np.float64)
