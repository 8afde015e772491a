"""Seeded synthetic inputs with the reference's distributions.

training_pairs follows FHESimilarityModel._prepare_training_data
(fhe_similarity.py:34-70) — which draws from the unseeded global RNG — with a
seeded numpy Generator and the same draw order. corpus() builds the search
workload of SURVEY.md §8d: a query and documents that are L2-normalised
N(0, 1)^D, half of them correlated with the query (q + 0.2 N, renormalised).
BERT/PCA (bert_embeddings.py, dimension_reduction.py) are upstream of the hot
path and need a network download; they are out of scope.
"""
from __future__ import annotations

import numpy as np


def training_embeddings(input_dim: int, n_samples: int = 1000, seed: int = 0):
    """The (emb1, emb2) pairs behind training_pairs (same draws): calibration
    data of the encrypted-corpus quantizer (fheicp.corpus)."""
    rng = np.random.default_rng(seed)
    emb1 = rng.standard_normal((n_samples, input_dim)).astype(np.float32)
    emb1 = emb1 / np.linalg.norm(emb1, axis=1, keepdims=True)
    emb2 = rng.standard_normal((n_samples, input_dim)).astype(np.float32)
    emb2 = emb2 / np.linalg.norm(emb2, axis=1, keepdims=True)
    mask = rng.random(n_samples) > 0.5
    emb2[mask] = emb1[mask] + 0.2 * rng.standard_normal((int(mask.sum()), input_dim))
    emb2 = emb2 / np.linalg.norm(emb2, axis=1, keepdims=True)
    return emb1, emb2


def training_pairs(input_dim: int, n_samples: int = 1000, seed: int = 0, similarity_type: str = "cosine"):
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


def corpus(input_dim: int, n_docs: int, seed: int, query_seed: int | None = None):
    """(query f32 [D], docs f32 [n_docs, D]). With query_seed=None the query
    is the first draw of the seed's stream (one stream, as
    oracle.quant_ref.make_corpus); otherwise it comes from its own stream so
    every shard of a sharded corpus shares it while docs differ per seed."""
    rng = np.random.default_rng(seed)
    qrng = rng if query_seed is None else np.random.default_rng(query_seed)
    q = qrng.standard_normal(input_dim).astype(np.float32)
    q /= np.linalg.norm(q)
    docs = rng.standard_normal((n_docs, input_dim)).astype(np.float32)
    docs /= np.linalg.norm(docs, axis=1, keepdims=True)
    mask = rng.random(n_docs) > 0.5
    docs[mask] = q[None, :] + 0.2 * rng.standard_normal((int(mask.sum()), input_dim)).astype(np.float32)
    docs /= np.linalg.norm(docs, axis=1, keepdims=True)
    return q.astype(np.float32), docs.astype(np.float32)
