"""BatchProcessor over the MI355X engine (mirror of the reference module).

Same names, arguments, results and errors as the reference's
``batch_operations`` (batch_operations.py:26-318): ``BatchConfig``,
``BatchProcessor.encrypt_documents / compare_encrypted / search_similar /
get_memory_stats``, RuntimeError while no model is initialised (:135-136,
:217-218, :255-256). What changes is the search: the reference loads,
unpickles and predicts one document at a time (:268-279); here the corpus is
stacked once (``EncryptedDocumentStore.corpus``), kept resident in HBM, and
every (query, doc) pair goes through the fused GPU path

    pair product + quantize -> encrypt -> leveled dot -> bit extraction
    (the encrypted ``score >= min_similarity`` bit, :278) -> decrypt -> top-k

with, under torch.distributed, one contiguous document range per rank and a
single all-gather of the per-rank top-k (fheicp.search). Results equal the
reference's: float ``>=`` threshold, stable descending sort, ``[:top_k]``
(:282-284).

The upstream text -> vector stage (BertEmbedder + DimensionReducer,
bert_embeddings.py / dimension_reduction.py) is outside this package: pass
objects with ``get_embedding(text)`` / ``get_embeddings_batch(texts)`` and
``transform(X)``; ``search_vector`` takes an already reduced query.
"""
from __future__ import annotations

import gc
import hashlib
import logging
import os
from dataclasses import dataclass
from datetime import datetime
from typing import Dict, List, Optional, Tuple

import numpy as np

from encrypted_storage import DEFAULT_DIMS, EncryptedDocument, EncryptedDocumentStore
from fhe_similarity import FHESimilarityModel

logger = logging.getLogger(__name__)

FHE_MODES = ("execute", "simulate", "disable")


@dataclass
class BatchConfig:
    # reference fields (batch_operations.py:26-40)
    batch_size: int = 10
    max_memory_mb: int = 4000
    checkpoint_interval: int = 50
    show_progress: bool = True
    force_gc: bool = True
    # engine fields
    fhe: str = "execute"            # how compare/search evaluate the model
    input_dim: int = 128            # the reference hard-codes 128 (:86)
    n_bits: int = 8                 # and 8 (:86)
    device: int = 0
    model_path: Optional[str] = None  # fheicp.persist file: load instead of retrain (§8f-2)
    seed: Optional[int] = None      # training-data seed when no model_path
    key_seed: Optional[int] = None  # keygen seed (None: os.urandom)
    search_chunk: int = 1 << 16     # pairs per fused GPU launch sequence

    def __post_init__(self):
        if self.batch_size < 1:
            raise ValueError("batch_size must be >= 1")
        if self.max_memory_mb < 100:
            raise ValueError("max_memory_mb must be >= 100")
        if self.fhe not in FHE_MODES:
            raise ValueError(f"fhe must be one of {FHE_MODES}")
        if self.search_chunk < 1:
            raise ValueError("search_chunk must be >= 1")


class BatchProcessor:
    def __init__(self, embedder=None, reducer=None, key_manager=None,
                 storage: Optional[EncryptedDocumentStore] = None, config: Optional[BatchConfig] = None,
                 fhe_model: Optional[FHESimilarityModel] = None):
        self.embedder = embedder
        self.reducer = reducer
        self.key_manager = key_manager
        self.storage = storage if storage is not None else EncryptedDocumentStore()
        self.config = config if config is not None else BatchConfig()
        if self.config.input_dim not in (EncryptedDocument.allowed_dims or (self.config.input_dim,)):
            EncryptedDocument.allowed_dims = tuple(sorted(set(DEFAULT_DIMS) | {self.config.input_dim}))
        self._resident = None  # (host array identity, device tensor)
        self.fhe_model = fhe_model
        if self.fhe_model is None:
            self._init_model()
        self.initial_memory = self._check_memory()

    # ------------------------------------------------------------- model --
    def _init_model(self):
        """Load (config.model_path) or train + compile the similarity model.

        As in the reference (:78-108), no model is created while the key
        manager has no current key. Unlike it, failures are not swallowed: a
        missing HIP library or GPU raises here instead of later."""
        if self.key_manager is not None and not self.key_manager.get_current_key():
            logger.info("no current key: model not initialised")
            return
        cfg = self.config
        needs_keys = cfg.fhe == "execute"
        if cfg.model_path and os.path.exists(cfg.model_path):
            m = FHESimilarityModel.load_compiled(cfg.model_path, device=cfg.device) if needs_keys else None
            if m is None:
                from fheicp import persist
                from fheicp.sklearn import LinearRegression
                qp, _, _ = persist.load_model(cfg.model_path)
                m = FHESimilarityModel(input_dim=len(qp.coef), n_bits=qp.n_bits, device=cfg.device)
                m.model = LinearRegression.from_quant_params(qp, device=cfg.device)
            if needs_keys and not m.compiled:
                m.compile(None, key_seed=cfg.key_seed)
        else:
            m = FHESimilarityModel(input_dim=cfg.input_dim, n_bits=cfg.n_bits, device=cfg.device, seed=cfg.seed)
            X, _ = m.train()
            if needs_keys:
                m.compile(X[:10], key_seed=cfg.key_seed)
        self.fhe_model = m

    def _require_model(self) -> FHESimilarityModel:
        if self.fhe_model is None:
            raise RuntimeError("No FHE model initialized. Generate keys first.")
        return self.fhe_model

    def _predict(self, X: np.ndarray) -> np.ndarray:
        est = self._require_model().model
        return est.predict(X, fhe=self.config.fhe)

    # ------------------------------------------------------------ memory --
    def _check_memory(self) -> float:
        try:
            import psutil
            return psutil.Process(os.getpid()).memory_info().rss / 2 ** 20
        except Exception:  # noqa: BLE001 - metrics only
            return 0.0

    def _maybe_gc(self):
        if self.config.force_gc:
            gc.collect()

    def get_memory_stats(self) -> Dict[str, float]:
        cur = self._check_memory()
        return {
            "initial_mb": self.initial_memory,
            "current_mb": cur,
            "used_mb": cur - self.initial_memory,
            "max_mb": self.config.max_memory_mb,
            "usage_percent": cur / self.config.max_memory_mb * 100,
        }

    # --------------------------------------------------------- documents --
    def _embed(self, texts: List[str]) -> np.ndarray:
        if self.embedder is None or self.reducer is None:
            raise RuntimeError("encrypt_documents/search_similar need an embedder and a reducer "
                               "(BERT + PCA are upstream of this package)")
        return self.reducer.transform(self.embedder.get_embeddings_batch(texts))

    def encrypt_documents(self, texts: List[str], doc_ids: Optional[List[str]] = None,
                          metadata: Optional[List[Dict]] = None) -> List[str]:
        """Embed, reduce and store documents (:120-204): one index rewrite per batch."""
        self._require_model()
        n = len(texts)
        if doc_ids is None:
            stamp = datetime.now().strftime("%Y%m%d_%H%M%S")
            doc_ids = [f"doc_{stamp}_{i}" for i in range(n)]
        metadata = metadata if metadata is not None else [{} for _ in range(n)]
        key_id = self.key_manager.get_current_key() if self.key_manager is not None else None
        out: List[str] = []
        for s in range(0, n, self.config.batch_size):
            e = min(n, s + self.config.batch_size)
            if self._check_memory() > self.config.max_memory_mb:
                self._maybe_gc()
            vecs = self._embed(texts[s:e])
            docs = [EncryptedDocument(doc_id=doc_ids[i], content_hash=hashlib.sha256(texts[i].encode()).hexdigest(),
                                      timestamp=datetime.now().isoformat(),
                                      encrypted_embedding=np.asarray(vecs[i - s]).astype(np.float32),
                                      key_id=key_id, metadata=metadata[i]) for i in range(s, e)]
            self.storage.save_many(docs)
            out.extend(d.doc_id for d in docs)
            if (s + self.config.batch_size) % self.config.checkpoint_interval == 0:
                self._maybe_gc()
        return out

    def compare_encrypted(self, doc_id1: str, doc_id2: str) -> float:
        self._require_model()
        a = self.storage.load(doc_id1).encrypted_embedding
        b = self.storage.load(doc_id2).encrypted_embedding
        return float(self._predict((a * b).reshape(1, -1))[0])

    # ------------------------------------------------------------ search --
    def search_similar(self, query_text: str, top_k: int = 5, min_similarity: float = 0.5) -> List[Tuple[str, float]]:
        self._require_model()
        if self.embedder is None or self.reducer is None:
            raise RuntimeError("search_similar needs an embedder and a reducer; use search_vector")
        q = self.embedder.get_embedding(query_text)
        q = self.reducer.transform(np.asarray(q).reshape(1, -1))[0]
        return self.search_vector(q, top_k, min_similarity)

    def search_vector(self, query: np.ndarray, top_k: int = 5, min_similarity: float = 0.5) -> List[Tuple[str, float]]:
        """Top-k documents with score >= min_similarity for a reduced query vector."""
        m = self._require_model()
        ids, E = self.storage.corpus()
        if not ids:
            return []
        query = np.asarray(query)
        if query.shape != (E.shape[1],):
            raise ValueError(f"query shape {query.shape} does not match corpus width {E.shape[1]}")
        k = len(ids) if top_k < 0 else min(int(top_k), len(ids))
        if k == 0:
            return []
        if self.config.fhe != "execute":
            hits = self._search_clear(m, query, E, min_similarity)
        else:
            hits = self._search_gpu(m, query, E, k, min_similarity)
        out = [(ids[i], s) for i, s in hits]
        return out[:top_k]

    @staticmethod
    def _search_clear(m, query, E, t):
        scores = m.model.predict(query[None, :] * E)
        keep = [(i, float(s)) for i, s in enumerate(scores) if s >= t]
        keep.sort(key=lambda x: x[1], reverse=True)
        return keep

    def _device_corpus(self, E, device):
        if self._resident is None or self._resident[0] is not E:
            import torch
            self._resident = (E, torch.from_numpy(np.ascontiguousarray(E)).to(device))
        return self._resident[1]

    def _search_gpu(self, m, query, E, k, t):
        import torch
        from fheicp.model import threshold_int
        from fheicp.search import sharded_topk
        fm = m.model._fitted()
        if not fm.compiled:
            raise RuntimeError("Model not compiled. Call compile() first.")
        eng = fm.engine
        dist = torch.distributed.is_available() and torch.distributed.is_initialized()
        world = torch.distributed.get_world_size() if dist else 1
        rank = torch.distributed.get_rank() if dist else 0
        n = E.shape[0]
        lo, hi = rank * n // world, (rank + 1) * n // world
        Ed = self._device_corpus(E, eng.device)
        qd = torch.from_numpy(np.ascontiguousarray(query)).to(eng.device)
        T = threshold_int(fm.qparams, t)
        accs, belows = [], []
        for s in range(lo, hi, self.config.search_chunk):
            e = min(hi, s + self.config.search_chunk)
            acc, below = fm.encrypted_acc(fm.quantize_dev(Ed[s:e], qd), T)
            accs.append(acc)
            belows.append(below)
        if accs:
            acc, below = torch.cat(accs), torch.cat(belows)
        else:  # more ranks than documents
            acc = torch.zeros(0, dtype=torch.int64, device=eng.device)
            below = torch.zeros(0, dtype=torch.int64, device=eng.device)
        topk_fn = lambda a, b, kk, base: eng.topk(a, b, kk, base)  # noqa: E731
        oa, oi = sharded_topk(acc, below, k, lo, topk_fn, world)
        oa, oi = oa.cpu().numpy(), oi.cpu().numpy()
        s = np.float64(fm.qparams.out_scale)
        return [(int(i), float(s * np.float64(a))) for a, i in zip(oa, oi) if i >= 0]
