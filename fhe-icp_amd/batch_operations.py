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
bert_embeddings.py / dimension_reduction.py) is outside this package. As in
the reference (:62-64), a processor built without them creates
``BertEmbedder()`` and ``DimensionReducer.load(config.reducer_path)`` from the
reference's modules on ``sys.path`` (lazily, on the first text operation, so
``compare`` never needs BERT), and a processor built without a key manager
creates ``FHEKeyManager()`` (``BatchConfig.key_manager_default=False`` runs
standalone instead: no key manager, the model is trained and compiled here).
``search_vector`` takes an already reduced query.

The reference CLI (fhe_cli.py:32-40) builds ``BatchConfig(show_progress=True)``
and nothing else, so its knobs come from the environment: ``FHE_ICP_DIM`` and
``FHE_ICP_N_BITS`` (the model width and quantisation bits, reference: 128 and
8, batch_operations.py:86) and ``FHE_ICP_FHE`` (execute | simulate | disable;
the reference's compare/search call predict() in the clear, :233, :276).
"""
from __future__ import annotations

import gc
import hashlib
import logging
import os
from dataclasses import dataclass, field
from datetime import datetime
from typing import Dict, List, Optional, Tuple

import numpy as np

from encrypted_storage import DEFAULT_DIMS, EncryptedDocument, EncryptedDocumentStore
from fhe_similarity import FHESimilarityModel

logger = logging.getLogger(__name__)

FHE_MODES = ("execute", "simulate", "disable")
# which reducer produced a stored vector (BatchConfig.gpu_reducer)
REDUCER_KEY = "fheicp_reducer"
GPU_REDUCER = "gpu-pca-f64"
# which encoder embedded it (BatchConfig.gpu_embedder; absent: the reference's
# torch fp32 forward), e.g. "hip-bert-f32" (fheicp.bert.GpuBert.provenance)
EMBEDDER_KEY = "fheicp_embedder"


@dataclass
class BatchConfig:
    # reference fields (batch_operations.py:26-40)
    batch_size: int = 10
    max_memory_mb: int = 4000
    checkpoint_interval: int = 50
    show_progress: bool = True
    force_gc: bool = True
    # engine fields
    fhe: str = field(default_factory=lambda: os.environ.get("FHE_ICP_FHE", "execute"))
    # the reference hard-codes 128 and 8 (:86); --dim / --n-bits knobs of an
    # unchanged fhe_cli via FHE_ICP_DIM / FHE_ICP_N_BITS
    input_dim: int = field(default_factory=lambda: int(os.environ.get("FHE_ICP_DIM", "128")))
    n_bits: int = field(default_factory=lambda: int(os.environ.get("FHE_ICP_N_BITS", "8")))
    reducer_path: str = "pca_reducer_128.pkl"  # DimensionReducer.load (:63)
    # run a fitted PCA DimensionReducer on the GPU (fheicp.pca, §8f-4).
    # Tolerance: the GPU transform accumulates in f64 and rounds once to
    # float32; sklearn's float32 BLAS sums in an unspecified order. The two
    # agree to ~1e-5 relative, so a feature can land on the other side of an
    # input-quantizer rounding boundary (one quantization level, hence a
    # different accumulator) than in a CPU-reduced store. Documents written
    # with gpu_reducer carry metadata[REDUCER_KEY] = GPU_REDUCER; searches and
    # compares refuse to mix the two reducers (ValueError) unless
    # allow_mixed_reducers, and are bit-exact within one reducer's vectors.
    gpu_reducer: bool = False
    allow_mixed_reducers: bool = False
    # run the BERT encoder of the default BertEmbedder in libfheicp
    # (fheicp.bert, §8f-4) instead of the reference's torch fp32 forward:
    # gpu_embedder_precision "f32" (the reference's arithmetic on the f32
    # MFMA, another summation order) or "bf16". Not bit-equal to torch, so
    # the same contract as gpu_reducer: stored vectors carry
    # metadata[EMBEDDER_KEY] = the encoder's provenance, and scores never mix
    # encoders (ValueError) unless allow_mixed_embedders.
    gpu_embedder: bool = False
    gpu_embedder_precision: str = "f32"
    allow_mixed_embedders: bool = False
    key_manager_default: bool = True  # no key_manager given: FHEKeyManager() as the reference (:64)
    device: int = 0
    model_path: Optional[str] = None  # fheicp.persist file: load instead of retrain (§8f-2)
    seed: Optional[int] = None      # training-data seed when no model_path
    key_seed: Optional[int] = None  # keygen seed (None: os.urandom)
    search_chunk: int = 1 << 16     # pairs per fused GPU launch sequence
    # encrypted-corpus mode (§8f-1, fheicp.corpus): documents are stored as
    # seeded LWE ciphertexts and searched without decryption (bilinear
    # quantisation; opt-in because its scores differ from the reference's)
    store_ciphertexts: bool = False
    embedding_bits: Optional[int] = None     # n_e (default: n_bits)
    embedding_scale: Optional[float] = None  # s_e (default: calibrated on training embeddings)
    corpus_path: Optional[str] = None        # fheicp.persist corpus file: load, or save after creation
    # the secret keys of model_path / corpus_path files are Fernet-wrapped
    # under this password (default: $FHE_MASTER_PASSWORD, fheicp.persist);
    # without one, saving a corpus needs allow_plaintext_secrets=True
    password: Optional[str] = None
    allow_plaintext_secrets: bool = False

    def __post_init__(self):
        if self.batch_size < 1:
            raise ValueError("batch_size must be >= 1")
        if self.max_memory_mb < 100:
            raise ValueError("max_memory_mb must be >= 100")
        if self.fhe not in FHE_MODES:
            raise ValueError(f"fhe must be one of {FHE_MODES}")
        if self.search_chunk < 1:
            raise ValueError("search_chunk must be >= 1")
        if self.input_dim < 1 or not 2 <= self.n_bits <= 16:
            raise ValueError("input_dim must be >= 1 and n_bits in [2, 16]")
        if self.gpu_embedder_precision not in ("f32", "bf16"):
            raise ValueError("gpu_embedder_precision must be 'f32' or 'bf16'")


def _world():
    """(world size, rank) of the torch.distributed group, (1, 0) without one."""
    try:
        import torch
        if torch.distributed.is_available() and torch.distributed.is_initialized():
            return torch.distributed.get_world_size(), torch.distributed.get_rank()
    except ImportError:  # pragma: no cover - torch is a hard dependency of the GPU path
        pass
    return 1, 0


class BatchProcessor:
    def __init__(self, embedder=None, reducer=None, key_manager=None,
                 storage: Optional[EncryptedDocumentStore] = None, config: Optional[BatchConfig] = None,
                 fhe_model: Optional[FHESimilarityModel] = None):
        self.embedder = embedder
        self.reducer = reducer
        self.config = config if config is not None else BatchConfig()
        if key_manager is None and self.config.key_manager_default:
            from key_management import FHEKeyManager
            key_manager = FHEKeyManager()
        self.key_manager = key_manager
        self.storage = storage if storage is not None else EncryptedDocumentStore()
        if self.config.input_dim not in (EncryptedDocument.allowed_dims or (self.config.input_dim,)):
            EncryptedDocument.allowed_dims = tuple(sorted(set(DEFAULT_DIMS) | {self.config.input_dim}))
        self._resident = None  # (host array identity, device tensor)
        self._resident_ct = None  # (host bodies, rank range, (device bodies, device ids))
        self.corpus_engine = None  # fheicp.corpus.EncryptedCorpus (store_ciphertexts)
        self.fhe_model = fhe_model
        if self.fhe_model is None:
            self._init_model()
        elif self.config.store_ciphertexts and self.config.fhe == "execute":
            self._init_corpus(self.fhe_model)
        if self.fhe_model is not None and EncryptedDocument.allowed_dims is not None and \
                self.fhe_model.input_dim not in EncryptedDocument.allowed_dims:
            EncryptedDocument.allowed_dims = tuple(sorted(set(EncryptedDocument.allowed_dims) |
                                                          {self.fhe_model.input_dim}))
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
        km_model = self._model_from_key_manager(needs_keys)
        if km_model is not None:
            m = km_model
        elif cfg.model_path and os.path.exists(cfg.model_path):
            m = FHESimilarityModel.load_compiled(cfg.model_path, device=cfg.device,
                                                 password=cfg.password) if needs_keys else None
            if m is None:
                from fheicp import persist
                from fheicp.sklearn import LinearRegression
                # the clear modes read only the quantisation: no password needed
                qp, _, _ = persist.load_model(cfg.model_path, keys=False)
                m = FHESimilarityModel(input_dim=len(qp.coef), n_bits=qp.n_bits, device=cfg.device)
                m.model = LinearRegression.from_quant_params(qp, device=cfg.device)
            if needs_keys and not m.compiled:
                m.compile(None, key_seed=cfg.key_seed)
        else:
            self._check_corpus_secret()
            m = FHESimilarityModel(input_dim=cfg.input_dim, n_bits=cfg.n_bits, device=cfg.device, seed=cfg.seed)
            X, _ = m.train()
            if needs_keys:
                m.compile(X[:10], key_seed=cfg.key_seed)
        self.fhe_model = m
        if cfg.store_ciphertexts and needs_keys:
            self._init_corpus(m)

    def _model_from_key_manager(self, needs_keys: bool):
        """The key manager's current key, when it holds fheicp key material
        (key_management.FHEKeyManager.store_keys): parameters and keys are
        loaded, not regenerated (§8f-2). None otherwise (a reference key
        manager, or a key written by the reference)."""
        km = self.key_manager
        if km is None or not hasattr(km, "load_key_material"):
            return None
        try:
            if not needs_keys:
                from fheicp.sklearn import LinearRegression
                qp, _, _ = km.load_key_material()
                m = FHESimilarityModel(input_dim=len(qp.coef), n_bits=qp.n_bits, device=self.config.device)
                m.model = LinearRegression.from_quant_params(qp, device=self.config.device)
                return m
            return km.load_compiled(device=self.config.device)
        except ValueError as e:  # no fheicp material under the current key
            logger.info("key manager: %s; training a new model", e)
            return None

    def _check_corpus_secret(self):
        """A corpus that will be saved needs a password for its secret keys
        (or the explicit plaintext opt-in): fail before the keygen, not after."""
        cfg = self.config
        if not (cfg.store_ciphertexts and cfg.fhe == "execute" and cfg.corpus_path) or os.path.exists(cfg.corpus_path):
            return
        from fheicp.persist import _password
        if _password(cfg.password) is None and not cfg.allow_plaintext_secrets:
            raise ValueError("saving the encrypted corpus needs a password (BatchConfig.password or "
                             "$FHE_MASTER_PASSWORD) or BatchConfig.allow_plaintext_secrets=True")

    def _init_corpus(self, m):
        """Load (config.corpus_path) or create the encrypted-corpus engine."""
        from fheicp import persist
        from fheicp.corpus import CorpusQuant, EncryptedCorpus
        cfg = self.config
        if cfg.corpus_path and os.path.exists(cfg.corpus_path):
            self.corpus_engine = persist.load_corpus(cfg.corpus_path, device=cfg.device, password=cfg.password)
            return
        self._check_corpus_secret()
        qp = m.model.quant_params
        if cfg.embedding_scale is not None:
            cq = CorpusQuant(qp, int(cfg.embedding_bits or qp.n_bits), float(cfg.embedding_scale))
        else:
            from fheicp.datagen import training_embeddings
            e1, e2 = training_embeddings(len(qp.coef), 1000, seed=0 if cfg.seed is None else cfg.seed)
            cq = CorpusQuant.calibrate(qp, np.concatenate([e1, e2]), cfg.embedding_bits)
        self.corpus_engine = EncryptedCorpus(cq).compile(key_seed=cfg.key_seed, device=cfg.device)
        if cfg.corpus_path:
            persist.save_corpus(cfg.corpus_path, self.corpus_engine, password=cfg.password,
                                allow_plaintext_secrets=cfg.allow_plaintext_secrets)

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
    def _upstream(self):
        """The embedder and reducer, created as the reference does on first
        use (:62-63): ``bert_embeddings.BertEmbedder()`` and
        ``dimension_reduction.DimensionReducer.load(config.reducer_path)``
        from the reference's modules on sys.path (with config.gpu_embedder the
        BertEmbedder mirror runs libfheicp's encoder)."""
        if self.embedder is None:
            from bert_embeddings import BertEmbedder
            cfg = self.config
            self.embedder = (BertEmbedder(gpu_encoder=True, gpu_precision=cfg.gpu_embedder_precision)
                             if cfg.gpu_embedder else BertEmbedder())
        if self.reducer is None:
            from dimension_reduction import DimensionReducer
            self.reducer = DimensionReducer.load(self.config.reducer_path)
        if self.config.gpu_reducer and not hasattr(self.reducer, "transform_dev"):
            from fheicp.pca import GpuPCA
            self.reducer = GpuPCA.from_reducer(self.reducer, device=self.config.device)
        return self.embedder, self.reducer

    def _embed(self, texts: List[str]) -> np.ndarray:
        embedder, reducer = self._upstream()
        return reducer.transform(embedder.get_embeddings_batch(texts))

    def _tags(self) -> Dict[str, Optional[str]]:
        """Provenance of the vectors this processor makes from text: the
        reducer (GPU PCA or not) and the encoder (None: torch fp32)."""
        embedder, _ = self._upstream()
        return {REDUCER_KEY: GPU_REDUCER if self.config.gpu_reducer else None,
                EMBEDDER_KEY: getattr(embedder, "provenance", None)}

    @staticmethod
    def _tagged(meta: List[Dict], tags: Dict[str, Optional[str]]) -> List[Dict]:
        set_ = {k: v for k, v in tags.items() if v is not None}
        return [dict(m, **set_) for m in meta] if set_ else meta

    def encrypt_documents(self, texts: List[str], doc_ids: Optional[List[str]] = None,
                          metadata: Optional[List[Dict]] = None) -> List[str]:
        """Embed, reduce and store documents (:120-204): one index rewrite per batch."""
        self._require_model()
        tags = self._tags()
        self._check_provenance(list(self.storage.index.keys()), tags)
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
            meta = self._tagged(metadata[s:e], tags)
            docs = self._make_documents(texts[s:e], doc_ids[s:e], vecs, key_id, meta)
            self.storage.save_many(docs)
            out.extend(d.doc_id for d in docs)
            if (s + self.config.batch_size) % self.config.checkpoint_interval == 0:
                self._maybe_gc()
        return out

    def _make_documents(self, texts, doc_ids, vecs, key_id, metadata) -> List[EncryptedDocument]:
        """Plaintext vectors as in the reference (:175-178), or, with
        store_ciphertexts, seeded-LWE payloads of the quantized vectors."""
        vecs = np.asarray(vecs).astype(np.float32)
        if self.corpus_engine is not None:
            from fheicp.corpus import PAYLOAD_VERSION
            bodies, ids = self.corpus_engine.encrypt_docs(vecs)
            payloads = self.corpus_engine.payloads(bodies, ids)
            version = PAYLOAD_VERSION
        else:
            payloads, version = list(vecs), "1.0"
        stamp = datetime.now().isoformat()
        return [EncryptedDocument(doc_id=doc_ids[i], content_hash=hashlib.sha256(texts[i].encode()).hexdigest(),
                                  timestamp=stamp, encrypted_embedding=payloads[i], model_version=version,
                                  key_id=key_id, metadata=metadata[i]) for i in range(len(doc_ids))]

    _CONFIG = object()

    def store_vectors(self, vecs: np.ndarray, doc_ids: List[str], texts: Optional[List[str]] = None,
                      metadata: Optional[List[Dict]] = None, reducer=_CONFIG,
                      embedder: Optional[str] = None) -> List[str]:
        """encrypt_documents for already reduced vectors (no embedder needed).

        ``reducer`` / ``embedder`` name where the vectors came from, for the
        provenance contract (default: the config's reducer, GPU_REDUCER under
        gpu_reducer; the reference's torch encoder); they are tagged and
        checked against the store as in encrypt_documents."""
        self._require_model()
        if reducer is BatchProcessor._CONFIG:
            reducer = GPU_REDUCER if self.config.gpu_reducer else None
        tags = {REDUCER_KEY: reducer, EMBEDDER_KEY: embedder}
        self._check_provenance(list(self.storage.index.keys()), tags)
        n = len(doc_ids)
        texts = texts if texts is not None else list(doc_ids)
        metadata = metadata if metadata is not None else [{} for _ in range(n)]
        key_id = self.key_manager.get_current_key() if self.key_manager is not None else None
        out: List[str] = []
        for s in range(0, n, self.config.batch_size):
            e = min(n, s + self.config.batch_size)
            meta = self._tagged(metadata[s:e], tags)
            docs = self._make_documents(texts[s:e], doc_ids[s:e], vecs[s:e], key_id, meta)
            self.storage.save_many(docs)
            out.extend(d.doc_id for d in docs)
        return out

    def _tag_of(self, doc_id: str, key: str):
        return self.storage.index[doc_id].get("metadata", {}).get(key)

    def _check_provenance(self, doc_ids, query_tags: Optional[Dict[str, Optional[str]]] = None):
        """The GPU-stage contract (BatchConfig.gpu_reducer, gpu_embedder): the
        vectors that meet in one score come from one reducer and one encoder.
        A GPU stage is not bit-equal to the CPU one it replaces, and a feature
        on the other side of an input-quantizer rounding boundary changes the
        accumulator; within one provenance every score is the oracle's.
        An untagged vector counts as the CPU stage (torch fp32 encoder, sklearn
        PCA). Stores written before round 4 are the exception: a BertEmbedder
        on a GPU then ran the HIP bf16 encoder without tagging, so vectors such
        a store holds have unknown encoder provenance (re-embed them, or accept
        the mix explicitly with allow_mixed_embedders)."""
        what = ((REDUCER_KEY, "dimension reducers", "the GPU and CPU PCA", "gpu_reducer", "allow_mixed_reducers"),
                (EMBEDDER_KEY, "embedders", "the HIP and torch BERT encoders", "gpu_embedder",
                 "allow_mixed_embedders"))
        for key, name, pair, knob, allow in what:
            if getattr(self.config, allow):
                continue
            seen = {self._tag_of(i, key) for i in doc_ids if i in self.storage.index}
            if query_tags is not None:
                seen.add(query_tags.get(key))
            if len(seen) > 1:
                raise ValueError(f"vectors from different {name} {sorted(map(str, seen))} would meet in one "
                                 f"score: {pair} differ at quantizer rounding boundaries "
                                 f"(BatchConfig.{knob}, {allow})")

    def compare_encrypted(self, doc_id1: str, doc_id2: str) -> float:
        self._require_model()
        self._check_provenance([doc_id1, doc_id2])
        d1, d2 = self.storage.load(doc_id1), self.storage.load(doc_id2)
        if self.storage.holds_ciphertexts() or d1.model_version != "1.0" or d2.model_version != "1.0":
            return self._compare_ciphertexts(d1, d2)
        a, b = d1.encrypted_embedding, d2.encrypted_embedding
        return float(self._predict((a * b).reshape(1, -1))[0])

    def _compare_ciphertexts(self, d1, d2) -> float:
        """Two stored ciphertexts: the key holder decrypts the first (the
        reference's single-party trust model) and runs it as the clear query
        against the second, which stays encrypted."""
        import torch
        from fheicp.corpus import unpack_payload
        c = self.corpus_engine
        if c is None:
            raise RuntimeError("ciphertext documents need BatchConfig(store_ciphertexts=True, fhe='execute')")
        p1, p2 = unpack_payload(d1.encrypted_embedding), unpack_payload(d2.encrypted_embedding)
        c.check_payload(p1)
        c.check_payload(p2)
        dq1 = c.decrypt_docs(p1["body"][None, :], [p1["id0"]])[0]
        query = np.float64(c.cq.s_e) * dq1.astype(np.float64)
        dev = c.engine.device
        body = torch.from_numpy(p2["body"][None, :].view(np.int64)).to(dev)
        ids = torch.from_numpy(np.array([p2["id0"]], np.uint64).view(np.int64)).to(dev)
        acc, _, _ = c.compare(body, ids, query, None)
        return float(c.scores(acc.cpu().numpy())[0])

    # ------------------------------------------------------------ search --
    def search_similar(self, query_text: str, top_k: int = 5, min_similarity: float = 0.5) -> List[Tuple[str, float]]:
        self._require_model()
        embedder, reducer = self._upstream()
        self._check_provenance(list(self.storage.index.keys()), self._tags())
        q = embedder.get_embedding(query_text)
        q = reducer.transform(np.asarray(q).reshape(1, -1))[0]
        return self.search_vector(q, top_k, min_similarity)

    def search_vector(self, query: np.ndarray, top_k: int = 5, min_similarity: float = 0.5) -> List[Tuple[str, float]]:
        """Top-k documents with score >= min_similarity for a reduced query vector."""
        m = self._require_model()
        if self.storage.holds_ciphertexts():
            return self._search_ciphertexts(query, top_k, min_similarity)
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
            if _world()[0] > 1:
                hits = self._search_clear_sharded(m, query, E, k, min_similarity)
            else:
                hits = self._search_clear(m, query, E, min_similarity)
        else:
            hits = self._search_gpu(m, query, E, k, min_similarity)
        out = [(ids[i], s) for i, s in hits]
        return out[:top_k]

    def _search_ciphertexts(self, query, top_k: int, t: float) -> List[Tuple[str, float]]:
        """Search over a store of seeded-LWE documents (fheicp.corpus): the
        corpus stays encrypted in HBM (one body word per feature); every rank
        of a torch.distributed group takes a contiguous range and the per-rank
        top-k meet in one all-gather, as in _search_gpu."""
        import torch
        from fheicp.search import sharded_topk
        c = self.corpus_engine
        if c is None:
            raise RuntimeError("ciphertext documents need BatchConfig(store_ciphertexts=True, fhe='execute')")
        ids, bodies, id0, head = self.storage.encrypted_corpus()
        if not ids:
            return []
        c.check_payload(head)
        query = np.asarray(query)
        if query.shape != (bodies.shape[1],):
            raise ValueError(f"query shape {query.shape} does not match corpus width {bodies.shape[1]}")
        k = len(ids) if top_k < 0 else min(int(top_k), len(ids))
        if k == 0:
            return []
        dist = torch.distributed.is_available() and torch.distributed.is_initialized()
        world = torch.distributed.get_world_size() if dist else 1
        rank = torch.distributed.get_rank() if dist else 0
        n = len(ids)
        lo, hi = rank * n // world, (rank + 1) * n // world
        eng = c.engine
        r = self._resident_ct
        if r is None or r[0] is not bodies or r[1] != (lo, hi):
            r = self._resident_ct = (bodies, (lo, hi), (
                torch.from_numpy(np.ascontiguousarray(bodies[lo:hi]).view(np.int64)).to(eng.device),
                torch.from_numpy(np.ascontiguousarray(id0[lo:hi]).view(np.int64)).to(eng.device)))
        bd, idd = r[2]
        accs, belows = [], []
        for s in range(0, hi - lo, self.config.search_chunk):
            e = min(hi - lo, s + self.config.search_chunk)
            acc, below, _ = c.compare(bd[s:e], idd[s:e], query, t)
            accs.append(acc)
            belows.append(below)
        if accs:
            acc, below = torch.cat(accs), torch.cat(belows)
        else:
            acc = torch.zeros(0, dtype=torch.int64, device=eng.device)
            below = torch.zeros(0, dtype=torch.int64, device=eng.device)
        oa, oi = sharded_topk(acc, below, k, lo, lambda a, b, kk, base: eng.topk(a, b, kk, base), world)
        oa, oi = oa.cpu().numpy(), oi.cpu().numpy()
        s = np.float64(c.cq.out_scale)
        hits = [(ids[int(i)], float(s * np.float64(a))) for a, i in zip(oa, oi) if i >= 0]
        return hits[:top_k]

    @staticmethod
    def _search_clear_sharded(m, query, E, k, t):
        """The clear search (fhe != "execute") under torch.distributed: each
        rank scores its contiguous document range, keeps its top-k by (acc
        desc, index asc), and the ranks meet in the same single all-gather
        as the encrypted search (fheicp.search.sharded_topk)."""
        import torch
        from fheicp.model import threshold_int
        from fheicp.search import host_topk, sharded_topk
        fm = m.model._fitted()
        world, rank = _world()
        n = E.shape[0]
        lo, hi = rank * n // world, (rank + 1) * n // world
        acc = fm.clear_acc(query[None, :] * E[lo:hi]) if hi > lo else np.zeros(0, np.int64)
        below = (acc < threshold_int(fm.qparams, t)).astype(np.int64)
        oa, oi = sharded_topk(torch.from_numpy(acc), torch.from_numpy(below), k, lo, host_topk, world)
        s = np.float64(fm.qparams.out_scale)
        return [(int(i), float(s * np.float64(a))) for a, i in zip(oa.tolist(), oi.tolist()) if i >= 0]

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
