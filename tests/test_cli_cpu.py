"""CPU: an UNCHANGED reference fhe_cli drives the mirrors.

The reference CLI (/root/reference/fhe_cli.py) builds ``FHEKeyManager()``,
``EncryptedDocumentStore()`` and ``BatchProcessor(key_manager=...,
storage=..., config=BatchConfig(show_progress=True))`` (:26-40) and relies on
the processor to create the BERT embedder and the PCA reducer itself
(batch_operations.py:62-63). Its call sequence is restated here (the
reference module is not imported): ``keys generate`` (:43-48), ``encrypt``
(:72-104), ``compare`` (:151-172), ``search`` (:183-210), ``stats`` (:212-241).
BERT and PCA are replaced by stub ``bert_embeddings`` / ``dimension_reduction``
modules (the weights are not available offline); the model width and bits
come from ``FHE_ICP_DIM`` / ``FHE_ICP_N_BITS`` (C1: 8-dim, n_bits=4) and the
evaluation mode from ``FHE_ICP_FHE`` (``disable``: the reference's own
compare/search call predict() in the clear, batch_operations.py:233, :276).
Results are checked against the oracle's restatement of the same semantics.
"""
import hashlib
import sys
import types

import numpy as np
import pytest

from oracle import quant_ref as Q

DIM = 8


def _vec(text: str) -> np.ndarray:
    seed = int.from_bytes(hashlib.sha256(text.encode()).digest()[:8], "little")
    return np.random.default_rng(seed).normal(size=768).astype(np.float32)


@pytest.fixture
def cli_env(tmp_path, monkeypatch):
    bert = types.ModuleType("bert_embeddings")
    dimred = types.ModuleType("dimension_reduction")

    class BertEmbedder:
        created = 0

        def __init__(self, *a, **k):
            BertEmbedder.created += 1

        def get_embedding(self, text):
            return _vec(text)

        def get_embeddings_batch(self, texts, batch_size=8):
            return np.stack([_vec(t) for t in texts])

    class DimensionReducer:
        loaded = []

        def __init__(self, dim):
            self.W = np.random.default_rng(5).normal(size=(768, dim)).astype(np.float32)

        @classmethod
        def load(cls, path):
            cls.loaded.append(path)
            return cls(DIM)

        def transform(self, X):
            Y = np.asarray(X, dtype=np.float32) @ self.W
            return Y / np.linalg.norm(Y, axis=1, keepdims=True)

    bert.BertEmbedder = BertEmbedder
    dimred.DimensionReducer = DimensionReducer
    monkeypatch.setitem(sys.modules, "bert_embeddings", bert)
    monkeypatch.setitem(sys.modules, "dimension_reduction", dimred)
    monkeypatch.setenv("HOME", str(tmp_path))
    monkeypatch.setenv("FHE_MASTER_PASSWORD", "correct horse")
    monkeypatch.setenv("FHE_ICP_DIM", str(DIM))
    monkeypatch.setenv("FHE_ICP_N_BITS", "4")
    monkeypatch.setenv("FHE_ICP_FHE", "disable")
    monkeypatch.chdir(tmp_path)
    return BertEmbedder, DimensionReducer


def test_unchanged_cli_sequence(cli_env):
    BertEmbedder, DimensionReducer = cli_env
    from batch_operations import BatchConfig, BatchProcessor
    from encrypted_storage import EncryptedDocumentStore
    from key_management import FHEKeyManager

    # FHEDocumentCLI.__init__ (:26-30) and `keys generate` (:43-48)
    key_manager = FHEKeyManager()
    storage = EncryptedDocumentStore()
    key_info = key_manager.generate_keys(None)
    assert key_info["key_id"] and key_info["created"]
    assert key_manager.get_current_key() == key_info["key_id"]
    assert list(key_manager.list_keys()) == [key_info["key_id"]]

    # _get_processor (:32-40)
    processor = BatchProcessor(key_manager=key_manager, storage=storage, config=BatchConfig(show_progress=True))
    assert processor.fhe_model is not None
    assert processor.fhe_model.input_dim == DIM and processor.fhe_model.n_bits == 4
    assert BertEmbedder.created == 0           # created on first use, not for compare

    # `encrypt` x 3 (:72-104)
    texts = {"doc1": "encrypted search over documents", "doc2": "searching encrypted documents",
             "doc3": "a recipe for lemon cake"}
    for doc_id, text in texts.items():
        doc_ids = processor.encrypt_documents([text], doc_ids=[doc_id], metadata=[{"tags": ["t"]}])
        assert doc_ids == [doc_id]
        assert processor.storage.index[doc_ids[0]]["size_bytes"] > 0
    assert DimensionReducer.loaded == ["pca_reducer_128.pkl"]     # batch_operations.py:63

    # the oracle's view of the same model and documents
    qp = Q.QuantizedLinearParams.from_json(processor.fhe_model.model.quant_params.to_dict())
    red = DimensionReducer(DIM)
    E = {k: red.transform(_vec(t)[None, :])[0] for k, t in texts.items()}

    # `compare doc1 doc2` (:151-172)
    similarity = processor.compare_encrypted("doc1", "doc2")
    assert similarity == float(Q.predict(qp, (E["doc1"] * E["doc2"]).reshape(1, -1))[0])

    # `search` (:183-210), float >= threshold, stable sort, slice
    q = red.transform(_vec("encrypted documents")[None, :])[0]
    docs = np.stack([E[k] for k in texts])
    for top_k, min_sim in ((5, 0.0), (1, -10.0), (5, 10.0)):
        results = processor.search_similar("encrypted documents", top_k=top_k, min_similarity=min_sim)
        assert results == Q.search(qp, q, docs, top_k, min_sim, doc_ids=list(texts))
        for doc_id, _ in results:
            assert storage.index.get(doc_id, {})["metadata"] == {"tags": ["t"]}

    # `stats` (:212-241)
    assert storage.get_stats()["total_documents"] == 3
    assert processor.get_memory_stats()["max_mb"] == 4000

    # a second CLI process: the model comes from the key manager, not a retrain
    p2 = BatchProcessor(key_manager=FHEKeyManager(), storage=EncryptedDocumentStore(),
                        config=BatchConfig(show_progress=True))
    assert p2.fhe_model.model.quant_params.to_dict() == processor.fhe_model.model.quant_params.to_dict()
    assert p2.compare_encrypted("doc1", "doc2") == similarity


def test_cli_without_keys_reports_no_model(cli_env):
    """`compare` before `keys generate`: fhe_model is None (fhe_cli.py:155-158)."""
    from batch_operations import BatchConfig, BatchProcessor
    from encrypted_storage import EncryptedDocumentStore
    from key_management import FHEKeyManager
    p = BatchProcessor(key_manager=FHEKeyManager(), storage=EncryptedDocumentStore(),
                       config=BatchConfig(show_progress=True))
    assert p.fhe_model is None
    # a processor given no key manager creates one, as the reference (:64)
    p2 = BatchProcessor(storage=EncryptedDocumentStore(), config=BatchConfig(show_progress=True))
    assert isinstance(p2.key_manager, FHEKeyManager) and p2.fhe_model is None


def test_env_knobs_validate(monkeypatch):
    from batch_operations import BatchConfig
    monkeypatch.setenv("FHE_ICP_DIM", "32")
    monkeypatch.setenv("FHE_ICP_N_BITS", "6")
    c = BatchConfig()
    assert (c.input_dim, c.n_bits) == (32, 6)
    monkeypatch.setenv("FHE_ICP_N_BITS", "1")
    with pytest.raises(ValueError):
        BatchConfig()
    monkeypatch.setenv("FHE_ICP_N_BITS", "8")
    monkeypatch.setenv("FHE_ICP_FHE", "gpu")
    with pytest.raises(ValueError):
        BatchConfig()
