"""CPU: the drop-in Python surface (fheicp.sklearn.LinearRegression and the
mirrors of fhe_similarity / batch_operations / encrypted_storage) on the
clear path, against the oracle. The encrypted path of the same objects is in
tests/test_gpu_dropin.py."""
import gzip
import json
import pickle
import pickletools

import numpy as np
import pytest

from oracle import quant_ref as Q

# Field order of the reference dataclass, read from encrypted_storage.py:19-28.
REF_FIELDS = ["doc_id", "content_hash", "timestamp", "encrypted_embedding", "model_version", "key_id", "metadata"]
# index.json entry keys, encrypted_storage.py:96-104.
REF_INDEX_KEYS = {"filename", "timestamp", "content_hash", "size_bytes", "model_version", "key_id", "metadata"}


# ------------------------------------------------------------- estimator --
def _data(D=16, seed=5):
    return Q.prepare_training_data(D, 1000, seed=seed)


@pytest.mark.parametrize("D,n_bits", [(8, 4), (16, 6), (32, 8)])
def test_linear_regression_matches_oracle(D, n_bits):
    from fheicp.sklearn import LinearRegression
    X, y = _data(D, seed=D)
    est = LinearRegression(n_bits=n_bits).fit(X, y)
    ref = Q.fit_quantized_linear(X, y, n_bits)
    assert est.quant_params.to_dict() == ref.to_json()
    np.testing.assert_array_equal(est.coef_, ref.coef)
    assert est.intercept_ == ref.intercept
    Xt = Q.pair_features(*Q.make_corpus(D, 200, seed=3))
    for mode in ("disable", "simulate"):
        np.testing.assert_array_equal(est.predict(Xt, fhe=mode), Q.predict(ref, Xt))
    assert est.score(X, y) > 0.9


def test_linear_regression_errors():
    from fheicp.sklearn import LinearRegression
    est = LinearRegression(n_bits=6)
    with pytest.raises(AttributeError):
        est.predict(np.zeros((1, 4)))
    X, y = _data(8)
    est.fit(X, y)
    with pytest.raises(ValueError):
        est.predict(X[:2], fhe="gpu")
    with pytest.raises(RuntimeError):
        est.predict(X[:2], fhe="execute")       # not compiled
    with pytest.raises(ValueError):
        LinearRegression(n_bits={"op_inputs": 6, "op_weights": 4})
    assert LinearRegression(n_bits={"op_inputs": 6, "op_weights": 6}).n_bits == 6


def test_compile_without_gpu_fails_loudly():
    """No CPU fallback: compile needs libfheicp on a GPU."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from fheicp.sklearn import LinearRegression
    X, y = _data(8)
    est = LinearRegression(n_bits=6).fit(X, y)
    with pytest.raises(Exception):
        est.compile(X[:10], key_seed=1)
    assert est.fhe_circuit is None


# ------------------------------------------------------ FHESimilarityModel --
def test_similarity_model_clear_and_persistence(tmp_path):
    from fhe_similarity import FHESimilarityModel
    m = FHESimilarityModel(input_dim=16, n_bits=6, seed=11)
    with pytest.raises(RuntimeError):
        m.predict_clear(np.zeros((1, 16)))
    with pytest.raises(RuntimeError):
        m.compile(np.zeros((1, 16)))
    X, y = m.train()
    rX, ry = Q.prepare_training_data(16, 1000, seed=11)
    np.testing.assert_array_equal(X, rX)
    ref = Q.fit_quantized_linear(rX, ry, 6)
    np.testing.assert_array_equal(m.predict_clear(X[:50]), Q.predict(ref, X[:50]))
    assert m.metrics["train_score"] > 0.9
    with pytest.raises(RuntimeError):
        m.predict_encrypted(X[:2])
    p = tmp_path / "model.pkl"
    m.save(str(p))
    with open(p, "rb") as f:
        raw = pickle.load(f)
    # the reference's keys (fhe_similarity.py:184-195) are all present
    assert {"input_dim", "n_bits", "similarity_type", "metrics", "model_params"} <= set(raw)
    m2 = FHESimilarityModel.load(str(p))
    np.testing.assert_array_equal(m2.predict_clear(X[:50]), m.predict_clear(X[:50]))
    assert not m2.compiled


def test_similarity_model_unknown_type():
    from fhe_similarity import FHESimilarityModel
    with pytest.raises(ValueError):
        FHESimilarityModel(input_dim=8, similarity_type="hamming", seed=1).train()


def test_persist_roundtrip(tmp_path):
    from fheicp import persist
    from fheicp.params import params_for_bits
    from fheicp.sklearn import LinearRegression
    X, y = _data(16)
    qp = LinearRegression(n_bits=6).fit(X, y).quant_params
    keys = {k: np.arange(5, dtype=np.uint64) * (i + 3) for i, k in enumerate(persist.KEY_NAMES)}
    keys["bsk"][0] = np.uint64(2 ** 64 - 1)
    path = str(tmp_path / "m.npz")
    persist.save_model(path, qp, params_for_bits(qp.msg_bits()), keys, allow_plaintext_secrets=True)
    qp2, sch, k2 = persist.load_model(path)
    assert qp2.to_dict() == qp.to_dict() and sch == params_for_bits(qp.msg_bits())
    for k in persist.KEY_NAMES:
        np.testing.assert_array_equal(k2[k], keys[k])
    persist.save_model(path, qp, sch)
    assert persist.load_model(path)[2] is None


def test_persist_wraps_secret_keys(tmp_path, monkeypatch):
    """Secret keys are Fernet-wrapped (PBKDF2 of the password, as the
    reference's key manager) and the file is mode 0600; no password -> refused
    unless explicitly opted out; a wrong password -> ValueError."""
    import os
    import stat
    from fheicp import persist
    from fheicp.params import params_for_bits
    from fheicp.sklearn import LinearRegression
    monkeypatch.delenv("FHE_MASTER_PASSWORD", raising=False)
    X, y = _data(16)
    qp = LinearRegression(n_bits=6).fit(X, y).quant_params
    rng = np.random.default_rng(3)
    keys = {"s_small": rng.integers(0, 2, 887).astype(np.uint64), "s_big": rng.integers(0, 2, 2048).astype(np.uint64),
            "bsk": rng.integers(0, 2 ** 63, 64, dtype=np.uint64), "ksk": rng.integers(0, 2 ** 63, 64, dtype=np.uint64)}
    sch = params_for_bits(qp.msg_bits())
    path = str(tmp_path / "m.npz")
    with pytest.raises(ValueError):
        persist.save_model(path, qp, sch, keys)
    persist.save_model(path, qp, sch, keys, password="pw")
    assert stat.S_IMODE(os.stat(path).st_mode) == 0o600
    raw = open(path, "rb").read()
    for k in ("s_small", "s_big"):
        assert keys[k].tobytes() not in raw
        assert np.packbits(keys[k].astype(np.uint8)).tobytes() not in raw
    with pytest.raises(ValueError):
        persist.load_model(path)                      # no password
    with pytest.raises(ValueError):
        persist.load_model(path, password="nope")
    monkeypatch.setenv("FHE_MASTER_PASSWORD", "pw")
    _, _, k2 = persist.load_model(path)
    for k in persist.KEY_NAMES:
        np.testing.assert_array_equal(k2[k], keys[k])


# ------------------------------------------------------- encrypted_storage --
def _doc(i, dim=128, **kw):
    from encrypted_storage import EncryptedDocument
    emb = np.random.default_rng(i).standard_normal(dim).astype(np.float32)
    return EncryptedDocument(doc_id=f"d{i}", content_hash=f"{i:064x}", timestamp=f"2025-01-01T00:00:{i:02d}",
                             encrypted_embedding=emb, **kw)


def test_document_format_matches_reference_layout():
    """Pickle class path and field order as encrypted_storage.py:19-28 (checked
    against the reference's source text: importing it was denied)."""
    from encrypted_storage import EncryptedDocument
    d = _doc(1, metadata={"k": "v"})
    payload = gzip.decompress(d.to_bytes())
    globals_ = [a for op, a, _ in pickletools.genops(payload) if op.name in ("GLOBAL", "STACK_GLOBAL", "SHORT_BINUNICODE")]
    assert "encrypted_storage" in globals_ and "EncryptedDocument" in globals_
    assert list(pickle.loads(payload).__dict__) == REF_FIELDS
    back = EncryptedDocument.from_bytes(d.to_bytes())
    assert back.doc_id == "d1" and back.metadata == {"k": "v"} and back.model_version == "1.0"
    np.testing.assert_array_equal(back.encrypted_embedding, d.encrypted_embedding)


def test_document_validation():
    from encrypted_storage import EncryptedDocument
    with pytest.raises(TypeError):
        EncryptedDocument("a", "h", "t", [1.0] * 128)
    with pytest.raises(ValueError):
        EncryptedDocument("a", "h", "t", np.zeros((2, 64), np.float32))
    with pytest.raises(ValueError):
        EncryptedDocument("a", "h", "t", np.zeros(16, np.float32))
    old = EncryptedDocument.allowed_dims
    try:
        EncryptedDocument.allowed_dims = None
        EncryptedDocument("a", "h", "t", np.zeros(16, np.float32))
    finally:
        EncryptedDocument.allowed_dims = old


def test_store_roundtrip_and_errors(tmp_path):
    from encrypted_storage import EncryptedDocumentStore
    st = EncryptedDocumentStore(str(tmp_path))
    st.save(_doc(0, key_id="k0", metadata={"cat": "AI"}))
    st.save_many([_doc(i, metadata={"cat": "ML" if i % 2 else "AI"}) for i in range(1, 5)])
    idx = json.loads((tmp_path / "index.json").read_text())
    assert list(idx) == ["d0", "d1", "d2", "d3", "d4"]
    assert all(set(v) == REF_INDEX_KEYS for v in idx.values())
    assert idx["d0"]["filename"] == "d0.enc" and idx["d0"]["key_id"] == "k0"
    st2 = EncryptedDocumentStore(str(tmp_path))   # reopen from disk
    assert [d["doc_id"] for d in st2.list_documents()] == ["d0", "d1", "d2", "d3", "d4"]
    assert st2.search_by_metadata("cat", "AI") == ["d0", "d2", "d4"]
    assert st2.search_by_metadata("missing", None) == []
    ids, E = st2.corpus()
    assert ids == ["d0", "d1", "d2", "d3", "d4"] and E.shape == (5, 128) and E.dtype == np.float32
    np.testing.assert_array_equal(E[3], _doc(3).encrypted_embedding)
    with pytest.raises(KeyError):
        st2.load("nope")
    (tmp_path / "d2.enc").unlink()
    with pytest.raises(FileNotFoundError):
        st2.load("d2")
    v = st2.validate_all()
    assert v["invalid"] == ["d2"] and len(v["valid"]) == 4
    assert st2.delete("d2") and not st2.delete("d2")
    s = st2.get_stats()
    assert s["total_documents"] == 4 and s["total_size_bytes"] > 0
    assert st2.corpus()[0] == ["d0", "d1", "d3", "d4"]


# --------------------------------------------------------- BatchProcessor --
class _Embedder:
    """Deterministic text -> 32-dim vector stand-in for BertEmbedder."""

    def get_embedding(self, text):
        h = np.frombuffer(text.encode().ljust(32, b"."), dtype=np.uint8)[:32].astype(np.float32)
        return h / np.linalg.norm(h)

    def get_embeddings_batch(self, texts):
        return np.stack([self.get_embedding(t) for t in texts])


class _Reducer:
    """Stand-in for DimensionReducer: fixed 32 -> 16 projection."""
    P = np.random.default_rng(0).standard_normal((32, 16)).astype(np.float32) / 4

    def transform(self, X):
        return np.asarray(X) @ self.P


class _Keys:
    def __init__(self, k):
        self.k = k

    def get_current_key(self):
        return self.k


def _processor(tmp_path, **cfg):
    from batch_operations import BatchConfig, BatchProcessor
    from encrypted_storage import EncryptedDocumentStore
    c = BatchConfig(**{"fhe": "disable", "input_dim": 16, "n_bits": 6, "seed": 21, "show_progress": False, "key_manager_default": False, **cfg})
    return BatchProcessor(embedder=_Embedder(), reducer=_Reducer(), storage=EncryptedDocumentStore(str(tmp_path)),
                          config=c)


def test_batch_config_validation():
    from batch_operations import BatchConfig
    for bad in ({"batch_size": 0}, {"max_memory_mb": 10}, {"fhe": "gpu"}, {"search_chunk": 0}):
        with pytest.raises(ValueError):
            BatchConfig(**bad)


def test_processor_without_key_has_no_model(tmp_path):
    from batch_operations import BatchConfig, BatchProcessor
    from encrypted_storage import EncryptedDocumentStore
    p = BatchProcessor(key_manager=_Keys(None), storage=EncryptedDocumentStore(str(tmp_path)),
                       config=BatchConfig(fhe="disable", input_dim=16))
    assert p.fhe_model is None
    for call in (lambda: p.compare_encrypted("a", "b"), lambda: p.search_vector(np.zeros(16)),
                 lambda: p.encrypt_documents(["x"])):
        with pytest.raises(RuntimeError):
            call()


def test_processor_search_matches_oracle(tmp_path):
    """Clear-path search over a stored corpus == the oracle's restatement of
    batch_operations.py:240-284 (float >=, stable sort desc, [:top_k])."""
    from encrypted_storage import EncryptedDocument
    p = _processor(tmp_path)
    q, docs = Q.make_corpus(16, 300, seed=9)
    docs[10] = docs[11]            # exact score ties: the earlier index wins
    docs[200] = docs[11]
    p.storage.save_many([EncryptedDocument(f"doc{i:03d}", "h", "t", docs[i]) for i in range(len(docs))])
    ref = Q.QuantizedLinearParams.from_json(p.fhe_model.model.quant_params.to_dict())
    ids = [f"doc{i:03d}" for i in range(len(docs))]
    for top_k, t in ((10, 0.5), (5, -10.0), (400, 0.3), (0, 0.5), (3, 99.0)):
        assert p.search_vector(q, top_k, t) == Q.search(ref, q, docs, top_k, t, doc_ids=ids)
    q64 = q.astype(np.float64) * 1.01
    assert p.search_vector(q64, 10, 0.2) == Q.search(ref, q64, docs, 10, 0.2, doc_ids=ids)
    s = p.compare_encrypted("doc001", "doc002")
    assert s == float(Q.predict(ref, (docs[1] * docs[2])[None, :])[0])
    with pytest.raises(ValueError):
        p.search_vector(np.zeros(8, np.float32))


def test_processor_encrypt_and_text_search(tmp_path):
    p = _processor(tmp_path, batch_size=3)
    texts = [f"document number {i} about topic {i % 3}" for i in range(8)]
    ids = p.encrypt_documents(texts, doc_ids=[f"t{i}" for i in range(8)], metadata=[{"i": i} for i in range(8)])
    assert ids == [f"t{i}" for i in range(8)]
    doc = p.storage.load("t4")
    assert doc.encrypted_embedding.shape == (16,) and doc.metadata == {"i": 4}
    res = p.search_similar(texts[4], top_k=3, min_similarity=-100)
    assert len(res) == 3
    assert res == p.search_vector(_Reducer().transform(_Embedder().get_embedding(texts[4])[None])[0], 3, -100)
    st = p.get_memory_stats()
    assert set(st) == {"initial_mb", "current_mb", "used_mb", "max_mb", "usage_percent"}


def test_processor_loads_persisted_model(tmp_path):
    from fheicp import persist
    p = _processor(tmp_path / "a")
    qp = p.fhe_model.model.quant_params
    path = str(tmp_path / "model.npz")
    persist.save_model(path, qp, p.fhe_model.model._fitted().scheme)
    p2 = _processor(tmp_path / "b", model_path=path, seed=999)   # a different seed would retrain differently
    assert p2.fhe_model.model.quant_params.to_dict() == qp.to_dict()


def test_clear_processor_loads_wrapped_model_without_password(tmp_path, monkeypatch):
    """The clear modes read only the quantisation of a model_path file, so a
    file whose secret keys are Fernet-wrapped loads without a password
    (persist.load_model(keys=False)); loading its keys still needs one."""
    from fheicp import persist
    monkeypatch.delenv("FHE_MASTER_PASSWORD", raising=False)
    p = _processor(tmp_path / "a")
    qp = p.fhe_model.model.quant_params
    rng = np.random.default_rng(4)
    keys = {"s_small": rng.integers(0, 2, 887).astype(np.uint64), "s_big": rng.integers(0, 2, 2048).astype(np.uint64),
            "bsk": rng.integers(0, 2 ** 63, 8, dtype=np.uint64), "ksk": rng.integers(0, 2 ** 63, 8, dtype=np.uint64)}
    path = str(tmp_path / "wrapped.npz")
    persist.save_model(path, qp, p.fhe_model.model._fitted().scheme, keys, password="pw")
    with pytest.raises(ValueError):
        persist.load_model(path)
    qp2, _, k = persist.load_model(path, keys=False)
    assert k is None and qp2.to_dict() == qp.to_dict()
    p2 = _processor(tmp_path / "b", model_path=path, seed=999)
    assert p2.fhe_model.model.quant_params.to_dict() == qp.to_dict()


def test_persist_versions(tmp_path):
    """Files are written as version 2; version-1 files (plaintext secret keys)
    still load; unknown versions are refused instead of read as key-less."""
    import json
    from fheicp import persist
    from fheicp.params import params_for_bits
    from fheicp.sklearn import LinearRegression
    X, y = _data(16)
    qp = LinearRegression(n_bits=6).fit(X, y).quant_params
    sch = params_for_bits(qp.msg_bits())
    keys = {k: np.arange(6, dtype=np.uint64) % 2 for k in persist.KEY_NAMES}
    path = str(tmp_path / "m.npz")
    persist.save_model(path, qp, sch, keys, allow_plaintext_secrets=True)
    with np.load(path) as z:
        assert json.loads(bytes(z["meta"]).decode())["version"] == 2
    for v, ok in ((1, True), (2, True), (3, False), (0, False)):
        meta = {"format": persist.FORMAT, "version": v, "quant": qp.to_dict(), "scheme": sch.as_dict()}
        arrays = {k: keys[k] for k in persist.KEY_NAMES}
        arrays["meta"] = np.frombuffer(json.dumps(meta).encode(), dtype=np.uint8)
        np.savez(path, **arrays)
        if ok:
            _, _, k2 = persist.load_model(path)
            for k in persist.KEY_NAMES:
                np.testing.assert_array_equal(k2[k], keys[k])
        else:
            with pytest.raises(ValueError):
                persist.load_model(path)


def test_persist_v1_with_password_blob_loads(tmp_path, monkeypatch):
    """The release before version 2 (da9f35f) wrote VERSION = 1 together with
    the Fernet-wrapped `secret` blob whenever a password was set. Such a file
    (rebuilt here byte for byte: the same arrays, meta version 1) loads with
    the password, and without one under keys=False (the clear modes)."""
    import json
    from fheicp import persist
    from fheicp.params import params_for_bits
    from fheicp.sklearn import LinearRegression
    monkeypatch.delenv("FHE_MASTER_PASSWORD", raising=False)
    X, y = _data(16)
    qp = LinearRegression(n_bits=6).fit(X, y).quant_params
    sch = params_for_bits(qp.msg_bits())
    keys = {k: np.arange(20, dtype=np.uint64) % 2 for k in persist.KEY_NAMES}
    path = str(tmp_path / "v1.npz")
    persist.save_model(path, qp, sch, keys, password="pw")
    with np.load(path) as z:
        arrays = {k: z[k].copy() for k in z.files}
    meta = json.loads(bytes(arrays["meta"]).decode())
    assert "secret" in meta and "secret" in arrays
    meta["version"] = 1
    arrays["meta"] = np.frombuffer(json.dumps(meta).encode(), dtype=np.uint8)
    np.savez(path, **arrays)
    _, _, k2 = persist.load_model(path, password="pw")
    for k in persist.KEY_NAMES:
        np.testing.assert_array_equal(k2[k], keys[k])
    q2, s2, none = persist.load_model(path, keys=False)
    assert none is None and q2.to_dict() == qp.to_dict() and s2 == sch
    with pytest.raises(ValueError, match="password"):
        persist.load_model(path)


def test_corpus_secret_checked_before_keygen(tmp_path, monkeypatch):
    """A processor that will save an encrypted corpus refuses to start without
    a password (or the plaintext opt-in) before any training or keygen."""
    monkeypatch.delenv("FHE_MASTER_PASSWORD", raising=False)
    with pytest.raises(ValueError, match="password"):
        _processor(tmp_path, fhe="execute", store_ciphertexts=True, corpus_path=str(tmp_path / "c.npz"))


class _GpuTaggedReducer(_Reducer):
    """A reducer the processor takes as already on the device (it has
    transform_dev), standing in for fheicp.pca.GpuPCA on a host without one."""

    def transform_dev(self, X):  # pragma: no cover - never called here
        raise AssertionError


def test_gpu_reducer_contract_refuses_mixed_stores(tmp_path):
    """BatchConfig.gpu_reducer: documents reduced on the GPU are tagged, and a
    score never mixes GPU- and CPU-reduced vectors (the two PCAs differ at
    quantizer rounding boundaries): searching, comparing or adding across
    reducers raises unless allow_mixed_reducers."""
    from batch_operations import GPU_REDUCER, REDUCER_KEY, BatchConfig, BatchProcessor
    from encrypted_storage import EncryptedDocumentStore
    store = EncryptedDocumentStore(str(tmp_path))

    def proc(**kw):
        c = BatchConfig(**{"fhe": "disable", "input_dim": 16, "n_bits": 6, "seed": 21, "show_progress": False,
                           "key_manager_default": False, **kw})
        red = _GpuTaggedReducer() if kw.get("gpu_reducer") else _Reducer()
        return BatchProcessor(embedder=_Embedder(), reducer=red, storage=store, config=c)

    g = proc(gpu_reducer=True)
    g.encrypt_documents(["alpha doc", "beta doc", "gamma doc"], doc_ids=["a", "b", "c"])
    assert all(store.index[i]["metadata"][REDUCER_KEY] == GPU_REDUCER for i in "abc")
    assert len(g.search_similar("alpha doc", top_k=2, min_similarity=-100)) == 2   # one reducer: fine
    cpu = proc()
    with pytest.raises(ValueError, match="reducers"):
        cpu.search_similar("alpha doc", top_k=2, min_similarity=-100)
    with pytest.raises(ValueError, match="reducers"):
        cpu.encrypt_documents(["delta doc"], doc_ids=["d"])
    mixed = proc(allow_mixed_reducers=True)
    mixed.encrypt_documents(["delta doc"], doc_ids=["d"])
    assert REDUCER_KEY not in store.index["d"]["metadata"]
    with pytest.raises(ValueError, match="reducers"):
        g.compare_encrypted("a", "d")
    assert isinstance(mixed.compare_encrypted("a", "d"), float)
    assert g.compare_encrypted("a", "b") == pytest.approx(mixed.compare_encrypted("a", "b"))


class _HipEmbedder(_Embedder):
    """Stand-in for BertEmbedder(gpu_encoder=True) (its provenance tag)."""
    provenance = "hip-bert-f32"


def test_gpu_embedder_contract_refuses_mixed_stores(tmp_path):
    """BatchConfig.gpu_embedder's contract, as the reducer's: documents the
    HIP encoder embedded carry metadata[EMBEDDER_KEY] = its provenance, and
    no score mixes them with torch-embedded vectors (search, compare, insert
    raise unless allow_mixed_embedders)."""
    from batch_operations import EMBEDDER_KEY, BatchConfig, BatchProcessor
    from encrypted_storage import EncryptedDocumentStore
    store = EncryptedDocumentStore(str(tmp_path))

    def proc(hip, **kw):
        c = BatchConfig(**{"fhe": "disable", "input_dim": 16, "n_bits": 6, "seed": 21, "show_progress": False,
                           "key_manager_default": False, **kw})
        return BatchProcessor(embedder=_HipEmbedder() if hip else _Embedder(), reducer=_Reducer(), storage=store,
                              config=c)

    g = proc(True)
    g.encrypt_documents(["alpha doc", "beta doc"], doc_ids=["a", "b"])
    assert all(store.index[i]["metadata"][EMBEDDER_KEY] == "hip-bert-f32" for i in "ab")
    assert len(g.search_similar("alpha doc", top_k=2, min_similarity=-100)) == 2
    cpu = proc(False)
    with pytest.raises(ValueError, match="embedders"):
        cpu.search_similar("alpha doc", top_k=2, min_similarity=-100)
    with pytest.raises(ValueError, match="embedders"):
        cpu.encrypt_documents(["delta doc"], doc_ids=["d"])
    with pytest.raises(ValueError, match="embedders"):       # untagged vectors are the torch encoder's
        g.store_vectors(np.zeros((1, 16), np.float32), ["v"])
    g.store_vectors(np.zeros((1, 16), np.float32), ["v"], embedder="hip-bert-f32")
    assert store.index["v"]["metadata"][EMBEDDER_KEY] == "hip-bert-f32"
    mixed = proc(False, allow_mixed_embedders=True)
    mixed.encrypt_documents(["delta doc"], doc_ids=["d"])
    assert EMBEDDER_KEY not in store.index["d"]["metadata"]
    with pytest.raises(ValueError, match="embedders"):
        g.compare_encrypted("a", "d")
    assert isinstance(mixed.compare_encrypted("a", "d"), float)
    with pytest.raises(ValueError, match="gpu_embedder_precision"):
        BatchConfig(gpu_embedder=True, gpu_embedder_precision="fp16")


def test_store_vectors_tags_the_reducer(tmp_path):
    """store_vectors takes the reducer of the config (GPU_REDUCER under
    gpu_reducer) or an explicit one, tags it and runs the same check as
    encrypt_documents."""
    from batch_operations import GPU_REDUCER, REDUCER_KEY, BatchConfig, BatchProcessor
    from encrypted_storage import EncryptedDocumentStore
    store = EncryptedDocumentStore(str(tmp_path))
    c = BatchConfig(fhe="disable", input_dim=16, n_bits=6, seed=21, show_progress=False, key_manager_default=False,
                    gpu_reducer=True)
    p = BatchProcessor(embedder=_Embedder(), reducer=_GpuTaggedReducer(), storage=store, config=c)
    v = np.random.default_rng(1).standard_normal((3, 16)).astype(np.float32)
    p.store_vectors(v[:2], ["x", "y"])
    assert store.index["x"]["metadata"][REDUCER_KEY] == GPU_REDUCER
    with pytest.raises(ValueError, match="reducers"):
        p.store_vectors(v[2:], ["z"], reducer=None)
    assert "z" not in store.index
