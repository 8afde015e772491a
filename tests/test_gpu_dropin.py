"""GPU: the drop-in Python surface on the encrypted path, bit-exact against
the oracle (scores and threshold decisions), through libfheicp."""
import numpy as np
import pytest

from oracle import quant_ref as Q

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def fitted(need_gpu):
    from fheicp.sklearn import LinearRegression
    X, y = Q.prepare_training_data(16, 1000, seed=31)
    est = LinearRegression(n_bits=6, key_seed=77).fit(X, y)
    est.compile(X[:10])
    ref = Q.fit_quantized_linear(X, y, 6)
    return est, ref


def test_estimator_execute_bit_exact(fitted):
    est, ref = fitted
    assert est.fhe_circuit.graph.maximum_integer_bit_width() == Q.message_bits(ref)
    q, docs = Q.make_corpus(16, 256, seed=4)
    X = Q.pair_features(q, docs)
    np.testing.assert_array_equal(est.predict(X, fhe="execute"), Q.predict(ref, X))
    Xc = Q.pair_features(*Q.make_corpus(16, 64, seed=5, clip_set=True))   # clipped inputs
    np.testing.assert_array_equal(est.predict(Xc, fhe="execute"), Q.predict(ref, Xc))


def test_estimator_threshold_bit(fitted):
    est, ref = fitted
    q, docs = Q.make_corpus(16, 256, seed=6)
    X = Q.pair_features(q, docs)
    clear = Q.predict(ref, X)
    for t in (0.5, float(np.median(clear)), -1e9, 1e9):
        scores, keep = est.predict_threshold(X, t)
        np.testing.assert_array_equal(scores, clear)
        np.testing.assert_array_equal(keep, clear >= t)


def _br_totals(eng):
    gs = ("main", "mid0", "mid", "mid2", "fast", "fast2")
    rd = {g: eng.profile_read(f"blind_rotate_{g}") for g in gs}
    return (sum(r["launches"] for r in rd.values()), sum(r["items"] for r in rd.values()),
            eng.profile_read("keyswitch")["launches"])


def test_execute_is_leveled_only(fitted):
    """predict(fhe="execute") is the reference's PBS-free leveled circuit
    (fhe_similarity.py:142-160, fhe_score_batch): bit-exact scores, and no
    key switch or blind rotation launches at all; predict_threshold runs the
    sign extraction, pbs_per_prediction bootstraps per compare (the count the
    bench reports as pbs_per_compare)."""
    from fheicp.params import sign_pbs_count
    est, ref = fitted
    eng = est._fitted().engine
    q, docs = Q.make_corpus(16, 300, seed=17)
    X = Q.pair_features(q, docs)
    eng.profile(True)
    got = est.predict(X, fhe="execute")
    br_launches, _, ks_launches = _br_totals(eng)
    eng.profile(False)
    np.testing.assert_array_equal(got, Q.predict(ref, X))
    assert br_launches == 0 and ks_launches == 0
    assert est.fhe_circuit.pbs_per_prediction == sign_pbs_count(eng.params)
    eng.profile(True)
    scores, keep = est.predict_threshold(X, 0.5)
    _, br_items, ks_launches = _br_totals(eng)
    eng.profile(False)
    np.testing.assert_array_equal(scores, Q.predict(ref, X))
    np.testing.assert_array_equal(keep, Q.predict(ref, X) >= 0.5)
    assert br_items == est.fhe_circuit.pbs_per_prediction * len(X)
    assert ks_launches == est.fhe_circuit.pbs_per_prediction


def test_similarity_model_encrypted_and_key_persistence(need_gpu, tmp_path, monkeypatch):
    from fhe_similarity import FHESimilarityModel
    monkeypatch.setenv("FHE_MASTER_PASSWORD", "persist-pw")   # wraps the secret keys (fheicp.persist)
    m = FHESimilarityModel(input_dim=16, n_bits=6, seed=12)
    X, _ = m.train()
    m.compile(X[:10], key_seed=5)
    assert m.metrics["circuit_max_bits"] >= 2
    enc = m.predict_encrypted(X[:100])
    np.testing.assert_array_equal(enc, m.predict_clear(X[:100]))
    path = str(tmp_path / "compiled.npz")
    m.save_compiled(path)
    m2 = FHESimilarityModel.load_compiled(path)
    assert m2.compiled
    np.testing.assert_array_equal(m2.predict_encrypted(X[:100]), enc)
    k1 = m.model._fitted().engine.export_keys()
    k2 = m2.model._fitted().engine.export_keys()
    for k in k1:
        np.testing.assert_array_equal(k1[k], k2[k])


def test_processor_encrypted_search_matches_oracle(need_gpu, tmp_path):
    """BatchProcessor.search_vector on the GPU == batch_operations.py:240-284
    restated by the oracle, including ties, chunking and slice semantics."""
    from batch_operations import BatchConfig, BatchProcessor
    from encrypted_storage import EncryptedDocument, EncryptedDocumentStore
    cfg = BatchConfig(fhe="execute", input_dim=16, n_bits=6, seed=40, key_seed=41, search_chunk=128,
                      show_progress=False, key_manager_default=False)
    p = BatchProcessor(storage=EncryptedDocumentStore(str(tmp_path)), config=cfg)
    q, docs = Q.make_corpus(16, 500, seed=13)
    docs[7] = docs[300]
    docs[450] = docs[300]
    p.storage.save_many([EncryptedDocument(f"doc{i:03d}", "h", "t", docs[i]) for i in range(len(docs))])
    ids = [f"doc{i:03d}" for i in range(len(docs))]
    ref = Q.QuantizedLinearParams.from_json(p.fhe_model.model.quant_params.to_dict())
    for top_k, t in ((10, 0.5), (25, -10.0), (600, 0.2), (-3, 0.6), (4, 99.0)):
        got = p.search_vector(q, top_k, t)
        assert got == Q.search(ref, q, docs, top_k, t, doc_ids=ids), (top_k, t)
    assert p.compare_encrypted("doc003", "doc004") == float(Q.predict(ref, (docs[3] * docs[4])[None, :])[0])


def test_reference_side_ctypes_binding(need_gpu):
    """integration/fhe_gpu.py — the numpy-only binding INTEGRATION.md shows —
    reproduces the oracle's accumulators and threshold bits."""
    import sys
    from pathlib import Path
    from fheicp import LIB_PATH
    from fheicp.params import params_for_bits
    sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "integration"))
    from fhe_gpu import GpuCompare
    X, y = Q.prepare_training_data(16, 1000, seed=2)
    ref = Q.fit_quantized_linear(X, y, 6)
    P = Q.message_bits(ref)
    q, docs = Q.make_corpus(16, 200, seed=8)
    qx = Q.quantize_input(ref, Q.pair_features(q, docs))
    acc_ref = Q.accumulate(ref, qx)
    lo, hi = Q.acc_bounds(ref)
    T = Q.threshold_int(ref, 0.5, lo, hi)
    eng = GpuCompare(params_for_bits(P).as_dict(), key_seed=99, lib_path=str(LIB_PATH))
    try:
        acc, below = eng.compare(qx, ref.q_w, ref.const_term, T)
        scored = eng.score(qx, ref.q_w, ref.const_term, (lo + hi) // 2)
    finally:
        eng.close()
    np.testing.assert_array_equal(acc, acc_ref)
    np.testing.assert_array_equal(below, (acc_ref < T).astype(np.int64))
    np.testing.assert_array_equal(scored, acc_ref)


def test_key_manager_generate_load_and_processor(need_gpu, tmp_path):
    """FHEKeyManager.generate_keys (GPU keygen) -> Fernet-wrapped secret keys +
    evaluation keys on disk -> a new manager's load_compiled gives the same keys
    and results, and a BatchProcessor handed the manager uses them instead of
    retraining (§8f-2), matching the oracle on search."""
    from batch_operations import BatchConfig, BatchProcessor
    from encrypted_storage import EncryptedDocument, EncryptedDocumentStore
    from key_management import FHEKeyManager
    km = FHEKeyManager(str(tmp_path / "keys"), password="pw")
    info = km.generate_keys("k16", input_dim=16, n_bits=6, seed=21, key_seed=22)
    assert km.get_current_key() == "k16" and info["model_file"].endswith("compiled_model.enc")
    km2 = FHEKeyManager(str(tmp_path / "keys"), password="pw")
    m = km2.load_compiled()
    qp, _, keys = km2.load_key_material()
    X, y = Q.prepare_training_data(16, 1000, seed=21)
    ref = Q.fit_quantized_linear(X, y, 6)
    assert ref.to_json() == qp.to_dict()
    np.testing.assert_array_equal(m.predict_encrypted(X[:64]), Q.predict(ref, X[:64]))
    exported = m.model._fitted().engine.export_keys()
    for k in keys:
        np.testing.assert_array_equal(exported[k], keys[k])
    cfg = BatchConfig(fhe="execute", input_dim=16, n_bits=6, seed=999, show_progress=False)
    p = BatchProcessor(key_manager=km2, storage=EncryptedDocumentStore(str(tmp_path / "docs")), config=cfg)
    assert p.fhe_model.model.quant_params.to_dict() == qp.to_dict()   # loaded, not retrained (seed 999)
    q, docs = Q.make_corpus(16, 200, seed=14)
    p.storage.save_many([EncryptedDocument(f"d{i}", "h", "t", docs[i]) for i in range(len(docs))])
    assert p.search_vector(q, 10, 0.5) == Q.search(ref, q, docs, 10, 0.5, doc_ids=[f"d{i}" for i in range(200)])
