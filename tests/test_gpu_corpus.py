"""GPU: the encrypted-corpus mode (§8f-1) through libfheicp against the oracle.

Bit-exact: seeded encryption (bodies), expansion, the seeded linear
combination; end to end, every decrypted accumulator and threshold bit of
fhe_compare_seeded_batch equals the oracle's restatement (quant_ref.corpus_*),
and the BatchProcessor store (ciphertext payloads on disk) returns the
oracle's top-k."""
import numpy as np
import pytest
import torch

from oracle import quant_ref as Q

from fheicp.engine import Engine
from fheicp.params import TOY, params_for_bits

pytestmark = pytest.mark.gpu


def dev_u64(eng, a):
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.uint64).view(np.int64)).to(eng.device)


@pytest.fixture(scope="module")
def toy(need_gpu, oracle_lib):
    eng = Engine(TOY, 0)
    eng.keygen(99)
    return eng, oracle_lib.RefTFHE(TOY.as_dict(), 99), oracle_lib


@pytest.mark.parametrize("B,D", [(1, 1), (7, 3), (64, 16)])
def test_seeded_encrypt_expand_linear_bit_exact(toy, B, D):
    eng, ref, ol = toy
    rng = np.random.default_rng(B * 31 + D)
    v = rng.integers(-(2 ** 7), 2 ** 7, (B, D))
    mk, nk = ol.key_from_seed(11), ol.key_from_seed(12)
    id0 = rng.integers(0, 2 ** 63, B, dtype=np.int64).astype(np.uint64) * np.uint64(2) + np.uint64(1)
    body = eng.encrypt_seeded(eng.to_dev(v), mk, nk, dev_u64(eng, id0))
    body_ref = ref.encrypt_seeded(v, mk, nk, id0)
    np.testing.assert_array_equal(body.cpu().numpy().view(np.uint64), body_ref)
    ct = eng.expand_seeded(body, dev_u64(eng, id0), B, D, mk)
    ct_ref = ref.expand_seeded(body_ref, id0, mk)
    np.testing.assert_array_equal(ct.cpu().numpy().view(np.uint64), ct_ref)
    np.testing.assert_array_equal(eng.decrypt(ct).cpu().numpy(), v.reshape(-1))
    w = rng.integers(-40, 40, D)
    out = eng.linear_seeded(body, dev_u64(eng, id0), mk, w, 5)
    np.testing.assert_array_equal(out.cpu().numpy().view(np.uint64), ref.linear(ct_ref, B, D, w, 5))


def test_seeded_rejects_bad_arguments(toy):
    import ctypes as C
    eng, _, ol = toy
    L, key = eng._L, eng._key(ol.key_from_seed(1))
    x = torch.zeros(64, dtype=torch.int64, device=eng.device)
    p = C.c_void_p(x.data_ptr())
    assert L.fhe_linear_seeded_batch(eng._ctx, p, p, 2, 0, key, p, 0, p, None) == -1          # D = 0
    assert L.fhe_compare_seeded_batch(eng._ctx, None, None, 4, 16, key, None, 0, 0, None, None, None) == -1
    assert L.fhe_encrypt_seeded_batch(eng._ctx, p, 2 ** 27, 32, key, key, p, p, None) == -1   # B*D >= 2^31
    assert b"seeded" in L.fhe_last_error(eng._ctx)
    assert L.fhe_expand_seeded_batch(eng._ctx, p, p, 0, 4, key, p, None) == 0                 # empty batch


@pytest.fixture(scope="module")
def corpus16(need_gpu):
    from fheicp.corpus import CorpusQuant, EncryptedCorpus
    from fheicp.datagen import training_embeddings
    from fheicp.model import FheLinearModel
    X, y = Q.prepare_training_data(16, 1000, seed=1236)
    m = FheLinearModel.fit(X, y, 6)
    oq = Q.fit_quantized_linear(X, y, 6)
    e1, e2 = training_embeddings(16, 1000, seed=0)
    cq = CorpusQuant.calibrate(m.qparams, np.concatenate([e1, e2]))
    c = EncryptedCorpus(cq).compile(key_seed=5, device=0, noise_seed=6)
    return c, oq


def test_corpus_compare_bit_exact(corpus16):
    c, oq = corpus16
    assert c.scheme == params_for_bits(c.P0)
    q, docs = Q.make_corpus(16, 512, seed=21)
    bodies, ids = c.encrypt_docs(docs)
    eng = c.engine
    np.testing.assert_array_equal(c.decrypt_docs(bodies, ids), Q.corpus_quant(c.cq.s_e, 6, docs))
    ref_acc = Q.corpus_accumulate(oq, c.cq.s_e, 6, q, docs)
    scores = np.float64(Q.corpus_out_scale(oq, c.cq.s_e)) * ref_acc.astype(np.float64)
    for t in (0.5, float(np.median(scores))):
        acc, below, P = c.compare(dev_u64(eng, bodies), dev_u64(eng, ids), q, t)
        np.testing.assert_array_equal(acc.cpu().numpy(), ref_acc)
        np.testing.assert_array_equal(below.cpu().numpy(), (scores < t).astype(np.int64))
        assert P < c.P0   # the per-query width (the rescaled path) is exercised


def test_corpus_compare_clipped_and_extreme_queries(corpus16):
    """Clipped (un-normalised) queries and docs, and the all-qmin query that
    reaches the worst case P0 (no rescale)."""
    c, oq = corpus16
    q, docs = Q.make_corpus(16, 128, seed=22, clip_set=True)
    bodies, ids = c.encrypt_docs(docs)
    eng = c.engine
    for query in (q, np.full(16, -10.0, np.float32)):
        ref_acc = Q.corpus_accumulate(oq, c.cq.s_e, 6, query, docs)
        scores = np.float64(Q.corpus_out_scale(oq, c.cq.s_e)) * ref_acc.astype(np.float64)
        acc, below, P = c.compare(dev_u64(eng, bodies), dev_u64(eng, ids), query, 0.0)
        np.testing.assert_array_equal(acc.cpu().numpy(), ref_acc)
        np.testing.assert_array_equal(below.cpu().numpy(), (scores < 0.0).astype(np.int64))


def test_batch_processor_ciphertext_store(tmp_path, need_gpu, monkeypatch):
    from batch_operations import BatchConfig, BatchProcessor
    monkeypatch.setenv("FHE_MASTER_PASSWORD", "corpus-pw")   # wraps the corpus file's secret keys
    from encrypted_storage import CIPHERTEXT_VERSION, EncryptedDocumentStore
    cfg = BatchConfig(input_dim=16, n_bits=6, seed=3, key_seed=8, store_ciphertexts=True,
                      corpus_path=str(tmp_path / "corpus.npz"), batch_size=100, key_manager_default=False)
    store = EncryptedDocumentStore(str(tmp_path / "docs"))
    bp = BatchProcessor(storage=store, config=cfg)
    q, docs = Q.make_corpus(16, 300, seed=23)
    names = [f"doc{i:04d}" for i in range(len(docs))]
    bp.store_vectors(docs, names)
    assert store.load("doc0007").model_version == CIPHERTEXT_VERSION
    c = bp.corpus_engine
    oq = Q.QuantizedLinearParams.from_json(bp.fhe_model.model.quant_params.to_dict())
    want = Q.corpus_search(oq, c.cq.s_e, c.cq.n_e, q, docs, 10, 0.5)
    got = bp.search_vector(q, top_k=10, min_similarity=0.5)
    assert got == [(names[i], s) for i, s in want]
    # compare two stored ciphertexts: doc 1 decrypted (key holder) as the query
    s_e = c.cq.s_e
    q1 = np.float64(s_e) * Q.corpus_quant(s_e, c.cq.n_e, docs[1]).astype(np.float64)
    acc = Q.corpus_accumulate(oq, s_e, c.cq.n_e, q1, docs[2:3])[0]
    assert bp.compare_encrypted("doc0001", "doc0002") == float(np.float64(c.cq.out_scale) * np.float64(acc))
    # a new process: keys + mask key from corpus_path, documents from disk
    bp2 = BatchProcessor(storage=EncryptedDocumentStore(str(tmp_path / "docs")), config=cfg)
    assert bp2.search_vector(q, top_k=10, min_similarity=0.5) == got
