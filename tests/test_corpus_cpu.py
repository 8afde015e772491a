"""CPU: the encrypted-corpus mode — host
logic against the oracle restatement, the seeded-LWE oracle against the plain
encryption it compresses, and the versioned document payload in the store."""
import numpy as np
import pytest

from oracle import quant_ref as Q

from fheicp.corpus import CorpusQuant, HEADER_WORDS, MAGIC, pack_payload, unpack_payload
from fheicp.model import FheLinearModel
from fheicp.params import TOY


@pytest.fixture(scope="module")
def quant():
    X, y = Q.prepare_training_data(16, 1000, seed=1236)
    m = FheLinearModel.fit(X, y, 6)
    oq = Q.fit_quantized_linear(X, y, 6)
    from fheicp.datagen import training_embeddings
    e1, e2 = training_embeddings(16, 1000, seed=0)
    cq = CorpusQuant.calibrate(m.qparams, np.concatenate([e1, e2]))
    return cq, oq, np.concatenate([e1, e2])


def test_corpus_quantizer_matches_oracle(quant):
    cq, oq, calib = quant
    assert cq.s_e == Q.corpus_scale(calib, 6)
    assert cq.out_scale == Q.corpus_out_scale(oq, cq.s_e)
    assert cq.q_b == Q.corpus_qb(oq, cq.s_e)
    assert cq.worst_msg_bits() == Q.corpus_worst_bits(oq, cq.s_e, 6)
    for seed in range(6):
        q, docs = Q.make_corpus(16, 64, seed=seed, clip_set=seed % 3 == 2)
        qq = cq.quant(q)
        np.testing.assert_array_equal(qq, Q.corpus_quant(cq.s_e, 6, q))
        lo, hi = cq.acc_range(cq.weights(qq))
        assert (lo, hi) == Q.corpus_bounds(oq, cq.s_e, 6, q)
        acc = Q.corpus_accumulate(oq, cq.s_e, 6, q, docs)
        assert lo <= acc.min() and acc.max() <= hi
        assert cq.bits_for(lo, hi) <= cq.worst_msg_bits()
        # threshold: acc >= T <=> float score >= t, on every accumulator value
        for t in (0.5, -0.25, 0.0):
            T = cq.threshold_int(lo, hi, t)
            s = np.float64(cq.out_scale)
            assert all((s * np.float64(a) >= t) == (a >= T) for a in range(lo, hi + 1, 97))


def test_query_plan_rescale(quant):
    """W' = W * 2^(P0 - P): sum_j W'_j dq_j 2^(64-P0) == sum_j W_j dq_j 2^(64-P) mod 2^64."""
    from fheicp.corpus import EncryptedCorpus
    cq, oq, _ = quant
    c = EncryptedCorpus(cq)
    q, docs = Q.make_corpus(16, 32, seed=9)
    Wr, cst, T, P = c.query_plan(q, 0.5)
    assert 4 <= P <= c.P0 and cst == cq.q_b
    dq = Q.corpus_quant(cq.s_e, 6, docs)
    with np.errstate(over="ignore"):
        lhs = (dq.astype(np.uint64) @ Wr.view(np.uint64)) << np.uint64(64 - c.P0)
        rhs = (dq.astype(np.uint64) @ cq.weights(cq.quant(q)).view(np.uint64)) << np.uint64(64 - P)
    np.testing.assert_array_equal(lhs, rhs)


def test_seeded_oracle_is_the_plain_encryption(oracle_lib):
    """With mask key == noise key, a seeded corpus expands to exactly the
    ciphertexts of ref_encrypt_ints (same streams, ids id0[b] + j)."""
    ref = oracle_lib.RefTFHE(TOY.as_dict(), 4321)
    B, D = 5, 3
    rng = np.random.default_rng(2)
    v = rng.integers(-(2 ** 7), 2 ** 7, (B, D))
    key = oracle_lib.key_from_seed(77)
    id0 = np.array([1000 + D * b for b in range(B)], np.uint64)
    body = ref.encrypt_seeded(v, key, key, id0)
    ct = ref.expand_seeded(body, id0, key)
    np.testing.assert_array_equal(ct, ref.encrypt_ints(v.reshape(-1), seed=77, id0=1000))
    np.testing.assert_array_equal(ref.decrypt_ints(ct), v.reshape(-1))
    # a different noise key changes only the bodies, and still decrypts
    body2 = ref.encrypt_seeded(v, key, oracle_lib.key_from_seed(78), id0)
    assert not np.array_equal(body2, body)
    np.testing.assert_array_equal(ref.decrypt_ints(ref.expand_seeded(body2, id0, key)), v.reshape(-1))


def test_key_from_seed_matches_library(oracle_lib):
    from fheicp.engine import Engine
    for s in (0, 1, 2 ** 63 + 5):
        np.testing.assert_array_equal(Engine.key_from_seed(s), oracle_lib.key_from_seed(s))


def test_payload_round_trip_and_store(tmp_path):
    from encrypted_storage import CIPHERTEXT_VERSION, EncryptedDocument, EncryptedDocumentStore
    key = np.arange(8, dtype=np.uint32) * 7919
    bodies = np.arange(3 * 16, dtype=np.uint64).reshape(3, 16) * np.uint64(0x9E3779B97F4A7C15)
    ids = np.array([5, 2 ** 63 + 1, 77], np.uint64)
    pls = [pack_payload(bodies[i], int(ids[i]), 21, key, 2048) for i in range(3)]
    assert pls[0].size == HEADER_WORDS + 16 and int(pls[0][0]) == MAGIC
    u = unpack_payload(pls[1])
    assert (u["D"], u["P0"], u["id0"], u["big"]) == (16, 21, int(ids[1]), 2048)
    np.testing.assert_array_equal(u["mask_key"], key)
    np.testing.assert_array_equal(u["body"], bodies[1])
    store = EncryptedDocumentStore(str(tmp_path / "store"))
    docs = [EncryptedDocument(doc_id=f"d{i}", content_hash="h", timestamp="t", encrypted_embedding=pls[i],
                              model_version=CIPHERTEXT_VERSION) for i in range(3)]
    store.save_many(docs)
    again = EncryptedDocumentStore(str(tmp_path / "store"))
    assert again.holds_ciphertexts()
    got_ids, got_bodies, got_id0, head = again.encrypted_corpus()
    assert got_ids == ["d0", "d1", "d2"]
    np.testing.assert_array_equal(got_bodies, bodies)
    np.testing.assert_array_equal(got_id0, ids)
    assert head["P0"] == 21 and head["D"] == 16
    with pytest.raises(ValueError):
        again.corpus()     # plaintext view refuses a ciphertext store
    assert again.index["d0"]["model_version"] == CIPHERTEXT_VERSION


def test_payload_validation():
    from encrypted_storage import CIPHERTEXT_VERSION, EncryptedDocument
    key = np.zeros(8, np.uint32)
    good = pack_payload(np.zeros(4, np.uint64), 1, 20, key, 2048)
    EncryptedDocument("a", "h", "t", good, model_version=CIPHERTEXT_VERSION)
    for bad in (good[:-1], good.astype(np.int64), np.concatenate([[np.uint64(1)], good[1:]])):
        with pytest.raises(ValueError):
            EncryptedDocument("a", "h", "t", bad, model_version=CIPHERTEXT_VERSION)
    v2 = good.copy()
    v2[1] = 2
    with pytest.raises(ValueError, match="version"):
        EncryptedDocument("a", "h", "t", v2, model_version=CIPHERTEXT_VERSION)
    # plaintext documents keep the reference's width check
    with pytest.raises(ValueError):
        EncryptedDocument("a", "h", "t", np.zeros(17, np.float32))
