"""GPU: encryption randomness per session.

Two sessions over the same imported keys encrypt the same quantized inputs:
their ciphertexts share no mask or body word (each session draws its own
256-bit stream key and a random 64-bit id start), while both decrypt to the
exact accumulators of the oracle's restatement. Before round 5 the stream key
was key_seed ^ const and the ids restarted at 0, so two processes with one
configured key_seed produced identical masks and noise.
"""
import numpy as np
import pytest
import torch

from oracle import quant_ref as Q

pytestmark = pytest.mark.gpu


def test_two_sessions_share_no_randomness(need_gpu):
    from fheicp.model import FheLinearModel
    from fheicp.engine import u64

    X, y = Q.prepare_training_data(16, 600, seed=91)
    oq = Q.fit_quantized_linear(X, y, 6)
    m0 = FheLinearModel.fit(X, y, n_bits=6).compile(device=0)       # 256-bit keygen key
    keys = m0.engine.export_keys()
    s1 = FheLinearModel(m0.qparams).compile(device=0, keys=keys)
    s2 = FheLinearModel(m0.qparams).compile(device=0, keys=keys)
    assert isinstance(s1.enc_seed, bytes) and len(s1.enc_seed) == 32
    assert s1.enc_seed != s2.enc_seed and s1.enc_seed != m0.enc_seed

    q, docs = Q.make_corpus(16, 256, seed=92)
    Xp = Q.pair_features(q, docs)
    qx = s1.quantize_dev(torch.from_numpy(np.ascontiguousarray(Xp)).to("cuda:0"))
    c1, c2 = u64(s1.encrypt_linear(qx)), u64(s2.encrypt_linear(qx))
    assert c1.shape == c2.shape == (256, s1.engine.W)
    # no shared mask word and no shared body: independent streams
    assert np.count_nonzero(c1[:, :-1] == c2[:, :-1]) == 0
    assert np.count_nonzero(c1[:, -1] == c2[:, -1]) == 0
    # a second batch of the same session uses fresh stream ids
    c1b = u64(s1.encrypt_linear(qx))
    assert np.count_nonzero(c1b[:, -1] == c1[:, -1]) == 0
    ref = Q.accumulate(oq, Q.quantize_input(oq, Xp))
    for sess, ct in ((s1, c1), (s2, c2), (s1, c1b)):
        acc = sess.engine.decrypt(sess.engine.to_dev(ct)).cpu().numpy()
        assert np.array_equal(acc, ref)
    # and the full encrypted compare agrees across sessions
    a1, b1 = s1.encrypted_acc(qx, T=int(np.median(ref)))
    a2, b2 = s2.encrypted_acc(qx, T=int(np.median(ref)))
    assert np.array_equal(a1.cpu().numpy(), ref) and np.array_equal(a2.cpu().numpy(), ref)
    assert np.array_equal(b1.cpu().numpy(), b2.cpu().numpy())
