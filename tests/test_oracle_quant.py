"""CPU: the clear-path oracle (Concrete-ML restatement) against the reference's
known-answer test and the committed golden vectors; product host logic
(calibration, threshold, accumulator width) against the oracle."""
import json
from pathlib import Path

import numpy as np
import pytest

from oracle import quant_ref as Q

GOLD = json.loads((Path(__file__).parent / "golden" / "quant_golden.json").read_text())
CONFIGS = [k for k in GOLD if k.startswith("C")]


def test_kat_reference_test_fhe():
    """/root/reference/test_fhe.py:13-60: y = 2x on x = 1..6, n_bits=8, predict x = 7."""
    X = np.array([[1], [2], [3], [4], [5], [6]], dtype=np.float32)
    y = np.array([2, 4, 6, 8, 10, 12], dtype=np.float32)
    qp = Q.fit_quantized_linear(X, y, 8)
    k = GOLD["KAT_test_fhe"]
    assert qp.to_json() == k["params"]
    # calibration: s_x = (6-1)/255, zp = round((-6*128 - 1*127) / 5) = -179
    assert qp.s_x == pytest.approx(5 / 255) and qp.zp_x == -179
    assert list(qp.q_w) == [127]
    qx = Q.quantize_input(qp, [[7.0]])
    assert qx.tolist() == [[127]] == k["q_x"]          # 7 is above rmax=6 -> clipped
    acc = Q.accumulate(qp, qx)
    assert acc.tolist() == [127 * 127 + 179 * 127] == k["acc"]
    score = Q.predict(qp, [[7.0]])[0]
    assert score == k["score"]
    assert abs(score - 12.0) < 1e-5                     # not the printed "Expected 14.0"
    # inside the calibration range the model reproduces y = 2x to quantisation accuracy
    for x in (1.0, 3.5, 6.0):
        assert abs(Q.predict(qp, [[x]])[0] - 2 * x) < 2 * 5 / 255


@pytest.mark.parametrize("name", CONFIGS)
def test_golden_vectors(name):
    g = GOLD[name]
    c = g["config"]
    X, y = Q.prepare_training_data(c["dim"], 1000, seed=g["train_seed"])
    qp = Q.fit_quantized_linear(X, y, c["n_bits"])
    assert qp.to_json() == g["params"]
    q, docs = Q.make_corpus(c["dim"], c["docs"], seed=g["corpus_seed"])
    Xp = Q.pair_features(q, docs)
    qx = Q.quantize_input(qp, Xp)
    assert qx[:4].tolist() == g["qx_head"]
    acc = Q.accumulate(qp, qx)
    assert acc.tolist() == g["acc"]
    assert [float(s) for s in Q.dequantize(qp, acc)] == g["scores"]
    top = Q.search(qp, q, docs, 10, 0.5)
    assert [[i, s] for i, s in top] == g["topk"]
    qc, dc = Q.make_corpus(c["dim"], 16, seed=g["clip_seed"], clip_set=True)
    qxc = Q.quantize_input(qp, Q.pair_features(qc, dc))
    assert qxc.tolist() == g["clip_qx"]
    assert set(np.unique(qxc)) & {qp.qx_min, qp.qx_max}, "clip set must exercise clipping"
    lo, hi = Q.acc_bounds(qp)
    assert [lo, hi] == g["acc_bounds"] and Q.message_bits(qp) == g["msg_bits"]
    assert lo <= acc.min() and acc.max() <= hi


@pytest.mark.parametrize("name", CONFIGS)
def test_product_quantisation_matches_oracle(name):
    from fheicp.model import FheLinearModel, QuantParams, threshold_int
    from fheicp.datagen import training_pairs, corpus
    g = GOLD[name]
    c = g["config"]
    X, y = training_pairs(c["dim"], 1000, seed=g["train_seed"])
    Xo, yo = Q.prepare_training_data(c["dim"], 1000, seed=g["train_seed"])
    assert np.array_equal(X, Xo) and np.array_equal(y, yo)
    m = FheLinearModel.fit(X, y, c["n_bits"])
    assert m.qparams.to_dict() == g["params"]
    assert m.msg_bits == g["msg_bits"]
    assert m.qparams.acc_range() == tuple(g["acc_bounds"])
    assert threshold_int(m.qparams, 0.5) == g["threshold_T"]
    q, docs = corpus(c["dim"], c["docs"], seed=g["corpus_seed"])
    qo, do = Q.make_corpus(c["dim"], c["docs"], seed=g["corpus_seed"])
    assert np.array_equal(q, qo) and np.array_equal(docs, do)
    # fhe="disable" host path of the drop-in estimator
    assert np.array_equal(m.predict_clear(Q.pair_features(q, docs)), np.asarray(g["scores"]))
    rt = QuantParams.from_dict(m.qparams.to_dict())
    assert rt.to_dict() == m.qparams.to_dict()


@pytest.mark.parametrize("name", ["C1", "C2", "C4"])
def test_threshold_equivalence_exhaustive(name):
    """acc >= T  <=>  float64(out_scale * acc) >= t, for every representable acc."""
    g = GOLD[name]
    qp = Q.QuantizedLinearParams.from_json(g["params"])
    lo, hi = Q.acc_bounds(qp)
    accs = np.arange(lo, hi + 1)
    scores = Q.dequantize(qp, accs)
    for t in (0.5, 0.0, -0.25, 0.9, float(scores[len(scores) // 3]), 1e9, -1e9):
        T = Q.threshold_int(qp, t, lo, hi)
        assert np.array_equal(accs >= T, scores >= t), t


def test_search_semantics_stable_ties():
    """batch_operations.py:278-284: float >=, stable sort desc (ties keep
    insertion order), slice top_k."""
    g = GOLD["C4"]
    qp = Q.QuantizedLinearParams.from_json(g["params"])
    q, docs = Q.make_corpus(16, 512, seed=g["corpus_seed"])
    res = Q.search(qp, q, docs, 50, 0.5)
    scores = Q.predict(qp, Q.pair_features(q, docs))
    manual = sorted([(i, float(s)) for i, s in enumerate(scores) if s >= 0.5], key=lambda x: -x[1])[:50]
    assert res == manual
    s = [x[1] for x in res]
    ties = [i for i in range(1, len(s)) if s[i] == s[i - 1]]
    assert ties, "the corpus should contain tied quantized scores"
    for i in ties:
        assert res[i][0] > res[i - 1][0]


def test_dtype_promotion_f64_query():
    """batch_operations.py:260 leaves the query in float64 while docs are float32."""
    g = GOLD["C2"]
    qp = Q.QuantizedLinearParams.from_json(g["params"])
    q, docs = Q.make_corpus(16, 64, seed=3)
    X32 = Q.pair_features(q, docs)
    X64 = Q.pair_features(q.astype(np.float64), docs)
    assert X32.dtype == np.float32 and X64.dtype == np.float64
    # quantisation may differ at rounding boundaries; both must be valid
    for X in (X32, X64):
        qx = Q.quantize_input(qp, X)
        assert qx.min() >= qp.qx_min and qx.max() <= qp.qx_max
