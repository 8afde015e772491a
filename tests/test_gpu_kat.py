"""GPU: the reference's only deterministic known-answer test, call for call
through the drop-in estimator and the HIP path.

/root/reference/test_fhe.py:13-60: LinearRegression(n_bits=8) fit on
y = 2x over x = 1..6, compile(X_train), predict([[7]]) in the clear and with
fhe="execute", |clear - FHE| < 0.01. Here fhe="execute" is
fheicp.sklearn.LinearRegression's packed encryption + leveled dot product +
decryption on the GPU (fhe_score_batch_key, no CPU fallback), and the value is
pinned to the committed fixture (tests/golden/quant_golden.json
"KAT_test_fhe": acc 38862, score 12.0000014; x = 7 lies above the calibration
max 6 and clips to q = 127).
"""
import json
from pathlib import Path

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

GOLD = json.loads((Path(__file__).parent / "golden" / "quant_golden.json").read_text())["KAT_test_fhe"]


def test_reference_test_fhe_through_hip(need_gpu):
    from fheicp.sklearn import LinearRegression
    from fheicp import _lib

    # test_fhe.py:13-14
    X_train = np.array([[1], [2], [3], [4], [5], [6]], dtype=np.float32)
    y_train = np.array([2, 4, 6, 8, 10, 12], dtype=np.float32)
    # :21-22
    model = LinearRegression(n_bits=8)
    model.fit(X_train, y_train)
    assert model.quant_params.to_dict() == GOLD["params"]
    # :29 (no key seed: 256-bit keys from os.urandom, as a deployment would)
    circuit = model.compile(X_train)
    width = model.fhe_circuit.graph.maximum_integer_bit_width()
    assert circuit is model.fhe_circuit and isinstance(width, int)
    lo, hi = model.quant_params.acc_range()
    assert hi - lo + 1 <= 2 ** (width - 1)          # the accumulator fits the encoding
    # :33-45
    test_value = np.array([[7]], dtype=np.float32)
    clear_pred = model.predict(test_value)
    fhe_pred = model.predict(test_value, fhe="execute")
    # the reference's own assertion (:55-60)
    assert abs(clear_pred[0] - fhe_pred[0]) < 0.01
    # bit-exact: the encrypted path equals the clear one and the fixture
    assert fhe_pred[0] == clear_pred[0] == GOLD["score"]
    assert round(fhe_pred[0] / model.quant_params.out_scale) == GOLD["acc"][0]
    # the encrypted decision on the same circuit (bootstrapped sign extraction)
    scores, keep = model.predict_threshold(test_value, 12.0)
    assert scores[0] == GOLD["score"] and bool(keep[0])
    scores, keep = model.predict_threshold(test_value, 12.01)
    assert not bool(keep[0])
    assert not _lib.ab_build()                       # the shipped library ran it
