"""CPU: where the key material and the encryption stream get their entropy
(VERDICT r04 item 2), checked with a recording stand-in for the device engine
(no GPU here; the GPU side is tests/test_gpu_sessions.py).

- LinearRegression.compile() with no seed generates keys through the 256-bit
  fhe_keygen_key form from 32 bytes of os.urandom; the 64-bit fhe_keygen form
  runs only when a seed is given explicitly.
- Every compile draws its own 32-byte stream key and a random 64-bit id start,
  independent of the key seed; nothing of it is derived from the keys.
"""
import numpy as np
import pytest

from oracle import quant_ref as Q


class _RecordingEngine:
    calls: list = []

    def __init__(self, params, device=0):
        self.params = params

    def keygen(self, seed=None, key=None):
        _RecordingEngine.calls.append(("keygen", seed, key))

    def import_keys(self, keys):
        _RecordingEngine.calls.append(("import", None, None))

    def to_dev(self, a, dtype=None):
        return np.asarray(a)


@pytest.fixture
def fake_engine(monkeypatch):
    import fheicp.engine
    _RecordingEngine.calls = []
    monkeypatch.setattr(fheicp.engine, "Engine", _RecordingEngine)
    return _RecordingEngine


def _fitted():
    from fheicp.sklearn import LinearRegression
    X, y = Q.prepare_training_data(8, 200, seed=5)
    return LinearRegression(n_bits=4).fit(X, y), X


def test_compile_without_seed_uses_256_bit_keygen(fake_engine):
    est, X = _fitted()
    est.compile(X[:10])
    (kind, seed, key), = fake_engine.calls
    assert kind == "keygen" and seed is None
    assert isinstance(key, bytes) and len(key) == 32
    m = est._model
    assert isinstance(m.enc_seed, bytes) and len(m.enc_seed) == 32 and m.enc_seed != key
    # a second compile: fresh keys, a fresh stream key and a fresh id start
    first = (m.enc_seed, m._enc_counter)
    assert 0 <= first[1] < 2 ** 64
    est.compile(X[:10])
    (_, _, key2) = fake_engine.calls[1]
    assert key2 != key and (est._model.enc_seed, est._model._enc_counter) != first


def test_explicit_seed_selects_64_bit_form_only(fake_engine):
    est, X = _fitted()
    est.compile(X[:10], key_seed=1234)
    assert fake_engine.calls == [("keygen", 1234, None)]
    m = est._model
    # the stream key is still session-random: not a function of key_seed
    assert isinstance(m.enc_seed, bytes) and len(m.enc_seed) == 32
    first = (m.enc_seed, m._enc_counter)
    est.compile(X[:10], key_seed=1234)
    assert (est._model.enc_seed, est._model._enc_counter) != first


def test_imported_keys_never_call_keygen(fake_engine):
    from fheicp.model import FheLinearModel
    X, y = Q.prepare_training_data(8, 200, seed=6)
    m = FheLinearModel.fit(X, y, n_bits=4).compile(keys={"any": 1})
    assert fake_engine.calls == [("import", None, None)]
    assert isinstance(m.enc_seed, bytes)


def test_stream_ids_advance_mod_2_64(fake_engine):
    from fheicp.model import FheLinearModel
    X, y = Q.prepare_training_data(8, 200, seed=7)
    m = FheLinearModel.fit(X, y, n_bits=4).compile()
    m._enc_counter = 2 ** 64 - 3
    assert m.next_id0(8) == 2 ** 64 - 3
    assert m.next_id0(1) == 5


def test_enc_seed_is_the_test_form(fake_engine):
    from fheicp.model import FheLinearModel
    X, y = Q.prepare_training_data(8, 200, seed=8)
    m = FheLinearModel.fit(X, y, n_bits=4).compile(key_seed=3, enc_seed=99)
    assert m.enc_seed == 99 and m.next_id0(4) == 0 and m.next_id0(1) == 4


def test_header_marks_seed_forms_non_production():
    from pathlib import Path
    h = (Path(__file__).resolve().parents[1] / "include" / "fhe_icp.h").read_text()
    for name in ("fhe_keygen_key", "fhe_compare_batch_key", "fhe_score_batch_key", "fhe_encrypt_linear_batch_key",
                 "fhe_encrypt_packed_batch_key", "fhe_encrypt_batch_key"):
        assert f"int {name}(" in h
    assert "NOT for production keys" in h
