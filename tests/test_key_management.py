"""CPU: Fernet / PBKDF2 without `cryptography` (pinned to FIPS-197 and to
tokens made by cryptography 3.4.8, tests/golden/make_fernet_golden.py) and the
FHEKeyManager mirror's files, metadata, errors and key round trip."""
import base64
import json
import os
import pickle
from pathlib import Path

import numpy as np
import pytest

from fheicp import fernet as F

GOLD = json.loads((Path(__file__).parent / "golden" / "fernet_golden.json").read_text())


def test_aes128_fips197_c1():
    rk = F._expand_key(bytes(range(16)))
    pt = bytes.fromhex("00112233445566778899aabbccddeeff")
    ct = F.aes128_encrypt_block(rk, pt)
    assert ct.hex() == "69c4e0d86a7b0430d8cdb78070b4c55a"
    assert F.aes128_decrypt_block(rk, ct) == pt


@pytest.mark.parametrize("case", range(len(GOLD["tokens"])))
def test_fernet_matches_cryptography(case):
    g = GOLD["tokens"][case]
    f = F.Fernet(g["key"].encode())
    msg = bytes.fromhex(g["msg"])
    tok = f._encrypt_from_parts(msg, g["time"], bytes.fromhex(g["iv"]))
    assert tok.decode() == g["token"]
    assert f.decrypt(g["token"].encode()) == msg


def test_fernet_rejects_tampering_and_wrong_keys():
    g = GOLD["tokens"][2]
    f = F.Fernet(g["key"].encode())
    raw = bytearray(base64.urlsafe_b64decode(g["token"]))
    for pos in (0, 5, 30, len(raw) - 40, len(raw) - 1):
        bad = bytearray(raw)
        bad[pos] ^= 1
        with pytest.raises(F.InvalidToken):
            f.decrypt(base64.urlsafe_b64encode(bytes(bad)))
    with pytest.raises(F.InvalidToken):
        F.Fernet(F.Fernet.generate_key()).decrypt(g["token"].encode())
    with pytest.raises(F.InvalidToken):
        f.decrypt(g["token"].encode(), ttl=60)   # issued in 1985
    with pytest.raises(ValueError):
        F.Fernet(base64.urlsafe_b64encode(b"short"))
    f2 = F.Fernet(F.Fernet.generate_key())
    assert f2.decrypt(f2.encrypt(b"round trip" * 50)) == b"round trip" * 50


@pytest.mark.parametrize("case", range(len(GOLD["pbkdf2"])))
def test_master_key_derivation_matches_cryptography(case):
    g = GOLD["pbkdf2"][case]
    assert F.derive_master_key(g["password"], bytes.fromhex(g["salt"]), g["iterations"]).decode() == g["key"]


@pytest.fixture(scope="module")
def toy_material(oracle_lib):
    from fheicp.model import FheLinearModel
    from fheicp.params import TOY
    from oracle import quant_ref as Q
    X, y = Q.prepare_training_data(8, 500, seed=3)
    qp = FheLinearModel.fit(X, y, 4).qparams
    ref = oracle_lib.RefTFHE(TOY.as_dict(), 55)
    keys = {"s_small": ref.s_small, "s_big": ref.s_big, "bsk": ref.bsk, "ksk": ref.ksk}
    return qp, TOY, keys


def test_key_manager_layout_and_round_trip(tmp_path, toy_material):
    from key_management import FHEKeyManager
    qp, scheme, keys = toy_material
    km = FHEKeyManager(str(tmp_path / "keys"), password="hunter2")
    assert km.get_current_key() is None and km.list_keys() == {}
    out = km.store_keys("k1", qp, scheme, keys, {"input_dim": 8, "n_bits": 4, "similarity_type": "cosine",
                                                 "metrics": {"train_score": 0.9}})
    assert out["key_id"] == "k1" and km.get_current_key() == "k1"
    master = json.loads((tmp_path / "keys" / ".master").read_text())
    assert set(master) == {"salt", "test", "created"}
    meta = json.loads((tmp_path / "keys" / "key_metadata.json").read_text())
    assert meta["current"] == "k1"
    assert {"created", "path", "active", "model_file", "size_bytes"} <= set(meta["keys"]["k1"])
    mf = Path(meta["keys"]["k1"]["model_file"])
    assert mf.name == "compiled_model.enc" and oct(mf.stat().st_mode & 0o777) == "0o600"
    assert mf.stat().st_size == meta["keys"]["k1"]["size_bytes"]
    # a fresh manager (new process) with the password reads everything back
    km2 = FHEKeyManager(str(tmp_path / "keys"), password="hunter2")
    data = km2.load_model()
    assert data["input_dim"] == 8 and data["compiled"] is True and data["metrics"] == {"train_score": 0.9}
    qp2, scheme2, keys2 = km2.load_key_material()
    assert qp2.to_dict() == qp.to_dict() and scheme2 == scheme
    for k in keys:
        np.testing.assert_array_equal(keys2[k], keys[k])
    # the token is a Fernet token under the PBKDF2 master key
    key = F.derive_master_key("hunter2", base64.b64decode(master["salt"]))
    assert pickle.loads(F.Fernet(key).decrypt(mf.read_bytes()))["n_bits"] == 4


def test_key_manager_errors(tmp_path, toy_material, monkeypatch):
    from key_management import FHEKeyManager
    qp, scheme, keys = toy_material
    km = FHEKeyManager(str(tmp_path / "k"), password="right")
    km.store_keys("a", qp, scheme, keys, {"input_dim": 8, "n_bits": 4})
    with pytest.raises(ValueError, match="Invalid master password"):
        FHEKeyManager(str(tmp_path / "k"), password="wrong").load_model()
    with pytest.raises(ValueError, match="not found"):
        km.load_model("missing")
    answers = iter(["one", "two"])
    km3 = FHEKeyManager(str(tmp_path / "fresh"))
    monkeypatch.setattr(km3, "_ask", lambda prompt: next(answers))
    with pytest.raises(ValueError, match="Passwords don't match"):
        km3._get_master_key()
    with pytest.raises(ValueError, match="No current key"):
        FHEKeyManager(str(tmp_path / "empty"), password="x").load_model()


def test_reference_written_key_and_unsafe_pickles(tmp_path):
    """A key written the reference's way (a Fernet token of the pickled config
    dict, key_management.py:150-166) loads as a dict but has no key material;
    a token carrying anything but plain data is refused."""
    from key_management import FHEKeyManager
    km = FHEKeyManager(str(tmp_path / "k"), password="pw")
    f = F.Fernet(km._get_master_key())
    kp = tmp_path / "k" / "ref_key"
    kp.mkdir()
    ref_data = {"input_dim": 128, "n_bits": 8, "similarity_type": "cosine", "metrics": {"train_time": 1.5},
                "compiled": True}
    (kp / "compiled_model.enc").write_bytes(f.encrypt(pickle.dumps(ref_data)))
    meta = {"keys": {"ref_key": {"created": "2025-01-01", "path": str(kp), "active": True,
                                 "model_file": str(kp / "compiled_model.enc"), "size_bytes": 1}},
            "current": "ref_key"}
    (tmp_path / "k" / "key_metadata.json").write_text(json.dumps(meta))
    assert km.load_model() == ref_data
    with pytest.raises(ValueError, match="no fheicp key material"):
        km.load_key_material()
    import datetime
    (kp / "compiled_model.enc").write_bytes(f.encrypt(pickle.dumps({"when": datetime.date(2020, 1, 1)})))
    with pytest.raises(pickle.UnpicklingError):
        km.load_model()
