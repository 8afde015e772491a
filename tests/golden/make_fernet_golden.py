#!/opt/conda/bin/python3.9
"""Fixture generator for fheicp.fernet (run with the image's conda Python 3.9,
which has cryptography 3.4.8 — the library the reference's key manager uses,
key_management.py:13-15; not reference code). Writes fernet_golden.json:
tokens for fixed keys / IVs / timestamps and PBKDF2 master keys."""
import base64
import json
from pathlib import Path

from cryptography.fernet import Fernet
from cryptography.hazmat.primitives import hashes
from cryptography.hazmat.primitives.kdf.pbkdf2 import PBKDF2HMAC


def master(password, salt, iterations):
    kdf = PBKDF2HMAC(algorithm=hashes.SHA256(), length=32, salt=salt, iterations=iterations)
    return base64.urlsafe_b64encode(kdf.derive(password.encode())).decode()


out = {"tokens": [], "pbkdf2": []}
for i, msg in enumerate([b"", b"test", b"hello", bytes(range(256)) * 3, b"\x00" * 16, b"x" * 15]):
    key = base64.urlsafe_b64encode(bytes((7 * i + j) & 0xFF for j in range(32)))
    iv = bytes((11 * i + 3 * j) & 0xFF for j in range(16))
    ts = 499162800 + 1000 * i
    tok = Fernet(key)._encrypt_from_parts(msg, ts, iv)
    out["tokens"].append({"key": key.decode(), "iv": iv.hex(), "time": ts, "msg": msg.hex(), "token": tok.decode()})
for pw, salt, it in [("correct horse", b"\x01" * 16, 100000), ("", bytes(range(16)), 1000), ("pässwörd", b"salt-16-bytes!!!", 100000)]:
    out["pbkdf2"].append({"password": pw, "salt": salt.hex(), "iterations": it, "key": master(pw, salt, it)})
Path(__file__).with_name("fernet_golden.json").write_text(json.dumps(out, indent=1) + "\n")
print("wrote", len(out["tokens"]), "tokens")
