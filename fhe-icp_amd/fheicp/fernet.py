"""Fernet tokens (AES-128-CBC + HMAC-SHA256) and the PBKDF2 master key of the
reference's key manager, without the ``cryptography`` package.

The reference wraps its key material with ``cryptography.fernet.Fernet`` under
a key derived by PBKDF2-HMAC-SHA256 (100 000 iterations) from the master
password (key_management.py:49-58, :97-105, :146-165, :230-235). That package
is not importable in this image, so this module implements the published
Fernet spec directly:

    token = urlsafe_b64( 0x80 | timestamp (u64 BE) | IV (16) | AES-128-CBC(PKCS7(msg)) | HMAC )
    HMAC  = HMAC-SHA256(signing_key, everything before it)
    key   = urlsafe_b64(signing_key (16) | encryption_key (16))

AES-128 is FIPS-197, in Python: it only ever wraps the secret keys and the
quantizer parameters (tens of KB), never the public evaluation keys. Parity:
tests/test_key_management.py checks FIPS-197 Appendix C.1 and tokens / PBKDF2
keys produced by ``cryptography`` 3.4.8 (tests/golden/make_fernet_golden.py).
"""
from __future__ import annotations

import base64
import hashlib
import hmac
import os
import struct
import time


class InvalidToken(Exception):
    """Bad signature, malformed token or bad padding (cryptography.fernet.InvalidToken)."""


# --------------------------------------------------------------- AES-128 ---
def _xtime(a: int) -> int:
    a <<= 1
    return (a ^ 0x11B) & 0xFF if a & 0x100 else a


def _gmul(a: int, b: int) -> int:
    r = 0
    while b:
        if b & 1:
            r ^= a
        a = _xtime(a)
        b >>= 1
    return r


def _make_sbox():
    sbox = [0] * 256
    inv = [0] * 256
    for x in range(256):
        # multiplicative inverse in GF(2^8) (0 -> 0), then the affine map
        y = 0 if x == 0 else next(c for c in range(1, 256) if _gmul(x, c) == 1)
        s = y
        for k in range(1, 5):
            s ^= ((y << k) | (y >> (8 - k))) & 0xFF
        s ^= 0x63
        sbox[x] = s
        inv[s] = x
    return sbox, inv


SBOX, INV_SBOX = _make_sbox()
_M2 = [_gmul(x, 2) for x in range(256)]
_M3 = [_gmul(x, 3) for x in range(256)]
_M9 = [_gmul(x, 9) for x in range(256)]
_M11 = [_gmul(x, 11) for x in range(256)]
_M13 = [_gmul(x, 13) for x in range(256)]
_M14 = [_gmul(x, 14) for x in range(256)]


def _expand_key(key: bytes):
    assert len(key) == 16
    w = [list(key[4 * i:4 * i + 4]) for i in range(4)]
    rcon = 1
    for i in range(4, 44):
        t = list(w[i - 1])
        if i % 4 == 0:
            t = [SBOX[b] for b in t[1:] + t[:1]]
            t[0] ^= rcon
            rcon = _xtime(rcon)
        w.append([a ^ b for a, b in zip(w[i - 4], t)])
    return [sum((w[4 * r + c] for c in range(4)), []) for r in range(11)]


def _shift(s, inv=False):
    # state is column-major: s[r + 4c]
    out = [0] * 16
    for r in range(4):
        for c in range(4):
            src = (c - r) % 4 if inv else (c + r) % 4
            out[r + 4 * c] = s[r + 4 * src]
    return out


def aes128_encrypt_block(rk, block: bytes) -> bytes:
    s = [b ^ k for b, k in zip(block, rk[0])]
    for rnd in range(1, 11):
        s = _shift([SBOX[b] for b in s])
        if rnd < 10:
            m = []
            for c in range(4):
                a0, a1, a2, a3 = s[4 * c:4 * c + 4]
                m += [_M2[a0] ^ _M3[a1] ^ a2 ^ a3, a0 ^ _M2[a1] ^ _M3[a2] ^ a3,
                      a0 ^ a1 ^ _M2[a2] ^ _M3[a3], _M3[a0] ^ a1 ^ a2 ^ _M2[a3]]
            s = m
        s = [b ^ k for b, k in zip(s, rk[rnd])]
    return bytes(s)


def aes128_decrypt_block(rk, block: bytes) -> bytes:
    s = [b ^ k for b, k in zip(block, rk[10])]
    for rnd in range(9, -1, -1):
        s = [INV_SBOX[b] for b in _shift(s, inv=True)]
        s = [b ^ k for b, k in zip(s, rk[rnd])]
        if rnd > 0:
            m = []
            for c in range(4):
                a0, a1, a2, a3 = s[4 * c:4 * c + 4]
                m += [_M14[a0] ^ _M11[a1] ^ _M13[a2] ^ _M9[a3], _M9[a0] ^ _M14[a1] ^ _M11[a2] ^ _M13[a3],
                      _M13[a0] ^ _M9[a1] ^ _M14[a2] ^ _M11[a3], _M11[a0] ^ _M13[a1] ^ _M9[a2] ^ _M14[a3]]
            s = m
    return bytes(s)


def _cbc_encrypt(key: bytes, iv: bytes, data: bytes) -> bytes:
    pad = 16 - len(data) % 16
    data = data + bytes([pad]) * pad
    rk = _expand_key(key)
    out, prev = bytearray(), iv
    for i in range(0, len(data), 16):
        prev = aes128_encrypt_block(rk, bytes(a ^ b for a, b in zip(data[i:i + 16], prev)))
        out += prev
    return bytes(out)


def _cbc_decrypt(key: bytes, iv: bytes, data: bytes) -> bytes:
    if not data or len(data) % 16:
        raise InvalidToken("ciphertext is not a whole number of blocks")
    rk = _expand_key(key)
    out, prev = bytearray(), iv
    for i in range(0, len(data), 16):
        blk = data[i:i + 16]
        out += bytes(a ^ b for a, b in zip(aes128_decrypt_block(rk, blk), prev))
        prev = blk
    pad = out[-1]
    if not 1 <= pad <= 16 or out[-pad:] != bytes([pad]) * pad:
        raise InvalidToken("bad padding")
    return bytes(out[:-pad])


# ---------------------------------------------------------------- Fernet ---
class Fernet:
    """Same constructor and encrypt/decrypt contract as cryptography.fernet.Fernet."""

    def __init__(self, key):
        raw = base64.urlsafe_b64decode(key)
        if len(raw) != 32:
            raise ValueError("Fernet key must be 32 url-safe base64-encoded bytes.")
        self._signing_key, self._encryption_key = raw[:16], raw[16:]

    @staticmethod
    def generate_key() -> bytes:
        return base64.urlsafe_b64encode(os.urandom(32))

    def encrypt(self, data: bytes) -> bytes:
        return self._encrypt_from_parts(data, int(time.time()), os.urandom(16))

    def _encrypt_from_parts(self, data: bytes, current_time: int, iv: bytes) -> bytes:
        body = b"\x80" + struct.pack(">Q", current_time) + iv + _cbc_encrypt(self._encryption_key, iv, data)
        return base64.urlsafe_b64encode(body + hmac.new(self._signing_key, body, hashlib.sha256).digest())

    def decrypt(self, token: bytes, ttl: int | None = None) -> bytes:
        try:
            raw = base64.urlsafe_b64decode(token)
        except (TypeError, ValueError) as e:
            raise InvalidToken("token is not url-safe base64") from e
        if len(raw) < 1 + 8 + 16 + 16 + 32 or raw[0] != 0x80:
            raise InvalidToken("malformed token")
        body, mac = raw[:-32], raw[-32:]
        if not hmac.compare_digest(hmac.new(self._signing_key, body, hashlib.sha256).digest(), mac):
            raise InvalidToken("signature mismatch")
        if ttl is not None:
            (ts,) = struct.unpack(">Q", body[1:9])
            if ts + ttl < int(time.time()):
                raise InvalidToken("token expired")
        return _cbc_decrypt(self._encryption_key, body[9:25], body[25:])


def derive_master_key(password: str, salt: bytes, iterations: int = 100_000) -> bytes:
    """key_management.py:49-58: PBKDF2HMAC(SHA256, length 32, salt, 100000), url-safe base64."""
    return base64.urlsafe_b64encode(hashlib.pbkdf2_hmac("sha256", password.encode(), salt, iterations, 32))
