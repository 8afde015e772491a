"""Versioned persistence of a compiled model: quantisation parameters + keys.

The reference cannot persist a compiled model (fhe_similarity.py:176-182,
:215-220 forces a retrain after load) and retrains + recompiles in every
process (batch_operations.py:78-108), so its results change run to run.
This file format makes a model reproducible across processes and GPUs
(SURVEY.md §8f-2):

    npz (no pickles; load with allow_pickle=False), mode 0600
      meta     uint8[]  UTF-8 JSON {"format": "fheicp-model", "version": 2,
                        "quant": QuantParams.to_dict(), "scheme": SchemeParams,
                        "secret": {"kdf": "pbkdf2-sha256", "iterations", "salt",
                                   "bits": {"s_small": n, "s_big": kN}}}
      secret   uint8[]  Fernet token of the bit-packed secret keys (s_small,
                        s_big), under PBKDF2-HMAC-SHA256(password, salt) as
                        the reference's key manager derives its master key
                        (key_management.py:49-58, :146-165)
      bsk, ksk uint64[] the PUBLIC evaluation keys (encryptions under the
                        secret key), fhe_export_keys layout

The password comes from ``password=`` or ``$FHE_MASTER_PASSWORD``; without
one, saving secret keys raises unless ``allow_plaintext_secrets=True`` (then
s_small / s_big are stored as plain uint64 arrays, as version-1 files did).
Version 2 marks the format with the Fernet-wrapped ``secret`` blob. Files
an earlier release wrote as version 1 hold either plaintext s_small / s_big
or, when it was given a password, that same ``secret`` blob under the same
``meta["secret"]`` entry: both still load (``_read_secrets`` goes by whether
the blob is present, not by the version). ``load_model(..., keys=False)``
reads only the quantisation and scheme (the clear modes need no secret).
"""
from __future__ import annotations

import base64
import json
import os

import numpy as np

from .fernet import Fernet, InvalidToken, derive_master_key
from .model import QuantParams
from .params import SchemeParams

FORMAT = "fheicp-model"
VERSION = 2                 # 2: Fernet-wrapped "secret" blob; 1: plaintext keys or the same blob
KEY_NAMES = ("s_small", "s_big", "bsk", "ksk")
SECRET_NAMES = ("s_small", "s_big")
KDF_ITERATIONS = 100_000


def _password(password):
    return password if password is not None else os.environ.get("FHE_MASTER_PASSWORD")


def _secret_arrays(keys: dict, password, allow_plaintext: bool, meta: dict) -> dict:
    """The secret keys as a Fernet-wrapped bit-packed blob (or, opted in, plain)."""
    pw = _password(password)
    if pw is None:
        if not allow_plaintext:
            raise ValueError("saving secret keys needs a password (password= or $FHE_MASTER_PASSWORD); "
                             "pass allow_plaintext_secrets=True to store them unencrypted")
        return {k: np.ascontiguousarray(keys[k], dtype=np.uint64) for k in SECRET_NAMES}
    parts, bits = [], {}
    for k in SECRET_NAMES:
        a = np.ascontiguousarray(keys[k], dtype=np.uint64)
        if a.size and int(a.max()) > 1:
            raise ValueError(f"{k} is not a binary secret key")
        parts.append(np.packbits(a.astype(np.uint8)).tobytes())
        bits[k] = int(a.size)
    salt = os.urandom(16)
    token = Fernet(derive_master_key(pw, salt, KDF_ITERATIONS)).encrypt(b"".join(parts))
    meta["secret"] = {"kdf": "pbkdf2-sha256", "iterations": KDF_ITERATIONS,
                      "salt": base64.b64encode(salt).decode(), "bits": bits}
    return {"secret": np.frombuffer(token, dtype=np.uint8)}


def _read_secrets(z, meta: dict, password, path: str) -> dict:
    if "secret" not in z.files:
        return {k: z[k].copy() for k in SECRET_NAMES}
    pw = _password(password)
    if pw is None:
        raise ValueError(f"{path}: the secret keys are encrypted; pass password= or set $FHE_MASTER_PASSWORD")
    sm = meta["secret"]
    key = derive_master_key(pw, base64.b64decode(sm["salt"]), int(sm["iterations"]))
    try:
        blob = Fernet(key).decrypt(bytes(z["secret"]))
    except InvalidToken:
        raise ValueError(f"{path}: wrong password for the secret keys") from None
    out, off = {}, 0
    for k in SECRET_NAMES:
        n = int(sm["bits"][k])
        nb = (n + 7) // 8
        out[k] = np.unpackbits(np.frombuffer(blob[off:off + nb], dtype=np.uint8))[:n].astype(np.uint64)
        off += nb
    return out


def _write_private(path: str, arrays: dict) -> None:
    """np.savez to path, created with mode 0600 (it may hold secrets)."""
    tmp = path + ".tmp.npz"
    fd = os.open(tmp, os.O_WRONLY | os.O_CREAT | os.O_TRUNC, 0o600)
    with os.fdopen(fd, "wb") as f:
        np.savez(f, **arrays)
    os.chmod(tmp, 0o600)
    os.replace(tmp, path)


def save_model(path: str, qparams: QuantParams, scheme: SchemeParams, keys: dict | None = None,
               password: str | None = None, allow_plaintext_secrets: bool = False) -> None:
    meta = {"format": FORMAT, "version": VERSION, "quant": qparams.to_dict(), "scheme": scheme.as_dict()}
    arrays = {}
    if keys is not None:
        arrays.update(_secret_arrays(keys, password, allow_plaintext_secrets, meta))
        for k in ("bsk", "ksk"):
            arrays[k] = np.ascontiguousarray(keys[k], dtype=np.uint64)
    arrays["meta"] = np.frombuffer(json.dumps(meta).encode(), dtype=np.uint8)
    _write_private(path, arrays)


def _check_version(path: str, meta: dict, supported: int) -> None:
    v = int(meta.get("version", 0))
    if not 1 <= v <= supported:
        raise ValueError(f"{path}: format version {meta.get('version')} is not supported (1..{supported})")


def load_model(path: str, password: str | None = None, keys: bool = True):
    """-> (QuantParams, SchemeParams, keys dict or None). keys=False skips the
    key material (and so needs no password)."""
    want_keys = keys
    with np.load(path, allow_pickle=False) as z:
        meta = json.loads(bytes(z["meta"]).decode())
        if meta.get("format") != FORMAT:
            raise ValueError(f"{path}: not an {FORMAT} file")
        _check_version(path, meta, VERSION)
        keys = None
        if want_keys and "bsk" in z.files and "ksk" in z.files:
            keys = {"bsk": z["bsk"].copy(), "ksk": z["ksk"].copy()}
            keys.update(_read_secrets(z, meta, password, path))
    return QuantParams.from_dict(meta["quant"]), SchemeParams(**meta["scheme"]), keys


CORPUS_FORMAT = "fheicp-corpus"
CORPUS_VERSION = 2          # as VERSION


def save_corpus(path: str, corpus, password: str | None = None, allow_plaintext_secrets: bool = False) -> None:
    """Persist an EncryptedCorpus (fheicp.corpus): the model's quantisation,
    the corpus quantizer, the scheme, the PUBLIC mask key and the secret
    keys (Fernet-wrapped as in save_model). Stored documents (seeded LWEs) are
    searchable again only with these keys; the session-local noise key is not
    stored (it is needed only to encrypt, and a fresh one is drawn per
    session)."""
    meta = {"format": CORPUS_FORMAT, "version": CORPUS_VERSION, "quant": corpus.cq.model.to_dict(),
            "corpus": corpus.cq.to_dict(), "P0": int(corpus.P0), "scheme": corpus.scheme.as_dict(),
            "mask_key": [int(x) for x in corpus.mask_key]}
    keys = corpus.engine.export_keys()
    arrays = _secret_arrays(keys, password, allow_plaintext_secrets, meta)
    for k in ("bsk", "ksk"):
        arrays[k] = np.ascontiguousarray(keys[k], dtype=np.uint64)
    arrays["meta"] = np.frombuffer(json.dumps(meta).encode(), dtype=np.uint8)
    _write_private(path, arrays)


def load_corpus(path: str, device: int = 0, password: str | None = None):
    """-> a compiled EncryptedCorpus with the stored keys and mask key."""
    from .corpus import CorpusQuant, EncryptedCorpus
    with np.load(path, allow_pickle=False) as z:
        meta = json.loads(bytes(z["meta"]).decode())
        if meta.get("format") != CORPUS_FORMAT:
            raise ValueError(f"{path}: not an {CORPUS_FORMAT} file")
        _check_version(path, meta, CORPUS_VERSION)
        keys = {"bsk": z["bsk"].copy(), "ksk": z["ksk"].copy()}
        keys.update(_read_secrets(z, meta, password, path))
    cq = CorpusQuant(QuantParams.from_dict(meta["quant"]), int(meta["corpus"]["n_e"]), float(meta["corpus"]["s_e"]))
    c = EncryptedCorpus(cq, SchemeParams(**meta["scheme"]))
    if c.P0 != int(meta["P0"]):
        raise ValueError(f"{path}: stored P0 {meta['P0']} does not match the quantizer's {c.P0}")
    return c.compile(device=device, keys=keys, mask_key=np.asarray(meta["mask_key"], dtype=np.uint32))
