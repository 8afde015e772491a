"""Versioned persistence of a compiled model: quantisation parameters + keys.

The reference cannot persist a compiled model (fhe_similarity.py:176-182,
:215-220 forces a retrain after load) and retrains + recompiles in every
process (batch_operations.py:78-108), so its results change run to run.
This file format makes a model reproducible across processes and GPUs
(SURVEY.md §8f-2):

    npz (no pickles; load with allow_pickle=False)
      meta     uint8[]  UTF-8 JSON {"format": "fheicp-model", "version": 1,
                        "quant": QuantParams.to_dict(), "scheme": SchemeParams}
      s_small, s_big, bsk, ksk   uint64[]  (optional; fhe_export_keys layout)

The key arrays hold the SECRET keys: protect the file like the reference's
key directory (key_management.py stores Fernet-encrypted blobs; the
``cryptography`` package is not available in this image, so wrapping the
file is left to the caller).
"""
from __future__ import annotations

import json
import os

import numpy as np

from .model import QuantParams
from .params import SchemeParams

FORMAT = "fheicp-model"
VERSION = 1
KEY_NAMES = ("s_small", "s_big", "bsk", "ksk")


def save_model(path: str, qparams: QuantParams, scheme: SchemeParams, keys: dict | None = None) -> None:
    meta = {"format": FORMAT, "version": VERSION, "quant": qparams.to_dict(), "scheme": scheme.as_dict()}
    arrays = {"meta": np.frombuffer(json.dumps(meta).encode(), dtype=np.uint8)}
    if keys is not None:
        for k in KEY_NAMES:
            arrays[k] = np.ascontiguousarray(keys[k], dtype=np.uint64)
    tmp = path + ".tmp.npz"
    np.savez(tmp, **arrays)
    os.replace(tmp, path)


def load_model(path: str):
    """-> (QuantParams, SchemeParams, keys dict or None)."""
    with np.load(path, allow_pickle=False) as z:
        meta = json.loads(bytes(z["meta"]).decode())
        if meta.get("format") != FORMAT:
            raise ValueError(f"{path}: not an {FORMAT} file")
        if int(meta.get("version", 0)) > VERSION:
            raise ValueError(f"{path}: format version {meta['version']} is newer than supported {VERSION}")
        keys = {k: z[k].copy() for k in KEY_NAMES} if all(k in z.files for k in KEY_NAMES) else None
    return QuantParams.from_dict(meta["quant"]), SchemeParams(**meta["scheme"]), keys


CORPUS_FORMAT = "fheicp-corpus"
CORPUS_VERSION = 1


def save_corpus(path: str, corpus) -> None:
    """Persist an EncryptedCorpus (fheicp.corpus): the model's quantisation,
    the corpus quantizer, the scheme, the PUBLIC mask key and the secret
    keys. Stored documents (seeded LWEs) are searchable again only with these
    keys; the session-local noise key is not stored (it is needed only to
    encrypt, and a fresh one is drawn per session)."""
    meta = {"format": CORPUS_FORMAT, "version": CORPUS_VERSION, "quant": corpus.cq.model.to_dict(),
            "corpus": corpus.cq.to_dict(), "P0": int(corpus.P0), "scheme": corpus.scheme.as_dict(),
            "mask_key": [int(x) for x in corpus.mask_key]}
    arrays = {"meta": np.frombuffer(json.dumps(meta).encode(), dtype=np.uint8)}
    keys = corpus.engine.export_keys()
    for k in KEY_NAMES:
        arrays[k] = np.ascontiguousarray(keys[k], dtype=np.uint64)
    tmp = path + ".tmp.npz"
    np.savez(tmp, **arrays)
    os.replace(tmp, path)


def load_corpus(path: str, device: int = 0):
    """-> a compiled EncryptedCorpus with the stored keys and mask key."""
    from .corpus import CorpusQuant, EncryptedCorpus
    with np.load(path, allow_pickle=False) as z:
        meta = json.loads(bytes(z["meta"]).decode())
        if meta.get("format") != CORPUS_FORMAT:
            raise ValueError(f"{path}: not an {CORPUS_FORMAT} file")
        if int(meta.get("version", 0)) > CORPUS_VERSION:
            raise ValueError(f"{path}: format version {meta['version']} is newer than supported {CORPUS_VERSION}")
        keys = {k: z[k].copy() for k in KEY_NAMES}
    cq = CorpusQuant(QuantParams.from_dict(meta["quant"]), int(meta["corpus"]["n_e"]), float(meta["corpus"]["s_e"]))
    c = EncryptedCorpus(cq, SchemeParams(**meta["scheme"]))
    if c.P0 != int(meta["P0"]):
        raise ValueError(f"{path}: stored P0 {meta['P0']} does not match the quantizer's {c.P0}")
    return c.compile(device=device, keys=keys, mask_key=np.asarray(meta["mask_key"], dtype=np.uint32))
