"""Document store with the reference's on-disk format, plus a batched corpus view.

Mirrors ``encrypted_storage`` of the reference (encrypted_storage.py:19-230):
the same module and class names, so a ``<doc_id>.enc`` file written by either
side unpickles into the other (the pickle class path is
``encrypted_storage.EncryptedDocument``), the same ``index.json`` schema
(:96-104) and the same errors (KeyError for an unknown id :120-121,
FileNotFoundError for a missing file :126-127).

Changes for the GPU search path:
  * the embedding width check accepts any configured D (``allowed_dims``),
    defaulting to the reference's (128, 256); the BASELINE configs use 8-768;
  * ``save_many`` writes a batch of documents and rewrites the index once;
  * ``corpus()`` returns ids and a stacked float32 [B, D] matrix in index
    order — the order that decides ties in search (:136-141) — cached until
    the store changes, so a search uploads the corpus to HBM once;
  * documents may carry a real ciphertext instead of the plaintext vector
    (§8f-1): ``model_version == "fheicp-seeded-lwe-v1"`` marks an
    ``encrypted_embedding`` that is a versioned seeded-LWE payload
    (fheicp.corpus); ``encrypted_corpus()`` stacks those payloads.
"""
from __future__ import annotations

import gzip
import json
import logging
import os
import pickle
from dataclasses import dataclass, field
from pathlib import Path
from typing import Any, Dict, List, Optional, Sequence

import numpy as np

logger = logging.getLogger(__name__)

DEFAULT_DIMS = (128, 256)
CIPHERTEXT_VERSION = "fheicp-seeded-lwe-v1"   # fheicp.corpus.PAYLOAD_VERSION


@dataclass
class EncryptedDocument:
    """One stored document (field order and defaults as encrypted_storage.py:19-28)."""
    doc_id: str
    content_hash: str
    timestamp: str
    encrypted_embedding: np.ndarray
    model_version: str = "1.0"
    key_id: Optional[str] = None
    metadata: Dict[str, Any] = field(default_factory=dict)

    # Widths accepted by validation; set per process (EncryptedDocument.allowed_dims = (16,))
    # or None for any width. Class attribute, not a dataclass field: not pickled.
    allowed_dims = DEFAULT_DIMS

    def __post_init__(self):
        emb = self.encrypted_embedding
        if emb is None:
            return
        if not isinstance(emb, np.ndarray):
            raise TypeError("encrypted_embedding must be numpy array")
        if emb.ndim != 1:
            raise ValueError(f"Expected 1D embedding, got shape {emb.shape}")
        if self.model_version == CIPHERTEXT_VERSION:
            from fheicp.corpus import unpack_payload
            unpack_payload(emb)  # raises ValueError on a malformed payload
            return
        dims = type(self).allowed_dims
        if dims is not None and emb.shape[0] not in dims:
            raise ValueError(f"Expected embedding width in {tuple(dims)}, got {emb.shape}")

    validate = __post_init__

    def to_bytes(self) -> bytes:
        return gzip.compress(pickle.dumps(self))

    @classmethod
    def from_bytes(cls, data: bytes) -> "EncryptedDocument":
        # The stored format is a gzip'd pickle (encrypted_storage.py:40-47):
        # only open stores you wrote yourself.
        return pickle.loads(gzip.decompress(data))

    def size_bytes(self) -> int:
        return len(self.to_bytes())


class EncryptedDocumentStore:
    """Directory of ``<doc_id>.enc`` files plus ``index.json``."""

    def __init__(self, storage_dir: str = "./encrypted_docs"):
        self.storage_dir = Path(storage_dir)
        self.storage_dir.mkdir(parents=True, exist_ok=True)
        self.index_file = self.storage_dir / "index.json"
        self.index: Dict[str, Dict[str, Any]] = self._load_index()
        self._corpus_cache = None
        self._ct_cache = None

    # ------------------------------------------------------------ writes --
    def _write_doc(self, doc: EncryptedDocument) -> Path:
        doc.validate()
        name = f"{doc.doc_id}.enc"
        blob = doc.to_bytes()
        (self.storage_dir / name).write_bytes(blob)
        self.index[doc.doc_id] = {
            "filename": name,
            "timestamp": doc.timestamp,
            "content_hash": doc.content_hash,
            "size_bytes": len(blob),
            "model_version": doc.model_version,
            "key_id": doc.key_id,
            "metadata": doc.metadata,
        }
        self._corpus_cache = None
        self._ct_cache = None
        return self.storage_dir / name

    def save(self, doc: EncryptedDocument) -> str:
        path = self._write_doc(doc)
        self._save_index()
        return str(path)

    def save_many(self, docs: Sequence[EncryptedDocument]) -> List[str]:
        paths = [str(self._write_doc(d)) for d in docs]
        self._save_index()
        return paths

    def delete(self, doc_id: str) -> bool:
        info = self.index.pop(doc_id, None)
        if info is None:
            return False
        f = self.storage_dir / info["filename"]
        if f.exists():
            f.unlink()
        self._corpus_cache = None
        self._ct_cache = None
        self._save_index()
        return True

    # ------------------------------------------------------------- reads --
    def load(self, doc_id: str) -> EncryptedDocument:
        if doc_id not in self.index:
            raise KeyError(f"Document {doc_id} not found")
        f = self.storage_dir / self.index[doc_id]["filename"]
        if not f.exists():
            raise FileNotFoundError(f"Document file missing: {f}")
        return EncryptedDocument.from_bytes(f.read_bytes())

    def list_documents(self) -> List[Dict[str, Any]]:
        return [dict(doc_id=k, **v) for k, v in self.index.items()]

    def search_by_metadata(self, key: str, value: Any) -> List[str]:
        return [k for k, v in self.index.items() if v.get("metadata", {}).get(key, _MISSING) == value]

    def get_stats(self) -> Dict[str, Any]:
        sizes = [v["size_bytes"] for v in self.index.values()]
        total = int(sum(sizes))
        return {
            "total_documents": len(sizes),
            "total_size_bytes": total,
            "total_size_mb": total / 1024 / 1024,
            "average_size_bytes": total / len(sizes) if sizes else 0,
            "storage_dir": str(self.storage_dir),
        }

    def validate_all(self) -> Dict[str, List[str]]:
        out: Dict[str, List[str]] = {"valid": [], "invalid": []}
        for doc_id in self.index:
            try:
                self.load(doc_id).validate()
                out["valid"].append(doc_id)
            except Exception as e:  # noqa: BLE001 - report every failure kind
                logger.error("validation failed for %s: %s", doc_id, e)
                out["invalid"].append(doc_id)
        return out

    def corpus(self):
        """(doc_ids in index order, [B, D] embeddings in their stored dtype). Cached."""
        if self._corpus_cache is None:
            ids = list(self.index.keys())
            if not ids:
                self._corpus_cache = ([], np.zeros((0, 0), np.float32))
            else:
                loaded = [self.load(i) for i in ids]
                if any(d.model_version == CIPHERTEXT_VERSION for d in loaded):
                    raise ValueError("store holds ciphertext documents: use encrypted_corpus()")
                rows = [np.asarray(d.encrypted_embedding) for d in loaded]
                widths = {r.shape[0] for r in rows}
                if len(widths) != 1:
                    raise ValueError(f"store mixes embedding widths {sorted(widths)}")
                kinds = {r.dtype for r in rows}
                if len(kinds) != 1:
                    # per-document numpy promotion of query * doc would differ by row
                    raise ValueError(f"store mixes embedding dtypes {sorted(map(str, kinds))}")
                self._corpus_cache = (ids, np.stack(rows))
        return self._corpus_cache

    def encrypted_corpus(self):
        """(doc_ids in index order, bodies uint64 [B, D], stream ids uint64 [B],
        payload header {P0, mask_key, big, D}) of a store of ciphertext
        documents. Cached like corpus()."""
        if self._ct_cache is None:
            from fheicp.corpus import unpack_payload
            ids = list(self.index.keys())
            if not ids:
                self._ct_cache = ([], np.zeros((0, 0), np.uint64), np.zeros(0, np.uint64), None)
            else:
                pls = []
                for i in ids:
                    d = self.load(i)
                    if d.model_version != CIPHERTEXT_VERSION:
                        raise ValueError(f"document {i} is not a ciphertext document")
                    pls.append(unpack_payload(d.encrypted_embedding))
                head = {k: pls[0][k] for k in ("P0", "big", "D", "mask_key")}
                for p in pls[1:]:
                    if (p["P0"], p["big"], p["D"]) != (head["P0"], head["big"], head["D"]) or \
                            not np.array_equal(p["mask_key"], head["mask_key"]):
                        raise ValueError("store mixes ciphertext parameters or mask keys")
                self._ct_cache = (ids, np.stack([p["body"] for p in pls]),
                                  np.array([p["id0"] for p in pls], dtype=np.uint64), head)
        return self._ct_cache

    def holds_ciphertexts(self) -> bool:
        ids = list(self.index.keys())
        return bool(ids) and self.index[ids[0]].get("model_version") == CIPHERTEXT_VERSION

    # ------------------------------------------------------------- index --
    def _load_index(self) -> Dict[str, Dict[str, Any]]:
        if not self.index_file.exists():
            return {}
        with open(self.index_file) as f:
            return json.load(f)

    def _save_index(self) -> None:
        tmp = self.index_file.with_suffix(".json.tmp")
        with open(tmp, "w") as f:
            json.dump(self.index, f, indent=2)
        os.replace(tmp, self.index_file)


_MISSING = object()
