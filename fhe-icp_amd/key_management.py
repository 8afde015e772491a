"""FHE key manager with the reference's directory layout (mirror of key_management.py).

Same class, methods, files and errors as the reference's ``FHEKeyManager``
(key_management.py:23-282):

    <key_dir>/.master              {"salt", "test", "created"} (JSON); the
                                   master key is PBKDF2-HMAC-SHA256 of the
                                   password (100 000 iterations, :49-58)
    <key_dir>/key_metadata.json    {"keys": {id: {...}}, "current": id}
    <key_dir>/<id>/compiled_model.enc   Fernet token of a pickled dict

What the reference stores in ``compiled_model.enc`` is only the model's
configuration (:150-157): its compiled circuit cannot be pickled, so every
process retrains and recompiles (batch_operations.py:78-108) and results
change run to run. Here the same dict also carries, under ``"fheicp"``, the
frozen quantisation parameters, the parameter set and the SECRET keys
(SURVEY.md §8f-2); the public evaluation keys (bootstrapping and key-switching
keys, ~190 MB) go next to it in ``eval_keys.npz``, unencrypted: they are
encryptions under the secret key and reveal nothing without it.
``load_compiled`` returns a ready FHESimilarityModel; BatchProcessor uses it
instead of retraining.

Fernet/PBKDF2 come from fheicp.fernet (the ``cryptography`` package is not in
this image); tokens are interchangeable with ``cryptography.fernet``. The
password is taken from ``password=`` or ``$FHE_MASTER_PASSWORD`` before
falling back to the reference's getpass prompts.
"""
from __future__ import annotations

import base64
import io
import json
import logging
import os
import pickle
import secrets
from datetime import datetime, timedelta
from pathlib import Path
from typing import Dict, Optional

import numpy as np

from fheicp.fernet import Fernet, InvalidToken, derive_master_key

logger = logging.getLogger(__name__)

FORMAT = "fheicp-keys"
VERSION = 1


class _DataUnpickler(pickle.Unpickler):
    """Only plain data (dict, list, str, numbers, bytes): what either side writes."""

    def find_class(self, module, name):
        raise pickle.UnpicklingError(f"refusing to load {module}.{name} from a key file")


def _loads(data: bytes):
    return _DataUnpickler(io.BytesIO(data)).load()


class FHEKeyManager:
    """Manage FHE keys with encryption and rotation (key_management.py:23)."""

    def __init__(self, key_dir: str = "~/.fhe_keys", password: Optional[str] = None):
        self.key_dir = Path(key_dir).expanduser()
        self.key_dir.mkdir(parents=True, exist_ok=True)
        self.metadata_file = self.key_dir / "key_metadata.json"
        self.current_key_id = None
        self._master_key = None
        self._password = password if password is not None else os.environ.get("FHE_MASTER_PASSWORD")
        self.expected_sizes = {"compiled_model": "secret keys + parameters: <1 MB; eval_keys.npz ~190 MB",
                               "metadata": "<1 KB"}
        logger.info("Key manager initialized. Key directory: %s", self.key_dir)

    # ------------------------------------------------------------ master --
    def _derive_master_key(self, password: str, salt: bytes) -> bytes:
        return derive_master_key(password, salt)

    def _ask(self, prompt: str) -> str:
        if self._password is not None:
            return self._password
        import getpass
        return getpass.getpass(prompt)

    def _get_master_key(self) -> bytes:
        if self._master_key is not None:
            return self._master_key
        master_key_file = self.key_dir / ".master"
        if master_key_file.exists():
            password = self._ask("Enter master password: ")
            data = json.loads(master_key_file.read_bytes())
            salt = base64.b64decode(data["salt"])
            key = self._derive_master_key(password, salt)
            try:
                Fernet(key).decrypt(base64.b64decode(data["test"]))
            except InvalidToken:
                raise ValueError("Invalid master password")
            self._master_key = key
        else:
            print("Creating new master key...")
            password = self._ask("Create master password: ")
            confirm = self._ask("Confirm master password: ")
            if password != confirm:
                raise ValueError("Passwords don't match")
            salt = secrets.token_bytes(16)
            self._master_key = self._derive_master_key(password, salt)
            test = Fernet(self._master_key).encrypt(b"test")
            master_key_file.write_bytes(json.dumps({
                "salt": base64.b64encode(salt).decode(),
                "test": base64.b64encode(test).decode(),
                "created": datetime.now().isoformat(),
            }).encode())
            os.chmod(master_key_file, 0o600)
        return self._master_key

    # -------------------------------------------------------------- keys --
    def generate_keys(self, key_id: Optional[str] = None, input_dim: Optional[int] = None,
                      n_bits: Optional[int] = None, device: int = 0, seed: Optional[int] = None,
                      key_seed: Optional[int] = None, fhe: Optional[str] = None) -> Dict[str, str]:
        """Train + compile the similarity model (GPU keygen) and store it
        (key_management.py:112-191; the reference fixes input_dim=128, n_bits=8;
        here $FHE_ICP_DIM / $FHE_ICP_N_BITS when not given, as for
        BatchConfig). With fhe != "execute" ($FHE_ICP_FHE; the reference's
        compare/search predict in the clear) only the quantized model is
        stored: no keys are generated and no GPU is needed."""
        from fhe_similarity import FHESimilarityModel
        if key_id is None:
            key_id = f"fhe_key_{datetime.now().strftime('%Y%m%d_%H%M%S')}"
        input_dim = int(input_dim if input_dim is not None else os.environ.get("FHE_ICP_DIM", "128"))
        n_bits = int(n_bits if n_bits is not None else os.environ.get("FHE_ICP_N_BITS", "8"))
        fhe = fhe if fhe is not None else os.environ.get("FHE_ICP_FHE", "execute")
        logger.info("Generating new FHE keys with ID: %s", key_id)
        model = FHESimilarityModel(input_dim=input_dim, n_bits=n_bits, device=device, seed=seed)
        X_train, _ = model.train()
        info = {"input_dim": model.input_dim, "n_bits": model.n_bits, "similarity_type": model.similarity_type,
                "metrics": model.metrics}
        if fhe != "execute":
            from fheicp.params import params_for_bits
            qp = model.model.quant_params
            return self.store_keys(key_id, qp, params_for_bits(qp.msg_bits()), None, info)
        model.compile(X_train[:10], key_seed=key_seed)
        fm = model.model._fitted()
        return self.store_keys(key_id, fm.qparams, fm.scheme, fm.engine.export_keys(), info)

    def store_keys(self, key_id: str, qparams, scheme, keys: Optional[dict], info: dict) -> Dict[str, str]:
        """Write <key_id>/compiled_model.enc (Fernet) + eval_keys.npz and make
        it current; keys=None stores the quantized model alone (clear mode)."""
        key_path = self.key_dir / key_id
        key_path.mkdir(exist_ok=True)
        f = Fernet(self._get_master_key())
        model_data = dict(info)
        model_data["compiled"] = keys is not None
        model_data["fheicp"] = {"format": FORMAT, "version": VERSION, "quant": qparams.to_dict(),
                                "scheme": scheme.as_dict()}
        if keys is not None:
            model_data["fheicp"]["s_small"] = np.ascontiguousarray(keys["s_small"], dtype=np.uint64).tobytes()
            model_data["fheicp"]["s_big"] = np.ascontiguousarray(keys["s_big"], dtype=np.uint64).tobytes()
        encrypted_model = f.encrypt(pickle.dumps(model_data))
        model_file = key_path / "compiled_model.enc"
        model_file.write_bytes(encrypted_model)
        os.chmod(model_file, 0o600)
        eval_file = key_path / "eval_keys.npz"
        if keys is not None:
            tmp = str(eval_file) + ".tmp.npz"
            np.savez(tmp, bsk=np.ascontiguousarray(keys["bsk"], dtype=np.uint64),
                     ksk=np.ascontiguousarray(keys["ksk"], dtype=np.uint64))
            os.replace(tmp, eval_file)
        metadata = self._load_metadata()
        created = datetime.now().isoformat()
        metadata["keys"][key_id] = {"created": created, "path": str(key_path), "active": True,
                                    "model_file": str(model_file), "size_bytes": len(encrypted_model),
                                    "eval_keys_file": str(eval_file) if keys is not None else None}
        metadata["current"] = key_id
        self.current_key_id = key_id
        self._save_metadata(metadata)
        return {"key_id": key_id, "model_file": str(model_file), "created": created}

    def list_keys(self) -> Dict[str, Dict]:
        return self._load_metadata().get("keys", {})

    def get_current_key(self) -> Optional[str]:
        return self._load_metadata().get("current")

    def _key_info(self, key_id: Optional[str]):
        if key_id is None:
            key_id = self.get_current_key()
            if key_id is None:
                raise ValueError("No current key set. Generate keys first.")
        metadata = self._load_metadata()
        if key_id not in metadata.get("keys", {}):
            raise ValueError(f"Key {key_id} not found")
        return key_id, metadata["keys"][key_id]

    def load_model(self, key_id: Optional[str] = None) -> dict:
        """The decrypted model dict (key_management.py:203-241); reads files
        written by the reference too (plain-data pickles only)."""
        key_id, info = self._key_info(key_id)
        model_file = Path(info["model_file"])
        if not model_file.exists():
            raise FileNotFoundError(f"Model file not found: {model_file}")
        data = _loads(Fernet(self._get_master_key()).decrypt(model_file.read_bytes()))
        logger.info("Loaded model configuration from key: %s", key_id)
        return data

    def load_key_material(self, key_id: Optional[str] = None):
        """-> (QuantParams, SchemeParams, keys dict or None) of an fheicp key
        (None: a clear-mode key, the quantized model without keys)."""
        from fheicp.model import QuantParams
        from fheicp.params import SchemeParams
        key_id, info = self._key_info(key_id)
        data = self.load_model(key_id)
        fh = data.get("fheicp")
        if not fh or fh.get("format") != FORMAT:
            raise ValueError(f"Key {key_id} holds no fheicp key material (written by the reference?)")
        if int(fh.get("version", 0)) > VERSION:
            raise ValueError(f"Key {key_id}: format version {fh['version']} is newer than supported {VERSION}")
        if "s_small" not in fh or not info.get("eval_keys_file"):
            return QuantParams.from_dict(fh["quant"]), SchemeParams(**fh["scheme"]), None
        with np.load(info["eval_keys_file"], allow_pickle=False) as z:
            keys = {"bsk": z["bsk"].copy(), "ksk": z["ksk"].copy()}
        keys["s_small"] = np.frombuffer(fh["s_small"], dtype=np.uint64).copy()
        keys["s_big"] = np.frombuffer(fh["s_big"], dtype=np.uint64).copy()
        return QuantParams.from_dict(fh["quant"]), SchemeParams(**fh["scheme"]), keys

    def load_compiled(self, key_id: Optional[str] = None, device: int = 0):
        """A compiled FHESimilarityModel with the stored parameters and keys."""
        from fhe_similarity import FHESimilarityModel
        from fheicp.sklearn import LinearRegression
        data = self.load_model(key_id)
        qp, _, keys = self.load_key_material(key_id)
        if keys is None:
            raise ValueError("this key holds the quantized model only (generated with fhe != 'execute')")
        m = FHESimilarityModel(input_dim=len(qp.coef), n_bits=qp.n_bits,
                               similarity_type=data.get("similarity_type", "cosine"), device=device)
        m.metrics = dict(data.get("metrics", {}))
        m.model = LinearRegression.from_quant_params(qp, device=device)
        m.compile(None, keys=keys)
        return m

    def rotate_keys(self, grace_period_days: int = 7, **generate_kwargs) -> Dict[str, str]:
        metadata = self._load_metadata()
        old_key_id = metadata.get("current") if metadata.get("current") in metadata.get("keys", {}) else None
        new_key_info = self.generate_keys(**generate_kwargs)
        metadata = self._load_metadata()
        if old_key_id is not None:
            metadata["keys"][old_key_id]["rotated_at"] = datetime.now().isoformat()
            metadata["keys"][old_key_id]["grace_until"] = (
                datetime.now() + timedelta(days=grace_period_days)).isoformat()
        self._save_metadata(metadata)
        print(f"Key rotation complete. Grace period: {grace_period_days} days")
        return new_key_info

    # ----------------------------------------------------------- metadata --
    def _load_metadata(self) -> Dict:
        if self.metadata_file.exists():
            with open(self.metadata_file) as f:
                return json.load(f)
        return {"keys": {}}

    def _save_metadata(self, metadata: Dict):
        with open(self.metadata_file, "w") as f:
            json.dump(metadata, f, indent=2)
        os.chmod(self.metadata_file, 0o600)
