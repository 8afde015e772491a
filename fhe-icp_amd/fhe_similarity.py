"""FHESimilarityModel over the MI355X engine (mirror of the reference module).

Same class, constructor, methods, metrics keys and errors as the reference's
``fhe_similarity.FHESimilarityModel`` (fhe_similarity.py:12-223); the
estimator in ``self.model`` is ``fheicp.sklearn.LinearRegression``, the
drop-in for ``concrete.ml.sklearn.LinearRegression`` (:5, :88-90).

Behavioural differences, all on the execution side:
  * predict_encrypted runs the whole batch through the GPU in one fused
    encrypt -> linear -> decrypt launch sequence instead of one
    ``predict(X[i:i+1], fhe="execute")`` per row (:147-158);
  * training data comes from a seeded generator (``seed``; the reference
    draws from the unseeded global numpy RNG, :43-52);
  * save() also writes the frozen quantisation parameters, so load() returns
    a trained model instead of forcing a retrain (:215-220); save_compiled()
    / load_compiled() additionally persist the keys (fheicp.persist).
"""
from __future__ import annotations

import os
import pickle
import time
from typing import Optional, Tuple

import numpy as np

from fheicp import datagen, persist
from fheicp.model import QuantParams
from fheicp.sklearn import LinearRegression

SIMILARITY_TYPES = ("cosine", "dot", "manhattan")


def _rss_mb() -> float:
    try:
        import psutil
        return psutil.Process(os.getpid()).memory_info().rss / 2 ** 20
    except Exception:  # noqa: BLE001 - metrics only
        return 0.0


class FHESimilarityModel:
    def __init__(self, input_dim: int = 256, n_bits: int = 8, similarity_type: str = "cosine",
                 device: int = 0, seed: Optional[int] = None):
        self.input_dim = input_dim
        self.n_bits = n_bits
        self.similarity_type = similarity_type
        self.device = device
        self.seed = seed
        self.model: Optional[LinearRegression] = None
        self.compiled = False
        self.metrics: dict = {}

    # ---------------------------------------------------------- training --
    def _prepare_training_data(self, n_samples: int = 1000) -> Tuple[np.ndarray, np.ndarray]:
        """Pairs as fhe_similarity.py:34-70 (X = e1 * e2, y = cosine / -L1)."""
        seed = self.seed if self.seed is not None else int(np.random.randint(0, 2 ** 31 - 1))
        return datagen.training_pairs(self.input_dim, n_samples, seed, self.similarity_type)

    def train(self, X_train: Optional[np.ndarray] = None, y_train: Optional[np.ndarray] = None,
              n_samples: int = 1000):
        if X_train is None or y_train is None:
            X_train, y_train = self._prepare_training_data(n_samples)
        self.model = LinearRegression(n_bits=self.n_bits, device=self.device)
        t0 = time.time()
        self.model.fit(X_train, y_train)
        self.metrics["train_time"] = time.time() - t0
        self.metrics["train_score"] = float(self.model.score(X_train, y_train))
        self.compiled = False
        return X_train, y_train

    # ---------------------------------------------------------- compiling --
    def compile(self, X_sample: np.ndarray, key_seed: Optional[int] = None, keys: Optional[dict] = None):
        if self.model is None:
            raise RuntimeError("Model not trained. Call train() first.")
        t0, m0 = time.time(), _rss_mb()
        circuit = self.model.compile(X_sample, key_seed=key_seed, keys=keys)
        self.compiled = True
        self.metrics["compile_time"] = time.time() - t0
        self.metrics["compile_memory_mb"] = _rss_mb() - m0
        self.metrics["circuit_max_bits"] = int(circuit.graph.maximum_integer_bit_width())
        return circuit

    # --------------------------------------------------------- prediction --
    def predict_encrypted(self, X: np.ndarray) -> np.ndarray:
        if not self.compiled:
            raise RuntimeError("Model not compiled. Call compile() first.")
        X = np.atleast_2d(np.asarray(X))
        t0 = time.time()
        out = self.model.predict(X, fhe="execute")
        dt = time.time() - t0
        self.metrics["fhe_prediction_time"] = dt / max(len(X), 1)
        self.metrics["fhe_batch_time"] = dt
        return out

    def predict_clear(self, X: np.ndarray) -> np.ndarray:
        if self.model is None:
            raise RuntimeError("Model not trained.")
        return self.model.predict(X)

    _get_memory_usage = staticmethod(_rss_mb)

    # -------------------------------------------------------- persistence --
    def save(self, path: str):
        """Pickle of the reference's dict layout (:184-195) plus 'quant_params'."""
        data = {
            "input_dim": self.input_dim,
            "n_bits": self.n_bits,
            "similarity_type": self.similarity_type,
            "metrics": self.metrics,
            "model_params": {
                "coef_": self.model.coef_ if self.model is not None else None,
                "intercept_": self.model.intercept_ if self.model is not None else None,
            },
            "quant_params": self.model.quant_params.to_dict() if self.model is not None else None,
        }
        with open(path, "wb") as f:
            pickle.dump(data, f)

    @classmethod
    def load(cls, path: str, device: int = 0) -> "FHESimilarityModel":
        """Load a file written by save() (or by the reference, which has no
        quant_params: the model then needs training, as there)."""
        with open(path, "rb") as f:
            data = pickle.load(f)  # a file this API wrote; never load untrusted paths
        m = cls(input_dim=data["input_dim"], n_bits=data["n_bits"], similarity_type=data["similarity_type"],
                device=device)
        m.metrics = data.get("metrics", {})
        qd = data.get("quant_params")
        if qd is not None:
            m.model = LinearRegression.from_quant_params(QuantParams.from_dict(qd), device=device)
        return m

    def save_compiled(self, path: str, password: Optional[str] = None):
        """Quantisation parameters AND keys -> npz (mode 0600); the secret keys
        are Fernet-wrapped under password= or $FHE_MASTER_PASSWORD (fheicp.persist)."""
        if not self.compiled:
            raise RuntimeError("Model not compiled. Call compile() first.")
        fm = self.model._fitted()
        persist.save_model(path, fm.qparams, fm.scheme, fm.engine.export_keys(), password=password)

    @classmethod
    def load_compiled(cls, path: str, similarity_type: str = "cosine", device: int = 0,
                      password: Optional[str] = None) -> "FHESimilarityModel":
        qp, _, keys = persist.load_model(path, password=password)
        m = cls(input_dim=len(qp.coef), n_bits=qp.n_bits, similarity_type=similarity_type, device=device)
        m.model = LinearRegression.from_quant_params(qp, device=device)
        if keys is not None:
            m.compile(None, keys=keys)
        return m
