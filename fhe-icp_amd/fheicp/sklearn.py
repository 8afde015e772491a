"""Concrete-ML-compatible estimator backed by the MI355X engine.

The reference holds a ``concrete.ml.sklearn.LinearRegression(n_bits)`` in
``FHESimilarityModel.model`` (fhe_similarity.py:88-90) and reaches it as:

    .fit(X, y)                      fhe_similarity.py:94
    .score(X, y)                    fhe_similarity.py:98
    .compile(X_sample)              fhe_similarity.py:120 (raises on failure)
    .fhe_circuit.graph.maximum_integer_bit_width()   fhe_similarity.py:129-130
    .predict(X, fhe="execute")      fhe_similarity.py:151
    .predict(X)                     fhe_similarity.py:167, batch_operations.py:233, :276
    .coef_ / .intercept_            fhe_similarity.py:191-192

This class keeps those names, argument meanings and return types. The
difference is where the work runs: predict(fhe="execute") encrypts, evaluates
and decrypts a whole batch on the GPU (libfheicp) instead of one row per call
on the CPU. fhe="disable" / "simulate" are the clear quantized inference,
which for this leveled circuit is what Concrete computes in both modes.
"""
from __future__ import annotations

import numpy as np

from .model import FheLinearModel, QuantParams, quantize_linear


class _Graph:
    def __init__(self, bits: int):
        self._bits = bits

    def maximum_integer_bit_width(self) -> int:
        return self._bits


class FheCircuit:
    """What compile() produces: parameters, keys on the device, the graph."""

    def __init__(self, model: FheLinearModel):
        self._model = model
        self.graph = _Graph(model.msg_bits)

    @property
    def parameters(self) -> dict:
        return self._model.scheme.as_dict()

    @property
    def pbs_per_prediction(self) -> int:
        """Key switches and bootstraps per encrypted prediction with a
        threshold (predict_threshold: the sign extraction's schedule,
        fhe_sign_pbs_count). predict(fhe="execute") itself runs none: it is
        the reference's leveled circuit."""
        from .params import sign_pbs_count
        return sign_pbs_count(self._model.scheme)


class LinearRegression:
    """Drop-in for concrete.ml.sklearn.LinearRegression (linear, leveled circuit)."""

    def __init__(self, n_bits=8, device: int = 0, key_seed: int | None = None):
        if isinstance(n_bits, dict):
            vals = set(n_bits.values())
            if len(vals) != 1:
                raise ValueError("per-operation n_bits must all be equal for this engine")
            n_bits = vals.pop()
        if not 2 <= int(n_bits) <= 16:
            raise ValueError(f"n_bits must be in [2, 16], got {n_bits}")
        self.n_bits = int(n_bits)
        self.device = device
        self.key_seed = key_seed
        self._model: FheLinearModel | None = None
        self.fhe_circuit: FheCircuit | None = None

    # ---------------------------------------------------------------- fit --
    def fit(self, X, y, *args, **kwargs):
        from sklearn.linear_model import LinearRegression as _OLS
        X = np.asarray(X)
        ols = _OLS().fit(X, np.asarray(y))
        coef = np.asarray(ols.coef_, dtype=np.float64).reshape(-1)
        intercept = float(np.asarray(ols.intercept_).reshape(-1)[0])
        self._model = FheLinearModel(quantize_linear(X, coef, intercept, self.n_bits))
        self.fhe_circuit = None
        return self

    @classmethod
    def from_quant_params(cls, qp: QuantParams, **kw) -> "LinearRegression":
        """Rebuild a fitted estimator from persisted quantisation parameters."""
        est = cls(n_bits=qp.n_bits, **kw)
        est._model = FheLinearModel(qp)
        return est

    def _fitted(self) -> FheLinearModel:
        if self._model is None:
            raise AttributeError("This LinearRegression instance is not fitted yet. Call 'fit' first.")
        return self._model

    @property
    def coef_(self) -> np.ndarray:
        return self._fitted().qparams.coef.copy()

    @property
    def intercept_(self) -> float:
        return self._fitted().qparams.intercept

    @property
    def quant_params(self) -> QuantParams:
        return self._fitted().qparams

    def score(self, X, y) -> float:
        """R^2 of the quantized predictions (sklearn's score on predict(X))."""
        y = np.asarray(y, dtype=np.float64).reshape(-1)
        pred = self.predict(X)
        ss_res = float(np.sum((y - pred) ** 2))
        ss_tot = float(np.sum((y - y.mean()) ** 2))
        return 1.0 - ss_res / ss_tot if ss_tot > 0 else 0.0

    # ------------------------------------------------------------ compile --
    def compile(self, X=None, *args, key_seed: int | None = None, keys: dict | None = None, **kwargs):
        """Create the GPU context and keys (Concrete: circuit + keygen).

        The encoding width comes from the worst case over every representable
        quantized input, so ``X`` (Concrete's inputset) only serves as a sanity
        check that it quantizes inside the calibrated range."""
        m = self._fitted()
        if X is not None:
            Xa = np.atleast_2d(np.asarray(X))
            if Xa.shape[1] != len(m.qparams.coef):
                raise ValueError(f"inputset has {Xa.shape[1]} features, model expects {len(m.qparams.coef)}")
        # no seed given: 256-bit keys from os.urandom (fhe_keygen_key); a seed
        # selects the reproducible 64-bit form (tests, benches)
        seed = key_seed if key_seed is not None else self.key_seed
        m.compile(key_seed=seed, device=self.device, keys=keys)
        self.fhe_circuit = FheCircuit(m)
        return self.fhe_circuit

    # ------------------------------------------------------------ predict --
    def predict(self, X, fhe: str = "disable") -> np.ndarray:
        m = self._fitted()
        X = np.atleast_2d(np.asarray(X))
        if fhe in ("disable", "simulate"):
            return m.predict_clear(X)
        if fhe == "execute":
            if not m.compiled:
                raise RuntimeError("The model is not compiled. Call compile() first.")
            scores, _ = m.predict_encrypted(X)
            return scores
        raise ValueError(f"fhe must be 'disable', 'simulate' or 'execute', got {fhe!r}")

    def predict_threshold(self, X, min_similarity: float):
        """Encrypted predict plus the encrypted decision ``score >= min_similarity``
        (batch_operations.py:278), decided by the bootstrapped sign bit.
        Returns (scores float64[B], keep bool[B])."""
        m = self._fitted()
        if not m.compiled:
            raise RuntimeError("The model is not compiled. Call compile() first.")
        scores, below = m.predict_encrypted(np.atleast_2d(np.asarray(X)), threshold=min_similarity)
        return scores, below == 0
