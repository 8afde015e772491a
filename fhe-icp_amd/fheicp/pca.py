"""The embedding stage's PCA on the GPU.

The reference reduces 768-dim BERT embeddings with a fitted sklearn PCA
(``DimensionReducer.transform``, dimension_reduction.py:67-72) before storing
them (batch_operations.py:166-178) and before every search query (:259-260).
``GpuPCA`` runs that transform with ``fhe_pca_transform``: the centred rows
times the components, accumulated in f64 and stored as float32. It keeps
``DimensionReducer``'s ``transform`` signature (numpy in, numpy out) and adds a
device form (torch in, torch out) that feeds ``fhe_quantize_pairs`` without a
host round trip.

Parity: the reference computes the same product in float32 BLAS, whose
summation order is unspecified, so the two agree to float32 rounding, not
bit for bit (tests/test_gpu_pca.py bounds the difference). BERT itself is not
reproducible offline (its weights are a network download): parity unpinned.
"""
from __future__ import annotations

import ctypes as C

import numpy as np
import torch

from . import _lib


class GpuPCA:
    def __init__(self, mean, components, device: int = 0):
        mean = np.ascontiguousarray(mean, dtype=np.float32).reshape(-1)
        comp = np.ascontiguousarray(components, dtype=np.float32)
        if comp.ndim != 2 or comp.shape[1] != mean.size:
            raise ValueError(f"components {comp.shape} do not match mean {mean.shape}")
        if mean.size > 1024:
            raise ValueError("at most 1024 input features")
        self.K, self.D = int(mean.size), int(comp.shape[0])
        self.device = torch.device("cuda", device) if isinstance(device, int) else torch.device(device)
        self._L = _lib.lib()
        P = _lib.params_struct({"n": 887, "k": 2, "N": 1024, "pbs_base_log": 15, "pbs_level": 2, "ks_base_log": 4,
                                "ks_level": 4, "lwe_noise_bits": 46, "glwe_noise_bits": 17, "msg_bits": 16})
        h = C.c_void_p()
        _lib.check(self._L.fhe_ctx_create(C.byref(P), self.device.index or 0, C.byref(h)))
        self._ctx = h
        self.mean = torch.from_numpy(mean).to(self.device)
        self.components = torch.from_numpy(comp).to(self.device)

    @classmethod
    def from_sklearn(cls, pca, device: int = 0) -> "GpuPCA":
        """From a fitted sklearn PCA (whiten=False)."""
        if getattr(pca, "whiten", False):
            raise ValueError("whitened PCA is not supported")
        return cls(pca.mean_, pca.components_, device)

    @classmethod
    def from_reducer(cls, reducer, device: int = 0) -> "GpuPCA":
        """From the reference's fitted DimensionReducer (method 'pca')."""
        if getattr(reducer, "method", "pca") != "pca" or not getattr(reducer, "is_fitted", True):
            raise ValueError("only a fitted 'pca' DimensionReducer maps to GpuPCA")
        return cls.from_sklearn(reducer.reducer, device)

    def transform_dev(self, X: torch.Tensor) -> torch.Tensor:
        """Device float32 [B, K] -> device float32 [B, D]."""
        X = X.to(self.device, dtype=torch.float32).contiguous()
        if X.ndim != 2 or X.shape[1] != self.K:
            raise ValueError(f"expected [B, {self.K}] rows, got {tuple(X.shape)}")
        B = X.shape[0]
        out = torch.empty((B, self.D), dtype=torch.float32, device=self.device)
        stream = torch.cuda.current_stream(self.device).cuda_stream
        _lib.check(self._L.fhe_pca_transform(self._ctx, C.c_void_p(X.data_ptr()), B, self.K,
                                             C.c_void_p(self.mean.data_ptr()), C.c_void_p(self.components.data_ptr()),
                                             self.D, C.c_void_p(out.data_ptr()), C.c_void_p(stream)), self._ctx)
        return out

    def transform(self, X) -> np.ndarray:
        """DimensionReducer.transform: numpy [B, K] (or [K]) -> numpy float32 [B, D]."""
        X = np.atleast_2d(np.asarray(X, dtype=np.float32))
        return self.transform_dev(torch.from_numpy(X)).cpu().numpy()

    def close(self) -> None:
        if getattr(self, "_ctx", None):
            self._L.fhe_ctx_destroy(self._ctx)
            self._ctx = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass
