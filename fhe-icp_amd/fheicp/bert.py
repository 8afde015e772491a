"""The embedding stage's BERT encoder on the GPU.

The reference runs ``transformers.AutoModel('bert-base-uncased')`` in torch
fp32 (bert_embeddings.py:45, :136) and pools ``last_hidden_state`` on the
host side of torch (:140-149). ``GpuBert`` takes the same model's weights (a
``transformers`` BertModel, or its state_dict + config) into libfheicp's
encoder (include/fhe_bert.h: MFMA GEMMs, fused attention, fp32 LayerNorm /
residual / pooling) and returns the pooled embeddings on the device.

``precision="f32"`` (default) is the reference's arithmetic: f32 operands on
the f32 MFMA, torch's fp32 forward in another summation order.
``precision="bf16"`` rounds the GEMM and attention operands to bf16 (about
3x faster, looser agreement). ``provenance`` names the arithmetic for the
stored-vector contract of batch_operations. There is no CPU
fallback here: without libfheicp or a GPU the constructor raises.
"""
from __future__ import annotations

import ctypes as C

import numpy as np
import torch

from . import _lib
from .engine import _ptr

POOLING = {"mean": 0, "cls": 1, "max": 2, "none": 3}
PRECISION = {"f32": 0, "bf16": 1}  # FHE_BERT_F32, FHE_BERT_BF16

# HF state_dict name -> (layer or -1, tensor id of fhe_bert_set_tensor)
_EMB = {"embeddings.word_embeddings.weight": 0, "embeddings.position_embeddings.weight": 1,
        "embeddings.token_type_embeddings.weight": 2, "embeddings.LayerNorm.weight": 3,
        "embeddings.LayerNorm.bias": 4}
_LAYER = {"attention.self.query.weight": 16, "attention.self.query.bias": 17,
          "attention.self.key.weight": 18, "attention.self.key.bias": 19,
          "attention.self.value.weight": 20, "attention.self.value.bias": 21,
          "attention.output.dense.weight": 22, "attention.output.dense.bias": 23,
          "attention.output.LayerNorm.weight": 24, "attention.output.LayerNorm.bias": 25,
          "intermediate.dense.weight": 26, "intermediate.dense.bias": 27,
          "output.dense.weight": 28, "output.dense.bias": 29,
          "output.LayerNorm.weight": 30, "output.LayerNorm.bias": 31}


class BertConfigC(C.Structure):
    _fields_ = [("vocab_size", C.c_int32), ("hidden_size", C.c_int32), ("num_layers", C.c_int32),
                ("num_heads", C.c_int32), ("intermediate_size", C.c_int32), ("max_position", C.c_int32),
                ("type_vocab_size", C.c_int32), ("layer_norm_eps", C.c_float)]


def _cfg_dict(config) -> dict:
    g = (lambda k: config[k]) if isinstance(config, dict) else (lambda k: getattr(config, k))
    act = g("hidden_act") if (isinstance(config, dict) and "hidden_act" in config) or hasattr(config, "hidden_act") \
        else "gelu"
    if act != "gelu":
        raise ValueError(f"hidden_act {act!r}: the encoder implements BERT's exact (erf) GELU only")
    return {"vocab_size": g("vocab_size"), "hidden_size": g("hidden_size"), "num_layers": g("num_hidden_layers"),
            "num_heads": g("num_attention_heads"), "intermediate_size": g("intermediate_size"),
            "max_position": g("max_position_embeddings"), "type_vocab_size": g("type_vocab_size"),
            "layer_norm_eps": g("layer_norm_eps")}


class GpuBert:
    """BERT forward + pooling on one MI355X through libfheicp (fhe_bert_*)."""

    def __init__(self, model=None, state_dict=None, config=None, device: int = 0, precision: str = "f32"):
        if precision not in PRECISION:
            raise ValueError(f"precision must be one of {tuple(PRECISION)}")
        if not torch.cuda.is_available():
            raise _lib.FheError("GpuBert needs a ROCm GPU (torch.cuda.is_available() is False)")
        if model is not None:
            config = model.config
            state_dict = model.state_dict()
        if state_dict is None or config is None:
            raise ValueError("pass a transformers BertModel, or state_dict= and config=")
        self.device = torch.device("cuda", device) if isinstance(device, int) else torch.device(device)
        self._L = _lib.lib()
        self.cfg = _cfg_dict(config)
        c = BertConfigC(**self.cfg)
        h = C.c_void_p()
        rc = self._L.fhe_bert_create(C.byref(c), self.device.index or 0, C.byref(h))
        if rc != 0:
            raise _lib.FheError(f"fhe_bert_create failed ({_lib.ERRORS.get(rc, rc)}): unsupported config {self.cfg}")
        self._h = h
        self._chk(self._L.fhe_bert_set_precision(self._h, PRECISION[precision]))
        self.precision = precision
        prefix = "bert." if any(k.startswith("bert.") for k in state_dict) else ""
        for name, t in state_dict.items():
            key = name[len(prefix):] if prefix and name.startswith(prefix) else name
            if key in _EMB:
                self._set(-1, _EMB[key], t)
            elif key.startswith("encoder.layer."):
                rest = key[len("encoder.layer."):]
                li, _, sub = rest.partition(".")
                if sub in _LAYER:
                    self._set(int(li), _LAYER[sub], t)
        if not self._L.fhe_bert_ready(self._h):
            raise ValueError("the state_dict lacks some encoder tensors")

    def _set(self, layer: int, which: int, t) -> None:
        a = np.ascontiguousarray(t.detach().cpu().numpy() if isinstance(t, torch.Tensor) else t, dtype=np.float32)
        self._chk(self._L.fhe_bert_set_tensor(self._h, layer, which, C.c_void_p(a.ctypes.data), a.size))

    def _chk(self, rc: int) -> None:
        if rc != 0:
            msg = self._L.fhe_bert_last_error(self._h)
            raise _lib.FheError(f"{_lib.ERRORS.get(rc, rc)}: {msg.decode() if msg else ''}")

    def close(self) -> None:
        if getattr(self, "_h", None):
            self._L.fhe_bert_destroy(self._h)
            self._h = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass

    @property
    def provenance(self) -> str:
        """The tag batch_operations stores with vectors this encoder embedded."""
        return f"hip-bert-{self.precision}"

    @property
    def hidden_size(self) -> int:
        return int(self.cfg["hidden_size"])

    def _dev_i32(self, a) -> torch.Tensor:
        t = a if isinstance(a, torch.Tensor) else torch.from_numpy(np.asarray(a))
        return t.to(self.device, dtype=torch.int32).contiguous()

    def forward(self, input_ids, attention_mask, token_type_ids=None, pooling: str = "mean") -> torch.Tensor:
        """[B][S] ids / mask (/ token types) -> float32 [B][hidden] pooled
        embeddings on the device ([B][S][hidden] last_hidden_state for
        pooling="none")."""
        if pooling not in POOLING:
            raise ValueError(f"Unknown pooling method: {pooling}")
        ids = self._dev_i32(input_ids)
        mask = self._dev_i32(attention_mask)
        if ids.dim() != 2 or mask.shape != ids.shape:
            raise ValueError("input_ids and attention_mask must both be [B, S]")
        B, S = ids.shape
        if S > self.cfg["max_position"]:
            raise ValueError(f"sequence length {S} exceeds max_position {self.cfg['max_position']}")
        if B and (int(ids.min()) < 0 or int(ids.max()) >= self.cfg["vocab_size"]):
            raise ValueError("token id out of the vocabulary")
        if B and int(mask[:, 0].min()) != 1:
            raise ValueError("every sequence needs its first token ([CLS]) unmasked")
        tt = self._dev_i32(token_type_ids) if token_type_ids is not None else None
        if tt is not None and B and (int(tt.min()) < 0 or int(tt.max()) >= self.cfg["type_vocab_size"]):
            raise ValueError("token type id out of range")
        H = self.hidden_size
        shape = (B, S, H) if pooling == "none" else (B, H)
        out = torch.empty(shape, dtype=torch.float32, device=self.device)
        with torch.cuda.device(self.device):
            st = C.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)
            self._chk(self._L.fhe_bert_forward(self._h, _ptr(ids), _ptr(tt), _ptr(mask), B, S, POOLING[pooling],
                                               _ptr(out), st))
        return out

    # --------------------------------------------------------- measurement --
    def profile(self, enable: bool) -> None:
        self._chk(self._L.fhe_bert_profile_enable(self._h, int(enable)))

    def profile_read(self, kernel: str) -> dict:
        ms, nl, fl = C.c_double(), C.c_int64(), C.c_double()
        self._chk(self._L.fhe_bert_profile_read(self._h, kernel.encode(), C.byref(ms), C.byref(nl), C.byref(fl)))
        return {"total_ms": ms.value, "launches": nl.value, "flops": fl.value}
