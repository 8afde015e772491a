"""Device-side engine: one libfheicp context per GPU, torch tensors as buffers.

PyTorch is plumbing here (device allocation, streams, host<->device copies);
all arithmetic runs in the HIP kernels of libfheicp.so. Ciphertext words are
stored in int64 tensors (bit patterns of the u64 words).
"""
from __future__ import annotations

import ctypes as C

import numpy as np
import torch

from . import _lib
from .params import SchemeParams


def _ptr(t: torch.Tensor | None):
    if t is None:
        return None
    assert t.is_contiguous(), "buffers must be contiguous"
    return C.c_void_p(t.data_ptr())


def _stream(device: torch.device):
    return C.c_void_p(torch.cuda.current_stream(device).cuda_stream)


class Engine:
    """A TFHE context on one MI355X (gfx950) device."""

    def __init__(self, params: SchemeParams, device: int | str | torch.device = 0):
        if not torch.cuda.is_available():
            raise _lib.FheError("fheicp.Engine needs a ROCm GPU (torch.cuda.is_available() is False)")
        self.device = torch.device("cuda", device) if isinstance(device, int) else torch.device(device)
        if self.device.index is None:
            self.device = torch.device("cuda", torch.cuda.current_device())
        self.params = params
        self._L = _lib.lib()
        self._P = _lib.params_struct(params.as_dict())
        h = C.c_void_p()
        _lib.check(self._L.fhe_ctx_create(C.byref(self._P), self.device.index, C.byref(h)))
        self._ctx = h
        self.big = params.k * params.N
        self.W = self.big + 1
        self.Ws = params.n + 1
        self.has_keys = False

    def close(self) -> None:
        if getattr(self, "_ctx", None):
            self._L.fhe_ctx_destroy(self._ctx)
            self._ctx = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass

    def _chk(self, rc: int) -> None:
        _lib.check(rc, self._ctx)

    def set_msg_bits(self, P: int) -> None:
        self._chk(self._L.fhe_set_msg_bits(self._ctx, int(P)))
        self.params = self.params.with_msg_bits(P)

    @property
    def msg_bits(self) -> int:
        return self.params.msg_bits

    # ---------------------------------------------------------------- keys --
    def keygen(self, seed: int | None = None, key=None) -> None:
        """Generate the keys from a 256-bit ChaCha20 key (8 u32 words or 32
        bytes; fhe_keygen_key), or from a 64-bit seed (fhe_keygen: 64 bits of
        entropy, reproducible tests and benches only). Exactly one is given."""
        if (seed is None) == (key is None):
            raise ValueError("keygen takes either a 64-bit seed or a 256-bit key")
        with torch.cuda.device(self.device):
            if key is not None:
                self._chk(self._L.fhe_keygen_key(self._ctx, self._key(key), _stream(self.device)))
            else:
                self._chk(self._L.fhe_keygen(self._ctx, C.c_uint64(seed), _stream(self.device)))
        self.has_keys = True

    def export_keys(self) -> dict:
        p = self.params
        out = {
            "s_small": np.zeros(p.n, np.uint64),
            "s_big": np.zeros(self.big, np.uint64),
            "bsk": np.zeros(self._L.fhe_bsk_words(C.byref(self._P)), np.uint64),
            "ksk": np.zeros(self._L.fhe_ksk_words(C.byref(self._P)), np.uint64),
        }
        self._chk(self._L.fhe_export_keys(self._ctx, *(C.c_void_p(out[k].ctypes.data)
                                                       for k in ("s_small", "s_big", "bsk", "ksk"))))
        return out

    def export_fast_bsk(self, which: int = 1) -> np.ndarray:
        """Another gadget's bootstrapping key (which = 1: params.pbs_fast_*,
        2: pbs_fast2_*, 3: pbs_mid_*, 4: pbs_mid2_*, 5: pbs_mid0_*)."""
        from .params import gadget_level
        p = self.params
        if which not in (1, 2, 3, 4, 5) or not gadget_level(p, which):
            raise ValueError(f"these parameters have no fast gadget {which}")
        q = _lib.params_struct(p.as_dict())
        out = np.zeros(self._L.fhe_fast_bsk_words(C.byref(q), which), np.uint64)
        self._chk(self._L.fhe_export_fast_bsk(self._ctx, which, C.c_void_p(out.ctypes.data)))
        return out

    def import_keys(self, keys: dict) -> None:
        arrs = [np.ascontiguousarray(keys[k], dtype=np.uint64) for k in ("s_small", "s_big", "bsk", "ksk")]
        self._chk(self._L.fhe_import_keys(self._ctx, *(C.c_void_p(a.ctypes.data) for a in arrs)))
        self.has_keys = True

    # ------------------------------------------------------------- buffers --
    def empty_big(self, count: int) -> torch.Tensor:
        return torch.empty((count, self.W), dtype=torch.int64, device=self.device)

    def empty_small(self, count: int) -> torch.Tensor:
        return torch.empty((count, self.Ws), dtype=torch.int64, device=self.device)

    def to_dev(self, a, dtype=torch.int64) -> torch.Tensor:
        if isinstance(a, torch.Tensor):
            return a.to(self.device, dtype=dtype).contiguous()
        a = np.ascontiguousarray(a)
        if a.dtype == np.uint64:
            a = a.view(np.int64)
        return torch.from_numpy(a).to(self.device, dtype=dtype).contiguous()

    # ------------------------------------------------------ client / server --
    def encrypt(self, msg, seed: int, id0: int = 0) -> torch.Tensor:
        m = self.to_dev(msg).reshape(-1)
        ct = self.empty_big(m.numel())
        self._chk(self._L.fhe_encrypt_batch(self._ctx, _ptr(m), m.numel(), C.c_uint64(seed), C.c_uint64(id0),
                                            _ptr(ct), _stream(self.device)))
        return ct

    def decrypt(self, ct: torch.Tensor) -> torch.Tensor:
        n = ct.numel() // self.W
        out = torch.empty(n, dtype=torch.int64, device=self.device)
        self._chk(self._L.fhe_decrypt_batch(self._ctx, _ptr(ct), n, _ptr(out), _stream(self.device)))
        return out

    def decrypt_bits(self, ct: torch.Tensor) -> torch.Tensor:
        n = ct.numel() // self.W
        out = torch.empty(n, dtype=torch.int64, device=self.device)
        self._chk(self._L.fhe_decrypt_bits_batch(self._ctx, _ptr(ct), n, _ptr(out), _stream(self.device)))
        return out

    def phase(self, ct: torch.Tensor) -> torch.Tensor:
        n = ct.numel() // self.W
        out = torch.empty(n, dtype=torch.int64, device=self.device)
        self._chk(self._L.fhe_phase_batch(self._ctx, _ptr(ct), n, _ptr(out), _stream(self.device)))
        return out

    def linear(self, ct: torch.Tensor, B: int, D: int, w, cst: int) -> torch.Tensor:
        wd = self.to_dev(w)
        out = self.empty_big(B)
        self._chk(self._L.fhe_linear_batch(self._ctx, _ptr(ct), B, D, _ptr(wd), int(cst), _ptr(out),
                                           _stream(self.device)))
        return out

    def encrypt_linear(self, msg, w, cst: int, seed, id0: int = 0) -> torch.Tensor:
        """Fused encrypt + linear (fhe_encrypt_linear_batch[_key]): msg B x D
        ints; `seed` is an int seed (tests) or a 256-bit stream key."""
        m = self.to_dev(msg)
        B, D = m.shape
        wd = self.to_dev(w)
        out = self.empty_big(B)
        if isinstance(seed, (int, np.integer)):
            rc = self._L.fhe_encrypt_linear_batch(self._ctx, _ptr(m), B, D, C.c_uint64(int(seed)), C.c_uint64(id0),
                                                  _ptr(wd), int(cst), _ptr(out), _stream(self.device))
        else:
            rc = self._L.fhe_encrypt_linear_batch_key(self._ctx, _ptr(m), B, D, self._key(seed), C.c_uint64(id0),
                                                      _ptr(wd), int(cst), _ptr(out), _stream(self.device))
        self._chk(rc)
        return out

    def encrypt_packed(self, msg, seed: int, id0: int = 0) -> torch.Tensor:
        """Packed GLWE encryption of B x D features (fhe_encrypt_packed_batch):
        [B][ceil(D / N)][(k + 1) N] words."""
        m = self.to_dev(msg)
        B, D = m.shape
        p = self.params
        G = -(-D // p.N)
        out = torch.empty((B, G, (p.k + 1) * p.N), dtype=torch.int64, device=self.device)
        self._chk(self._L.fhe_encrypt_packed_batch(self._ctx, _ptr(m), B, D, C.c_uint64(seed), C.c_uint64(id0),
                                                   _ptr(out), _stream(self.device)))
        return out

    def linear_packed(self, glwe: torch.Tensor, D: int, w, cst: int) -> torch.Tensor:
        """Leveled dot product on packed GLWE inputs (fhe_linear_packed_batch)."""
        B = glwe.shape[0]
        wd = self.to_dev(w)
        out = self.empty_big(B)
        self._chk(self._L.fhe_linear_packed_batch(self._ctx, _ptr(glwe), B, D, _ptr(wd), int(cst), _ptr(out),
                                                  _stream(self.device)))
        return out

    def keyswitch(self, ct: torch.Tensor, shift: int = 0, add_body: int = 0) -> torch.Tensor:
        n = ct.numel() // self.W
        out = self.empty_small(n)
        self._chk(self._L.fhe_keyswitch_batch(self._ctx, _ptr(ct), n, shift, C.c_uint64(add_body), _ptr(out),
                                              _stream(self.device)))
        return out

    def pbs(self, small: torch.Tensor, tv: int) -> torch.Tensor:
        n = small.numel() // self.Ws
        out = self.empty_big(n)
        self._chk(self._L.fhe_pbs_batch(self._ctx, _ptr(small), n, C.c_uint64(tv), _ptr(out), _stream(self.device)))
        return out

    def pbs_gadget(self, small: torch.Tensor, gadget: int, tv: int) -> torch.Tensor:
        """fhe_pbs_batch on gadget 0 (main), 1 (fast) or 2 (fast2) (fhe_pbs_gadget_batch)."""
        n = small.numel() // self.Ws
        out = self.empty_big(n)
        self._chk(self._L.fhe_pbs_gadget_batch(self._ctx, _ptr(small), n, int(gadget), C.c_uint64(tv), _ptr(out),
                                               _stream(self.device)))
        return out

    def pbs_lut(self, small: torch.Tensor, base: int, step: int, log_slots: int) -> torch.Tensor:
        """Staircase bootstrap (fhe_pbs_lut_batch)."""
        n = small.numel() // self.Ws
        out = self.empty_big(n)
        self._chk(self._L.fhe_pbs_lut_batch(self._ctx, _ptr(small), n, C.c_uint64(base), C.c_uint64(step),
                                            int(log_slots), _ptr(out), _stream(self.device)))
        return out

    def pbs_table(self, small: torch.Tensor, lut, lut_bits: int, gadget: int | None = None) -> torch.Tensor:
        """Table bootstrap (fhe_pbs_table_batch; fhe_pbs_table_gadget_batch
        with an explicit gadget): input m in [0, 2^lut_bits) at
        2^(63 - lut_bits); output lut[m] at 2^(64 - msg_bits)."""
        n = small.numel() // self.Ws
        lut_d = self.to_dev(np.asarray(lut, dtype=np.int64)) if not isinstance(lut, torch.Tensor) else lut
        out = self.empty_big(n)
        if gadget is None:
            rc = self._L.fhe_pbs_table_batch(self._ctx, _ptr(small), n, _ptr(lut_d), int(lut_bits), _ptr(out),
                                             _stream(self.device))
        else:
            rc = self._L.fhe_pbs_table_gadget_batch(self._ctx, _ptr(small), n, int(gadget), _ptr(lut_d),
                                                    int(lut_bits), _ptr(out), _stream(self.device))
        self._chk(rc)
        return out

    def table_gadget(self) -> int:
        """The gadget fhe_pbs_table_batch runs on (fhe_pbs_table_gadget)."""
        return self._L.fhe_pbs_table_gadget(C.byref(self._P_now()))

    def threshold(self, ct_acc: torch.Tensor, T: int) -> torch.Tensor:
        """Encryption of [acc >= T] at 2^63 (fhe_threshold_batch); ct_acc is kept."""
        n = ct_acc.numel() // self.W
        bit = self.empty_big(n)
        self._chk(self._L.fhe_threshold_batch(self._ctx, _ptr(ct_acc), n, int(T), _ptr(bit), _stream(self.device)))
        return bit

    def sign(self, ct_v: torch.Tensor) -> torch.Tensor:
        """Consumes ct_v; returns the encryption of [v < 0] at 2^63 (fhe_sign_batch)."""
        n = ct_v.numel() // self.W
        sign = self.empty_big(n)
        self._chk(self._L.fhe_sign_batch(self._ctx, _ptr(ct_v), n, _ptr(sign), _stream(self.device)))
        return sign

    def sign_trace(self, ct_v: torch.Tensor, sched=None, rounds: int = 0, phases: bool = True):
        """Measurement only (fhe_sign_trace_batch): consumes ct_v and runs the
        sign extraction's rounds (all, or the first `rounds`) on an explicit
        gadget schedule (None: the plan's). Returns (sign ciphertexts or None,
        phases uint32 tensor [R][count] of every round's rotation exponent or
        None)."""
        n = ct_v.numel() // self.W
        R = len(sched) if sched is not None else None
        if R is None:
            cap = (C.c_int32 * 64)()
            R = self._L.fhe_sign_schedule(C.byref(self._P_now()), cap, 64)
            if R < 0:
                _lib.check(R)
        last = rounds in (0, R)
        sign = self.empty_big(n) if last else None
        ph = torch.empty((R, n), dtype=torch.int32, device=self.device) if phases else None
        hs = (C.c_int32 * R)(*[int(g) for g in sched]) if sched is not None else None
        self._chk(self._L.fhe_sign_trace_batch(self._ctx, _ptr(ct_v), n, hs, int(rounds), _ptr(sign), _ptr(ph),
                                               _stream(self.device)))
        return sign, ph

    def _P_now(self):
        return _lib.params_struct(self.params.as_dict())

    def bit_extract(self, ct_v: torch.Tensor):
        """Consumes ct_v; returns (refreshed, sign) ciphertexts."""
        n = ct_v.numel() // self.W
        ref = self.empty_big(n)
        sign = self.empty_big(n)
        self._chk(self._L.fhe_bit_extract_batch(self._ctx, _ptr(ct_v), n, _ptr(ref), _ptr(sign),
                                                _stream(self.device)))
        return ref, sign

    def compare(self, q_x: torch.Tensor, w: torch.Tensor, cst: int, T: int, enc, id0: int = 0):
        """Fused encrypt -> linear -> decrypt + sign extraction for B pairs.
        `enc` is the session's 256-bit stream key (8 u32 words or 32 bytes:
        fhe_compare_batch_key) or an int seed (fhe_compare_batch, tests).

        Returns (acc int64[B], below int64[B])."""
        B, D = q_x.shape
        acc = torch.empty(B, dtype=torch.int64, device=self.device)
        below = torch.empty(B, dtype=torch.int64, device=self.device)
        if isinstance(enc, (int, np.integer)):
            rc = self._L.fhe_compare_batch(self._ctx, _ptr(q_x), B, D, _ptr(w), int(cst), int(T), C.c_uint64(int(enc)),
                                           C.c_uint64(id0), _ptr(acc), _ptr(below), _stream(self.device))
        else:
            rc = self._L.fhe_compare_batch_key(self._ctx, _ptr(q_x), B, D, _ptr(w), int(cst), int(T), self._key(enc),
                                               C.c_uint64(id0), _ptr(acc), _ptr(below), _stream(self.device))
        self._chk(rc)
        return acc, below

    def score(self, q_x: torch.Tensor, w: torch.Tensor, cst: int, T: int, enc, id0: int = 0):
        """The leveled circuit alone (fhe_score_batch[_key]): encrypt -> linear
        -> decrypt, no key switch or bootstrap. T centres acc in the encoding;
        `enc` as in compare(). Returns acc int64[B]."""
        B, D = q_x.shape
        acc = torch.empty(B, dtype=torch.int64, device=self.device)
        if isinstance(enc, (int, np.integer)):
            rc = self._L.fhe_score_batch(self._ctx, _ptr(q_x), B, D, _ptr(w), int(cst), int(T), C.c_uint64(int(enc)),
                                         C.c_uint64(id0), _ptr(acc), _stream(self.device))
        else:
            rc = self._L.fhe_score_batch_key(self._ctx, _ptr(q_x), B, D, _ptr(w), int(cst), int(T), self._key(enc),
                                             C.c_uint64(id0), _ptr(acc), _stream(self.device))
        self._chk(rc)
        return acc

    # ------------------------------------------- seeded (stored) corpus --
    @staticmethod
    def key_from_seed(seed: int) -> np.ndarray:
        out = np.zeros(8, np.uint32)
        _lib.lib().fhe_key_from_seed(C.c_uint64(seed), C.c_void_p(out.ctypes.data))
        return out

    @staticmethod
    def _key(k) -> C.Array:
        if isinstance(k, (bytes, bytearray)):
            if len(k) != 32:
                raise ValueError("a ChaCha20 key is 32 bytes")
            k = np.frombuffer(bytes(k), dtype="<u4")
        k = np.ascontiguousarray(k, dtype=np.uint32).reshape(8)
        return (C.c_uint32 * 8)(*[int(x) for x in k])

    def quantize(self, x: torch.Tensor, scale: float, zero_point: int, qmin: int, qmax: int) -> torch.Tensor:
        """clip(rint(x / scale + zp), qmin, qmax) of a device f32/f64 [B, D] (fhe_quantize_pairs)."""
        B, D = x.shape
        q = torch.empty((B, D), dtype=torch.int64, device=self.device)
        self._chk(self._L.fhe_quantize_pairs(self._ctx, None, 0, _ptr(x), 1 if x.dtype == torch.float64 else 0, B, D,
                                             C.c_double(scale), int(zero_point), int(qmin), int(qmax), _ptr(q),
                                             _stream(self.device)))
        return q

    def encrypt_seeded(self, msg: torch.Tensor, mask_key, noise_key, id0: torch.Tensor) -> torch.Tensor:
        B, D = msg.shape
        body = torch.empty((B, D), dtype=torch.int64, device=self.device)
        self._chk(self._L.fhe_encrypt_seeded_batch(self._ctx, _ptr(msg), B, D, self._key(mask_key),
                                                   self._key(noise_key), _ptr(id0), _ptr(body), _stream(self.device)))
        return body

    def expand_seeded(self, body: torch.Tensor, id0: torch.Tensor, B: int, D: int, mask_key) -> torch.Tensor:
        ct = self.empty_big(B * D)
        self._chk(self._L.fhe_expand_seeded_batch(self._ctx, _ptr(body), _ptr(id0), B, D, self._key(mask_key),
                                                  _ptr(ct), _stream(self.device)))
        return ct

    def linear_seeded(self, body: torch.Tensor, id0: torch.Tensor, mask_key, w, cst: int) -> torch.Tensor:
        B, D = body.shape
        wd = self.to_dev(w)
        out = self.empty_big(B)
        self._chk(self._L.fhe_linear_seeded_batch(self._ctx, _ptr(body), _ptr(id0), B, D, self._key(mask_key),
                                                  _ptr(wd), int(cst), _ptr(out), _stream(self.device)))
        return out

    def compare_seeded(self, body: torch.Tensor, id0: torch.Tensor, mask_key, w: torch.Tensor, cst: int, T: int):
        """fhe_compare_seeded_batch: (acc int64[B], below int64[B])."""
        B, D = body.shape
        acc = torch.empty(B, dtype=torch.int64, device=self.device)
        below = torch.empty(B, dtype=torch.int64, device=self.device)
        self._chk(self._L.fhe_compare_seeded_batch(self._ctx, _ptr(body), _ptr(id0), B, D, self._key(mask_key),
                                                   _ptr(w), int(cst), int(T), _ptr(acc), _ptr(below),
                                                   _stream(self.device)))
        return acc, below

    def topk(self, acc: torch.Tensor, below: torch.Tensor | None, k: int, base_idx: int = 0):
        oa = torch.empty(k, dtype=torch.int64, device=self.device)
        oi = torch.empty(k, dtype=torch.int64, device=self.device)
        self._chk(self._L.fhe_topk(self._ctx, _ptr(acc), _ptr(below), acc.numel(), base_idx, k, _ptr(oa), _ptr(oi),
                                   _stream(self.device)))
        return oa, oi

    # --------------------------------------------------------- measurement --
    def profile(self, enable: bool) -> None:
        self._chk(self._L.fhe_profile_enable(self._ctx, int(enable)))

    def kernel_name(self, kernel: str) -> str:
        """The instantiation last launched for a profile bucket (fhe_profile_kernel_name)."""
        buf = C.create_string_buffer(256)
        self._chk(self._L.fhe_profile_kernel_name(self._ctx, kernel.encode(), buf, 256))
        return buf.value.decode()

    def profile_read(self, kernel: str) -> dict:
        ms = C.c_double()
        nl = C.c_int64()
        items = C.c_int64()
        self._chk(self._L.fhe_profile_read(self._ctx, kernel.encode(), C.byref(ms), C.byref(nl), C.byref(items)))
        return {"total_ms": ms.value, "launches": nl.value, "items": items.value}


def u64(t: torch.Tensor) -> np.ndarray:
    """Device int64 tensor -> host uint64 array (bit pattern)."""
    return t.detach().cpu().numpy().view(np.uint64)
