"""Reference-side ctypes binding of libfheicp.so (no torch, numpy only).

This is the file a maintainer of the reference would add next to
fhe_similarity.py to call the MI355X engine through its C ABI
(include/fhe_icp.h) directly; INTEGRATION.md shows where it plugs in. It is
kept here, runnable, so tests/test_gpu_dropin.py can prove that the binding
works as written.

    eng = GpuCompare(params_dict, lib_path=".../libfheicp.so")
    acc, below = eng.compare(q_x, q_w, cst, T)   # int64 numpy arrays

Keys come from 32 bytes of os.urandom (fhe_keygen_key) and every session
encrypts under its own 32-byte stream key with a random 64-bit id start
(fhe_compare_batch_key / fhe_score_batch_key). key_seed / enc_seed select the
64-bit seed forms, for reproducible tests only.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

FIELDS = ("n", "k", "N", "pbs_base_log", "pbs_level", "ks_base_log", "ks_level",
          "lwe_noise_bits", "glwe_noise_bits", "msg_bits", "sign_digit_bits",
          "pbs_fast_base_log", "pbs_fast_level", "pbs_fast2_base_log", "pbs_fast2_level",
          "pbs_fast_group", "pbs_fast2_group", "pbs_mid_base_log", "pbs_mid_level", "pbs_mid2_base_log",
          "pbs_mid2_level", "pbs_mid_group", "pbs_mid2_group", "pbs_mid0_base_log", "pbs_mid0_level",
          "pbs_mid0_group")


class fhe_params(C.Structure):
    # struct_size (= sizeof(fhe_params), checked by the library) leads
    _fields_ = [("struct_size", C.c_int32)] + [(f, C.c_int32) for f in FIELDS]


_vp, _i32, _i64, _u64 = C.c_void_p, C.c_int32, C.c_int64, C.c_uint64
_PROTOS = {
    "fhe_ctx_create": (C.c_int, [C.POINTER(fhe_params), C.c_int, C.POINTER(_vp)]),
    "fhe_ctx_destroy": (None, [_vp]),
    "fhe_last_error": (C.c_char_p, [_vp]),
    "fhe_keygen": (C.c_int, [_vp, _u64, _vp]),
    "fhe_keygen_key": (C.c_int, [_vp, _vp, _vp]),
    "fhe_dev_alloc": (C.c_int, [_vp, C.c_size_t, C.POINTER(_vp)]),
    "fhe_dev_free": (C.c_int, [_vp, _vp]),
    "fhe_memcpy_h2d": (C.c_int, [_vp, _vp, _vp, C.c_size_t, _vp]),
    "fhe_memcpy_d2h": (C.c_int, [_vp, _vp, _vp, C.c_size_t, _vp]),
    "fhe_compare_batch": (C.c_int, [_vp, _vp, _i64, _i32, _vp, _i64, _i64, _u64, _u64, _vp, _vp, _vp]),
    "fhe_topk": (C.c_int, [_vp, _vp, _vp, _i64, _i64, _i32, _vp, _vp, _vp]),
    "fhe_score_batch": (C.c_int, [_vp, _vp, _i64, _i32, _vp, _i64, _i64, _u64, _u64, _vp, _vp]),
    "fhe_compare_batch_key": (C.c_int, [_vp, _vp, _i64, _i32, _vp, _i64, _i64, _vp, _u64, _vp, _vp, _vp]),
    "fhe_score_batch_key": (C.c_int, [_vp, _vp, _i64, _i32, _vp, _i64, _i64, _vp, _u64, _vp, _vp]),
}


def _key32() -> C.Array:
    """A 256-bit ChaCha20 key (8 u32 words) from the OS CSPRNG."""
    return (C.c_uint32 * 8).from_buffer_copy(os.urandom(32))


class GpuCompare:
    """One device context + keys; batched encrypted compares from numpy."""

    def __init__(self, params: dict, key_seed: int | None = None, device: int = 0, lib_path: str | None = None,
                 enc_seed: int | None = None):
        path = lib_path or os.environ.get("FHEICP_LIB", "libfheicp.so")
        self.L = L = C.CDLL(path)
        for name, (res, args) in _PROTOS.items():
            getattr(L, name).restype = res
            getattr(L, name).argtypes = args
        self.P = fhe_params(struct_size=C.sizeof(fhe_params), **{f: int(params.get(f, 0)) for f in FIELDS})
        self.ctx = _vp()
        self._ok(L.fhe_ctx_create(C.byref(self.P), device, C.byref(self.ctx)))
        if key_seed is None:
            self._ok(L.fhe_keygen_key(self.ctx, _key32(), None))
        else:
            self._ok(L.fhe_keygen(self.ctx, key_seed, None))  # 64-bit seed: tests only
        # the session's encryption stream: its own 256-bit key and a random id
        # start (enc_seed: the seeded test form, ids from 0)
        self.enc_seed = enc_seed
        self.enc_key = None if enc_seed is not None else _key32()
        self.next_id = 0 if enc_seed is not None else int.from_bytes(os.urandom(8), "little")

    def _take_ids(self, count: int) -> int:
        id0 = self.next_id
        self.next_id = (self.next_id + count) & 0xFFFFFFFFFFFFFFFF
        return id0

    def _ok(self, rc: int) -> None:
        if rc != 0:
            msg = self.L.fhe_last_error(self.ctx if self.ctx else None)
            raise RuntimeError(f"libfheicp error {rc}: {msg.decode() if msg else ''}")

    def _to_dev(self, a: np.ndarray) -> _vp:
        a = np.ascontiguousarray(a)
        d = _vp()
        self._ok(self.L.fhe_dev_alloc(self.ctx, a.nbytes, C.byref(d)))
        self._ok(self.L.fhe_memcpy_h2d(self.ctx, d, a.ctypes.data, a.nbytes, None))
        return d

    def _alloc(self, nbytes: int) -> _vp:
        d = _vp()
        self._ok(self.L.fhe_dev_alloc(self.ctx, nbytes, C.byref(d)))
        return d

    def _to_host(self, d: _vp, count: int) -> np.ndarray:
        out = np.empty(count, np.int64)
        self._ok(self.L.fhe_memcpy_d2h(self.ctx, out.ctypes.data, d, out.nbytes, None))
        return out

    def compare(self, q_x: np.ndarray, q_w: np.ndarray, cst: int, T: int):
        """Encrypted compare of B quantized feature rows: (acc int64[B], below int64[B])."""
        q_x = np.asarray(q_x, np.int64)
        B, D = q_x.shape
        bufs = [self._to_dev(q_x), self._to_dev(np.asarray(q_w, np.int64)), self._alloc(8 * B), self._alloc(8 * B)]
        try:
            id0 = self._take_ids(B * D)
            if self.enc_key is not None:
                rc = self.L.fhe_compare_batch_key(self.ctx, bufs[0], B, D, bufs[1], int(cst), int(T), self.enc_key,
                                                  id0, bufs[2], bufs[3], None)
            else:
                rc = self.L.fhe_compare_batch(self.ctx, bufs[0], B, D, bufs[1], int(cst), int(T), self.enc_seed,
                                              id0, bufs[2], bufs[3], None)
            self._ok(rc)
            return self._to_host(bufs[2], B), self._to_host(bufs[3], B)
        finally:
            for d in bufs:
                self.L.fhe_dev_free(self.ctx, d)

    def score(self, q_x: np.ndarray, q_w: np.ndarray, cst: int, centre: int):
        """The reference's own encrypted predict (fhe_similarity.py:151,
        predict(fhe="execute")): packed encryption + leveled dot + decryption,
        no bootstrap; the accumulators int64[B] (dequantize on the host).
        centre: the middle of the accumulator range, (lo + hi) // 2, so that
        acc - centre fits the msg_bits encoding."""
        q_x = np.asarray(q_x, np.int64)
        B, D = q_x.shape
        bufs = [self._to_dev(q_x), self._to_dev(np.asarray(q_w, np.int64)), self._alloc(8 * B)]
        try:
            id0 = self._take_ids(B * D)
            if self.enc_key is not None:
                rc = self.L.fhe_score_batch_key(self.ctx, bufs[0], B, D, bufs[1], int(cst), int(centre), self.enc_key,
                                                id0, bufs[2], None)
            else:
                rc = self.L.fhe_score_batch(self.ctx, bufs[0], B, D, bufs[1], int(cst), int(centre), self.enc_seed,
                                            id0, bufs[2], None)
            self._ok(rc)
            return self._to_host(bufs[2], B)
        finally:
            for d in bufs:
                self.L.fhe_dev_free(self.ctx, d)

    def close(self) -> None:
        if self.ctx:
            self.L.fhe_ctx_destroy(self.ctx)
            self.ctx = _vp()

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001
            pass
