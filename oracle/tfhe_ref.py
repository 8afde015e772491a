"""ORACLE (test infrastructure only) — ctypes binding of oracle/build/libtfhe_ref.so.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use
this, and only as the checker. See oracle/tfhe_ref.c for what it restates.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
from pathlib import Path

import numpy as np

_HERE = Path(__file__).resolve().parent
_LIB_PATH = _HERE / "build" / "libtfhe_ref.so"

FIELDS = ("n", "k", "N", "pbs_base_log", "pbs_level", "ks_base_log", "ks_level",
          "lwe_noise_bits", "glwe_noise_bits", "msg_bits", "sign_digit_bits",
          "pbs_fast_base_log", "pbs_fast_level", "pbs_fast2_base_log", "pbs_fast2_level",
          "pbs_fast_group", "pbs_fast2_group", "pbs_mid_base_log", "pbs_mid_level", "pbs_mid2_base_log",
          "pbs_mid2_level", "pbs_mid_group", "pbs_mid2_group", "pbs_mid0_base_log", "pbs_mid0_level",
          "pbs_mid0_group")
OPTIONAL = FIELDS[FIELDS.index("sign_digit_bits"):]
# gadget g = 1..5 (fast, fast2, mid, mid2, mid0) and the level field that enables it
GADGET_LEVEL = {1: "pbs_fast_level", 2: "pbs_fast2_level", 3: "pbs_mid_level", 4: "pbs_mid2_level",
                5: "pbs_mid0_level"}


class RefParams(C.Structure):
    _fields_ = [(f, C.c_int32) for f in FIELDS]


def build() -> Path:
    """Compile the oracle with make (gcc). Output only under oracle/build/."""
    subprocess.run(["make", "-s", "-C", str(_HERE)], check=True)
    return _LIB_PATH


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not _LIB_PATH.exists():
            build()
        L = C.CDLL(str(_LIB_PATH))
        P = C.POINTER(RefParams)
        u64p = C.POINTER(C.c_uint64)
        i64p = C.POINTER(C.c_int64)
        u32p = C.POINTER(C.c_uint32)
        L.ref_bsk_words.argtypes = [P]; L.ref_bsk_words.restype = C.c_size_t
        L.ref_ksk_words.argtypes = [P]; L.ref_ksk_words.restype = C.c_size_t
        L.ref_keygen.argtypes = [P, C.c_uint64, u64p, u64p, u64p, u64p]
        L.ref_encrypt_raw.argtypes = [P, u64p, u64p, C.c_int64, C.c_uint64, C.c_uint64, u64p]
        L.ref_encrypt_ints.argtypes = [P, u64p, i64p, C.c_int64, C.c_uint64, C.c_uint64, u64p]
        L.ref_phase.argtypes = [u64p, u64p, C.c_int, C.c_int64, u64p]
        L.ref_decrypt_ints.argtypes = [P, u64p, u64p, C.c_int64, i64p]
        L.ref_decrypt_bits.argtypes = [P, u64p, u64p, C.c_int64, i64p]
        L.ref_linear.argtypes = [P, u64p, C.c_int64, C.c_int32, i64p, C.c_int64, u64p]
        L.ref_keyswitch.argtypes = [P, u64p, u64p, C.c_int64, u64p]
        L.ref_modswitch.argtypes = [P, u64p, C.c_int64, u32p]
        L.ref_pbs_const.argtypes = [P, u64p, u64p, C.c_int64, C.c_uint64, u64p]
        L.ref_pbs_gadget.argtypes = [P, u64p, u64p, C.c_int64, C.c_int, C.c_uint64, u64p]
        L.ref_bit_extract.argtypes = [P, u64p, u64p, u64p, C.c_int64, u64p, u64p]
        L.ref_pbs_lut.argtypes = [P, u64p, u64p, C.c_int64, C.c_uint64, C.c_uint64, C.c_int, u64p]
        L.ref_sign_extract.argtypes = [P, u64p, u64p, u64p, C.c_int64, u64p]
        L.ref_pbs_table.argtypes = [P, u64p, u64p, C.c_int64, i64p, C.c_int, u64p]
        L.ref_pbs_table_gadget.argtypes = [P, u64p, u64p, C.c_int64, C.c_int, i64p, C.c_int, u64p]
        L.ref_sign_extract3.argtypes = [P, u64p, u64p, u64p, u64p, u64p, C.c_int64, u64p]
        L.ref_sign_extract_keys.argtypes = [P, u64p, C.POINTER(u64p), u64p, u64p, C.c_int64, u64p]
        L.ref_sign_schedule.argtypes = [P, C.POINTER(C.c_int32), C.c_int32]; L.ref_sign_schedule.restype = C.c_int
        L.ref_sign_plan.argtypes = [P, C.POINTER(C.c_int32), C.POINTER(C.c_int32), C.POINTER(C.c_int32)]
        L.ref_sign_precise_rounds.argtypes = [P]; L.ref_sign_precise_rounds.restype = C.c_int
        L.ref_bsk2_words.argtypes = [P, C.c_int]; L.ref_bsk2_words.restype = C.c_size_t
        L.ref_keygen_fast_bsk.argtypes = [P, C.c_uint64, C.c_int, u64p, u64p, u64p]
        L.ref_sign_pbs_count.argtypes = [P]; L.ref_sign_pbs_count.restype = C.c_int
        L.ref_sign_digit_bits.argtypes = [P]; L.ref_sign_digit_bits.restype = C.c_int
        L.ref_negacyclic_mul.argtypes = [u64p, u64p, u64p, C.c_int]
        L.ref_decompose.argtypes = [C.c_uint64, C.c_int, C.c_int, i64p]
        L.ref_decompose_ks.argtypes = [C.c_uint64, C.c_int, C.c_int, i64p]
        L.ref_tuniform.argtypes = [C.c_uint64, C.c_int]; L.ref_tuniform.restype = C.c_int64
        L.ref_chacha20_block.argtypes = [u32p, C.c_uint32, u32p, u32p]
        L.ref_encrypt_seeded.argtypes = [P, u64p, i64p, C.c_int64, C.c_int32, u32p, u32p, u64p, u64p]
        L.ref_encrypt_packed.argtypes = [P, u64p, i64p, C.c_int64, C.c_int32, C.c_uint64, C.c_uint64, u64p]
        L.ref_linear_packed.argtypes = [P, u64p, C.c_int64, C.c_int32, i64p, C.c_int64, u64p]
        L.ref_expand_seeded.argtypes = [P, u64p, u64p, C.c_int64, C.c_int32, u32p, u64p]
        L.ref_key_from_seed.argtypes = [C.c_uint64, u32p]
        _lib = L
    return _lib


def _p(a: np.ndarray, ct):
    assert a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(C.POINTER(ct))


def u64(a):
    return _p(a, C.c_uint64)


def i64(a):
    return _p(a, C.c_int64)


class RefTFHE:
    """Exact CPU TFHE with the same parameters and PRNG streams as the GPU."""

    def __init__(self, params: dict, seed: int):
        self.params = {f: int(params.get(f, 0) if f in OPTIONAL else params[f]) for f in FIELDS}
        self.P = RefParams(**self.params)
        L = lib()
        self.n, self.k, self.N = self.params["n"], self.params["k"], self.params["N"]
        self.big = self.k * self.N
        self.s_small = np.zeros(self.n, np.uint64)
        self.s_big = np.zeros(self.big, np.uint64)
        self.bsk = np.zeros(L.ref_bsk_words(C.byref(self.P)), np.uint64)
        self.ksk = np.zeros(L.ref_ksk_words(C.byref(self.P)), np.uint64)
        L.ref_keygen(C.byref(self.P), C.c_uint64(seed), u64(self.s_small), u64(self.s_big), u64(self.bsk),
                     u64(self.ksk))
        # the other gadgets' bootstrapping keys (fhe_keygen generates them
        # too): keys[g] for g = 1..5 (fast, fast2, mid, mid2, mid0)
        self.keys = {}
        for which, lv in GADGET_LEVEL.items():
            if self.params[lv]:
                b = np.zeros(L.ref_bsk2_words(C.byref(self.P), which), np.uint64)
                L.ref_keygen_fast_bsk(C.byref(self.P), C.c_uint64(seed), which, u64(self.s_small), u64(self.s_big),
                                      u64(b))
                self.keys[which] = b
        self.bsk2, self.bsk3 = self.keys.get(1), self.keys.get(2)

    def with_msg_bits(self, P: int) -> "RefTFHE":
        self.params["msg_bits"] = int(P)
        self.P = RefParams(**self.params)
        return self

    def encrypt_ints(self, v, seed: int, id0: int = 0) -> np.ndarray:
        v = np.ascontiguousarray(v, dtype=np.int64).reshape(-1)
        ct = np.zeros((v.size, self.big + 1), np.uint64)
        lib().ref_encrypt_ints(C.byref(self.P), u64(self.s_big), i64(v), v.size, seed, id0, u64(ct))
        return ct

    def encrypt_raw(self, msg, seed: int, id0: int = 0) -> np.ndarray:
        msg = np.ascontiguousarray(msg, dtype=np.uint64).reshape(-1)
        ct = np.zeros((msg.size, self.big + 1), np.uint64)
        lib().ref_encrypt_raw(C.byref(self.P), u64(self.s_big), u64(msg), msg.size, seed, id0, u64(ct))
        return ct

    def encrypt_packed(self, v, seed: int, id0: int = 0) -> np.ndarray:
        """Packed GLWE encryption of B x D features: B x G x (k+1)N words."""
        v = np.ascontiguousarray(v, dtype=np.int64)
        B, D = v.shape
        N, k = self.params["N"], self.params["k"]
        G = -(-D // N)
        glwe = np.zeros((B, G, (k + 1) * N), np.uint64)
        lib().ref_encrypt_packed(C.byref(self.P), u64(self.s_big), i64(v), B, D, seed, id0, u64(glwe))
        return glwe

    def linear_packed(self, glwe: np.ndarray, D: int, w, cst: int) -> np.ndarray:
        """Leveled dot product of packed GLWEs (sample extraction at 0)."""
        glwe = np.ascontiguousarray(glwe, dtype=np.uint64)
        B = glwe.shape[0]
        w = np.ascontiguousarray(w, dtype=np.int64)
        out = np.zeros((B, self.big + 1), np.uint64)
        lib().ref_linear_packed(C.byref(self.P), u64(glwe), B, D, i64(w), cst, u64(out))
        return out

    def encrypt_seeded(self, v, mask_key, noise_key, id0) -> np.ndarray:
        """Seeded corpus encryption (bodies only), v: B x D ints, id0: B stream ids."""
        v = np.ascontiguousarray(v, dtype=np.int64)
        B, D = v.shape
        ids = np.ascontiguousarray(id0, dtype=np.uint64)
        mk = np.ascontiguousarray(mask_key, dtype=np.uint32)
        nk = np.ascontiguousarray(noise_key, dtype=np.uint32)
        body = np.zeros((B, D), np.uint64)
        lib().ref_encrypt_seeded(C.byref(self.P), u64(self.s_big), i64(v), B, D, _p(mk, C.c_uint32),
                                 _p(nk, C.c_uint32), u64(ids), u64(body))
        return body

    def expand_seeded(self, body, id0, mask_key) -> np.ndarray:
        body = np.ascontiguousarray(body, dtype=np.uint64)
        B, D = body.shape
        ids = np.ascontiguousarray(id0, dtype=np.uint64)
        mk = np.ascontiguousarray(mask_key, dtype=np.uint32)
        ct = np.zeros((B * D, self.big + 1), np.uint64)
        lib().ref_expand_seeded(C.byref(self.P), u64(body), u64(ids), B, D, _p(mk, C.c_uint32), u64(ct))
        return ct

    def phase(self, ct: np.ndarray, small: bool = False) -> np.ndarray:
        ct = np.ascontiguousarray(ct, dtype=np.uint64)
        s = self.s_small if small else self.s_big
        dim = s.size
        cnt = ct.size // (dim + 1)
        out = np.zeros(cnt, np.uint64)
        lib().ref_phase(u64(ct), u64(s), dim, cnt, u64(out))
        return out

    def decrypt_ints(self, ct: np.ndarray) -> np.ndarray:
        ct = np.ascontiguousarray(ct, dtype=np.uint64)
        cnt = ct.size // (self.big + 1)
        out = np.zeros(cnt, np.int64)
        lib().ref_decrypt_ints(C.byref(self.P), u64(self.s_big), u64(ct), cnt, i64(out))
        return out

    def decrypt_bits(self, ct: np.ndarray) -> np.ndarray:
        ct = np.ascontiguousarray(ct, dtype=np.uint64)
        cnt = ct.size // (self.big + 1)
        out = np.zeros(cnt, np.int64)
        lib().ref_decrypt_bits(C.byref(self.P), u64(self.s_big), u64(ct), cnt, i64(out))
        return out

    def linear(self, ct: np.ndarray, B: int, D: int, w, cst: int) -> np.ndarray:
        ct = np.ascontiguousarray(ct, dtype=np.uint64)
        w = np.ascontiguousarray(w, dtype=np.int64)
        out = np.zeros((B, self.big + 1), np.uint64)
        lib().ref_linear(C.byref(self.P), u64(ct), B, D, i64(w), cst, u64(out))
        return out

    def keyswitch(self, ct: np.ndarray) -> np.ndarray:
        ct = np.ascontiguousarray(ct, dtype=np.uint64)
        cnt = ct.size // (self.big + 1)
        out = np.zeros((cnt, self.n + 1), np.uint64)
        lib().ref_keyswitch(C.byref(self.P), u64(self.ksk), u64(ct), cnt, u64(out))
        return out

    def modswitch(self, small: np.ndarray) -> np.ndarray:
        small = np.ascontiguousarray(small, dtype=np.uint64)
        cnt = small.size // (self.n + 1)
        out = np.zeros((cnt, self.n + 1), np.uint32)
        lib().ref_modswitch(C.byref(self.P), u64(small), cnt, _p(out, C.c_uint32))
        return out

    def pbs_const(self, small: np.ndarray, tv: int) -> np.ndarray:
        small = np.ascontiguousarray(small, dtype=np.uint64)
        cnt = small.size // (self.n + 1)
        out = np.zeros((cnt, self.big + 1), np.uint64)
        lib().ref_pbs_const(C.byref(self.P), u64(self.bsk), u64(small), cnt, C.c_uint64(tv), u64(out))
        return out

    def pbs_gadget(self, small: np.ndarray, gadget: int, tv: int) -> np.ndarray:
        """pbs_const on gadget 0 (main), 1 (fast), 2 (fast2), 3 (mid), 4
        (mid2) or 5 (mid0), classic or multi-bit by that gadget's group
        (fhe_pbs_gadget_batch)."""
        small = np.ascontiguousarray(small, dtype=np.uint64)
        cnt = small.size // (self.n + 1)
        out = np.zeros((cnt, self.big + 1), np.uint64)
        key = self.bsk if gadget == 0 else self.keys[gadget]
        lib().ref_pbs_gadget(C.byref(self.P), u64(key), u64(small), cnt, int(gadget), C.c_uint64(tv), u64(out))
        return out

    def pbs_lut(self, small: np.ndarray, base: int, step: int, log_slots: int) -> np.ndarray:
        small = np.ascontiguousarray(small, dtype=np.uint64)
        cnt = small.size // (self.n + 1)
        out = np.zeros((cnt, self.big + 1), np.uint64)
        lib().ref_pbs_lut(C.byref(self.P), u64(self.bsk), u64(small), cnt, C.c_uint64(base), C.c_uint64(step),
                          int(log_slots), u64(out))
        return out

    def pbs_table(self, small: np.ndarray, lut, lut_bits: int, gadget: int = 0) -> np.ndarray:
        """fhe_pbs_table_gadget_batch restated (oracle/tfhe_ref.c
        ref_pbs_table / ref_pbs_table_gadget): gadget 0 the classic main
        gadget, else that gadget's key on its group's rotation."""
        small = np.ascontiguousarray(small, dtype=np.uint64)
        lut = np.ascontiguousarray(lut, dtype=np.int64)
        assert lut.size == 1 << lut_bits
        cnt = small.size // (self.n + 1)
        out = np.zeros((cnt, self.big + 1), np.uint64)
        if gadget == 0:
            lib().ref_pbs_table(C.byref(self.P), u64(self.bsk), u64(small), cnt, i64(lut), int(lut_bits), u64(out))
        else:
            lib().ref_pbs_table_gadget(C.byref(self.P), u64(self.keys[gadget]), u64(small), cnt, int(gadget), i64(lut),
                                       int(lut_bits), u64(out))
        return out

    def threshold(self, ct_acc: np.ndarray, T: int) -> np.ndarray:
        """fhe_threshold_batch restated: the sign extraction of acc - T
        (trivially subtracted), then 1 - sign: [acc >= T] at 2^63."""
        cv = np.array(ct_acc, dtype=np.uint64, copy=True, order="C").reshape(-1, self.big + 1)
        cv[:, -1] -= np.uint64((int(T) << (64 - self.params["msg_bits"])) % (1 << 64))
        bit = (np.uint64(0) - self.sign_extract(cv)).astype(np.uint64)
        bit[:, -1] += np.uint64(1 << 63)
        return bit

    def sign_extract(self, ct_v: np.ndarray) -> np.ndarray:
        """fhe_sign_batch restated: encryption of [v < 0] at 2^63 (ct_v copied)."""
        cv = np.array(ct_v, dtype=np.uint64, copy=True, order="C")
        cnt = cv.size // (self.big + 1)
        sign = np.zeros((cnt, self.big + 1), np.uint64)
        keys = (C.POINTER(C.c_uint64) * 5)(*[u64(self.keys[g]) if g in self.keys else None for g in range(1, 6)])
        lib().ref_sign_extract_keys(C.byref(self.P), u64(self.bsk), keys, u64(self.ksk), u64(cv), cnt, u64(sign))
        return sign

    def bit_extract(self, ct_v: np.ndarray):
        cv = np.array(ct_v, dtype=np.uint64, copy=True, order="C")
        cnt = cv.size // (self.big + 1)
        ref = np.zeros((cnt, self.big + 1), np.uint64)
        sign = np.zeros((cnt, self.big + 1), np.uint64)
        lib().ref_bit_extract(C.byref(self.P), u64(self.bsk), u64(self.ksk), u64(cv), cnt, u64(ref), u64(sign))
        return ref, sign


def negacyclic_mul(a, b) -> np.ndarray:
    a = np.ascontiguousarray(a, dtype=np.uint64)
    b = np.ascontiguousarray(b, dtype=np.uint64)
    c = np.zeros_like(a)
    lib().ref_negacyclic_mul(u64(a), u64(b), u64(c), a.size)
    return c


def decompose(x: int, base_log: int, levels: int) -> np.ndarray:
    d = np.zeros(levels, np.int64)
    lib().ref_decompose(C.c_uint64(x), base_log, levels, i64(d))
    return d


def decompose_ks(x: int, base_log: int, levels: int) -> np.ndarray:
    """The key switch's zero-mean digits (tfhe_ref.c decompose_ks)."""
    d = np.zeros(levels, np.int64)
    lib().ref_decompose_ks(C.c_uint64(x), base_log, levels, i64(d))
    return d


def tuniform(w: int, b: int) -> int:
    return int(lib().ref_tuniform(C.c_uint64(w), b))


def chacha20_block(key_words, counter: int, nonce_words) -> np.ndarray:
    k = np.ascontiguousarray(key_words, dtype=np.uint32)
    n = np.ascontiguousarray(nonce_words, dtype=np.uint32)
    out = np.zeros(16, np.uint32)
    lib().ref_chacha20_block(_p(k, C.c_uint32), counter, _p(n, C.c_uint32), _p(out, C.c_uint32))
    return out


def key_from_seed(seed: int) -> np.ndarray:
    out = np.zeros(8, np.uint32)
    lib().ref_key_from_seed(C.c_uint64(seed), _p(out, C.c_uint32))
    return out


def _ref_params(params: dict) -> RefParams:
    return RefParams(**{f: int(params.get(f, 0) if f in OPTIONAL else params[f]) for f in FIELDS})


def sign_digit_bits(params: dict) -> int:
    return int(lib().ref_sign_digit_bits(C.byref(_ref_params(params))))


def sign_pbs_count(params: dict) -> int:
    return int(lib().ref_sign_pbs_count(C.byref(_ref_params(params))))


def sign_precise_rounds(params: dict) -> int:
    return int(lib().ref_sign_precise_rounds(C.byref(_ref_params(params))))


def sign_plan(params: dict):
    d, j1, j2 = C.c_int32(), C.c_int32(), C.c_int32()
    lib().ref_sign_plan(C.byref(_ref_params(params)), C.byref(d), C.byref(j1), C.byref(j2))
    return d.value, j1.value, j2.value


def sign_schedule(params: dict) -> list:
    """The gadget (0 main, 1 fast, 2 fast2, 3 mid, 4 mid2, 5 mid0) of every bootstrap
    of the sign extraction (ref_sign_schedule)."""
    out = (C.c_int32 * 64)()
    R = lib().ref_sign_schedule(C.byref(_ref_params(params)), out, 64)
    return [int(out[r]) for r in range(R)]
