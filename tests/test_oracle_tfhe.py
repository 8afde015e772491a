"""CPU: the exact TFHE oracle — primitives against published vectors and
schoolbook math, the scheme end-to-end on the TOY set, and spec digests."""
import hashlib
import json
from pathlib import Path

import numpy as np
import pytest

from fheicp.params import TOY, params_for_bits

GOLD = json.loads((Path(__file__).parent / "golden" / "tfhe_golden.json").read_text())


def test_chacha20_rfc8439_block(oracle_lib):
    """RFC 8439 §2.3.2 test vector."""
    key = np.frombuffer(bytes(range(32)), dtype="<u4")
    nonce = np.frombuffer(bytes.fromhex("000000090000004a00000000"), dtype="<u4")
    out = oracle_lib.chacha20_block(key, 1, nonce)
    expect = [0xe4e7f110, 0x15593bd1, 0x1fdd0f50, 0xc47120a3, 0xc7f4d1c7, 0x0368c033, 0x9aaa2204, 0x4e6cd4c3,
              0x466482d2, 0x09aa9f07, 0x05d7c214, 0xa2028bd9, 0xd19c12b5, 0xb94e16de, 0xe883d0cb, 0x4e3c50a2]
    assert out.tolist() == expect


def test_tuniform_support(oracle_lib):
    b = 5
    vals = [oracle_lib.tuniform(w, b) for w in range(1 << (b + 2))]
    assert min(vals) == -(1 << b) and max(vals) == (1 << b)
    counts = np.bincount(np.array(vals) + (1 << b))
    assert counts[0] == 1 and counts[-1] == 1 and set(counts[1:-1]) == {2}


@pytest.mark.parametrize("N", [16, 64, 256])
def test_negacyclic_karatsuba_vs_schoolbook(oracle_lib, N):
    rng = np.random.default_rng(N)
    a = rng.integers(0, 2 ** 63, N, dtype=np.uint64) * np.uint64(2) + np.uint64(1)
    b = rng.integers(0, 2 ** 63, N, dtype=np.uint64)
    c = oracle_lib.negacyclic_mul(a, b)
    ref = [0] * N
    for i in range(N):
        for j in range(N):
            p = int(a[i]) * int(b[j])
            if i + j < N:
                ref[i + j] += p
            else:
                ref[i + j - N] -= p
    assert c.tolist() == [x % 2 ** 64 for x in ref]


@pytest.mark.parametrize("beta,levels", [(15, 2), (12, 3), (7, 6), (4, 4)])
def test_gadget_decomposition(oracle_lib, beta, levels):
    rng = np.random.default_rng(beta)
    for x in list(rng.integers(0, 2 ** 64, 200, dtype=np.uint64)) + [0, 2 ** 64 - 1, 2 ** 63]:
        d = oracle_lib.decompose(int(x), beta, levels)
        assert np.all(d >= -(2 ** (beta - 1))) and np.all(d < 2 ** (beta - 1))
        rec = sum(int(d[l]) << (64 - (l + 1) * beta) for l in range(levels)) % 2 ** 64
        err = (int(x) - rec) % 2 ** 64
        err = err - 2 ** 64 if err >= 2 ** 63 else err
        assert abs(err) <= 2 ** (63 - levels * beta)


@pytest.fixture(scope="module")
def toy_ref(oracle_lib):
    return oracle_lib.RefTFHE(TOY.as_dict(), GOLD["key_seed"])


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def test_spec_digests(toy_ref):
    """Key streams and encryption streams are frozen by the spec."""
    assert sha(toy_ref.s_small) == GOLD["sha256_s_small"]
    assert sha(toy_ref.s_big) == GOLD["sha256_s_big"]
    assert sha(toy_ref.bsk) == GOLD["sha256_bsk"]
    assert sha(toy_ref.ksk) == GOLD["sha256_ksk"]
    ct = toy_ref.encrypt_ints(np.array(GOLD["messages"]), seed=GOLD["enc_seed"], id0=GOLD["id0"])
    assert sha(ct) == GOLD["sha256_ct"]


def test_encrypt_linear_decrypt(toy_ref):
    P = TOY.msg_bits
    rng = np.random.default_rng(1)
    x = rng.integers(-4, 4, (30, 8))
    w = rng.integers(-7, 8, 8)
    ct = toy_ref.encrypt_ints(x, seed=5)
    assert np.array_equal(toy_ref.decrypt_ints(ct), x.reshape(-1))
    lin = toy_ref.linear(ct, 30, 8, w, 3)
    half = 2 ** (P - 1)
    assert np.array_equal(toy_ref.decrypt_ints(lin), (x @ w + 3 + half) % (2 * half) - half)


def _ahat_linear(glwe, D, w, cst, N, k, P):
    """numpy restatement of the fused kernel's formulas (k_encrypt_linear /
    k_linear_packed): a_{i,u} = sum_t w_t Ahat_i[t - u], Ahat[m] = A[m] (m >= 0),
    -A[m + N] (m < 0); b = sum_t w_t B[t] + cst Delta; summed over chunks."""
    B, G, _ = glwe.shape
    out = np.zeros((B, k * N + 1), np.uint64)
    u = np.arange(N)
    with np.errstate(over="ignore"):
        for g in range(G):
            Dg = min(D - g * N, N)
            for t in range(Dg):
                wt = np.uint64(np.int64(w[g * N + t]) & np.int64(-1)) if w[g * N + t] >= 0 else \
                    np.uint64(2 ** 64 + int(w[g * N + t]))
                m = t - u
                for i in range(k):
                    A = glwe[:, g, i * N:(i + 1) * N]
                    ah = np.where(m >= 0, A[:, m % N], np.uint64(0) - A[:, (m + N) % N])
                    out[:, i * N:(i + 1) * N] += wt * ah
                out[:, k * N] += wt * glwe[:, g, k * N + t]
        out[:, k * N] += np.uint64((int(cst) << (64 - P)) % 2 ** 64)
    return out


@pytest.mark.parametrize("B,D", [(6, 8), (3, 300)])
def test_packed_encrypt_linear(toy_ref, B, D):
    """Packed features: the GLWE of a row decrypts
    coefficient-wise to its features (the noise within TUniform's bound), the
    textbook leveled product (GLWE x W, sample extraction) decrypts to
    x @ w + cst, and equals the fused kernel's formulas restated in numpy bit
    for bit, across a chunk boundary (D = 300 > N = 256: two GLWEs per row)."""
    P = TOY.msg_bits
    N, k = TOY.N, TOY.k
    rng = np.random.default_rng(3)
    x = rng.integers(-4, 4, (B, D))
    w = rng.integers(-7, 8, D)
    glwe = toy_ref.encrypt_packed(x, seed=9, id0=40)
    G = -(-D // N)
    assert glwe.shape == (B, G, (k + 1) * N)
    from oracle.tfhe_ref import negacyclic_mul
    S = toy_ref.s_big.astype(np.uint64)
    with np.errstate(over="ignore"):
        for b in range(B):
            for g in range(G):
                ph = glwe[b, g, k * N:].copy()
                for i in range(k):
                    ph -= negacyclic_mul(glwe[b, g, i * N:(i + 1) * N], S[i * N:(i + 1) * N])
                want = np.zeros(N, np.int64)
                seg = x[b, g * N:(g + 1) * N]
                want[:seg.size] = seg
                err = ph.view(np.int64) - (want << (64 - P))
                assert np.abs(err).max() <= 2 ** TOY.glwe_noise_bits
    lin = toy_ref.linear_packed(glwe, D, w, 3)
    half = 2 ** (P - 1)
    assert np.array_equal(toy_ref.decrypt_ints(lin), (x @ w + 3 + half) % (2 * half) - half)
    assert np.array_equal(lin, _ahat_linear(glwe, D, w, 3, N, k, P))


def test_keyswitch_noise(toy_ref):
    rng = np.random.default_rng(2)
    v = rng.integers(-100, 100, 40)
    ct = toy_ref.encrypt_ints(v, seed=6)
    sm = toy_ref.keyswitch(ct)
    ph = toy_ref.phase(sm, small=True).view(np.int64)
    err = ph - (v.astype(np.int64) << (64 - TOY.msg_bits))
    assert np.abs(err).max() < 2 ** 58     # TOY n=64: sigma_ks ~ 2^-8 of the torus


def test_pbs_sign_and_bit_extraction(toy_ref):
    P = TOY.msg_bits
    v = np.array([-(2 ** (P - 1)), -77, -1, 0, 1, 42, 2 ** (P - 1) - 1], dtype=np.int64)
    ct = toy_ref.encrypt_ints(v, seed=7)
    ref, sign = toy_ref.bit_extract(ct)
    assert np.array_equal(toy_ref.decrypt_ints(ref), v)
    assert np.array_equal(toy_ref.decrypt_bits(sign), (v < 0).astype(np.int64))
    # a single constant-TV bootstrap follows the phase half-torus
    big = np.array([-100, -50, 50, 100], dtype=np.int64)
    sm = toy_ref.keyswitch(toy_ref.encrypt_ints(big, seed=8))
    out = toy_ref.pbs_const(sm, 1 << 61)
    ph = toy_ref.phase(out).view(np.int64)
    assert np.array_equal(ph > 0, big >= 0)


def test_real_params_roundtrip(oracle_lib):
    p = params_for_bits(16)
    ref = oracle_lib.RefTFHE(p.as_dict(), 5)
    assert ref.bsk.size == p.n * 3 * p.pbs_level * 3 * p.N
    v = np.array([-32768, -1, 0, 12345, 32767], dtype=np.int64)
    ct = ref.encrypt_ints(v, seed=1)
    assert np.array_equal(ref.decrypt_ints(ct), v)
    sm = ref.keyswitch(ct)
    err = ref.phase(sm, small=True).view(np.int64) - (v << 48)
    assert np.abs(err).max() < 2 ** 58


@pytest.mark.parametrize("d", [3, 4])
@pytest.mark.parametrize("P", [2, 3, 4, 5, 6, 7, 8, 9])
def test_sign_extract_digits_all_values(toy_ref, P, d):
    """The d-bit digit sign algorithm (fhe_sign_batch) on every P-bit value,
    covering each branch shape: P < 4, full digits, a 3-bit leftover digit
    (d = 4, P = 7), leftover single bits, top chunk only (d = 4, P = 4)."""
    r = toy_ref.with_msg_bits(P)
    r.params["sign_digit_bits"] = d
    r.P = type(r.P)(**r.params)
    v = np.arange(-(2 ** (P - 1)), 2 ** (P - 1), dtype=np.int64)
    sign = r.sign_extract(r.encrypt_ints(v, seed=100 + P))
    assert np.array_equal(r.decrypt_bits(sign), (v < 0).astype(np.int64))


def test_sign_pbs_count(oracle_lib):
    from oracle.tfhe_ref import sign_pbs_count
    from fheicp.params import params_for_bits
    # 4-bit digits where the noise bar allows them (P <= 26 here, with a more
    # precise main gadget from P = 17), else 3-bit
    want = {1: 1, 2: 2, 3: 3, 4: 1, 6: 3, 7: 3, 8: 3, 9: 4, 16: 7, 17: 8, 21: 10, 26: 13, 27: 17}
    assert {P: sign_pbs_count(params_for_bits(P).as_dict()) for P in want} == want
    want3 = {4: 2, 6: 3, 7: 4, 8: 5, 9: 5, 16: 10, 21: 13, 26: 17}
    got3 = {P: sign_pbs_count({**params_for_bits(P).as_dict(), "sign_digit_bits": 3}) for P in want3}
    assert got3 == want3


def test_pbs_lut_staircase(toy_ref):
    """4-slot staircase bootstrap: phase D*2^61 + 2^60 -> D * step."""
    D = np.array([0, 1, 2, 3, 3, 2, 1, 0], dtype=np.uint64)
    msg = (D << np.uint64(61)) + np.uint64(1 << 60)
    sm = toy_ref.keyswitch(toy_ref.encrypt_raw(msg, seed=11))
    out = toy_ref.pbs_lut(sm, 0, 1 << 50, 2)
    err = toy_ref.phase(out).view(np.int64) - (D.astype(np.int64) << 50)
    assert np.abs(err).max() < 2 ** 45


TOY_FAST = {"pbs_base_log": 12, "pbs_level": 3, "pbs_fast_base_log": 8, "pbs_fast_level": 2}


@pytest.mark.parametrize("P,d", [(5, 4), (8, 3), (11, 4)])
def test_sign_extract_fast_gadget_values(oracle_lib, P, d):
    """Per-round gadgets: a toy set whose fast gadget (8, 2) is too coarse for
    the leading rounds, so sign_plan splits the rounds between the two keys
    (j main rounds, the rest on bsk2); every P-bit value (P <= 8; boundaries
    and a sample above) keeps its sign."""
    from dataclasses import replace
    from fheicp.params import TOY, sign_plan, sign_rounds
    prm = replace(TOY, msg_bits=P, sign_digit_bits=d, **TOY_FAST)
    dd, j, _ = sign_plan(prm)
    assert dd == d and (j < len(sign_rounds(P, d)) or P == 5)
    r = oracle_lib.RefTFHE(prm.as_dict(), 4321)
    assert r.bsk2 is not None and oracle_lib.sign_precise_rounds(prm.as_dict()) == j
    h = 2 ** (P - 1)
    v = np.arange(-h, h, dtype=np.int64)
    if P > 8:
        v = np.concatenate([[-h, -h + 1, -2, -1, 0, 1, h - 2, h - 1],
                            np.random.default_rng(P).integers(-h, h, 120)]).astype(np.int64)
    sign = r.sign_extract(r.encrypt_ints(v, seed=200 + P))
    assert np.array_equal(r.decrypt_bits(sign), (v < 0).astype(np.int64))


TOY_FAST3 = {"pbs_base_log": 12, "pbs_level": 3, "pbs_fast_base_log": 8, "pbs_fast_level": 2,
             "pbs_fast2_base_log": 11, "pbs_fast2_level": 1}


@pytest.mark.parametrize("P,d", [(8, 3), (11, 4)])
def test_sign_extract_three_gadgets(oracle_lib, P, d):
    """Three gadgets on a toy set whose fast (8,2) and fast2 (11,1) gadgets are
    coarse enough that the plan uses all three keys; the values keep their
    sign and the plan matches the library's."""
    from dataclasses import replace
    from fheicp.params import TOY, sign_plan, sign_rounds
    prm = replace(TOY, msg_bits=P, sign_digit_bits=d, **TOY_FAST3)
    dd, j1, j2 = sign_plan(prm)
    assert dd == d and 0 < j1 < j2 < len(sign_rounds(P, d)), (j1, j2)
    assert oracle_lib.sign_plan(prm.as_dict()) == (dd, j1, j2)
    r = oracle_lib.RefTFHE(prm.as_dict(), 4322)
    assert r.bsk2 is not None and r.bsk3 is not None
    h = 2 ** (P - 1)
    v = np.concatenate([[-h, -h + 1, -2, -1, 0, 1, h - 2, h - 1],
                        np.random.default_rng(P).integers(-h, h, 120)]).astype(np.int64)
    sign = r.sign_extract(r.encrypt_ints(v, seed=300 + P))
    assert np.array_equal(r.decrypt_bits(sign), (v < 0).astype(np.int64))


@pytest.mark.parametrize("P,d,mid2", [(11, 4, None), (11, 3, (9, 2))])
def test_sign_extract_mid_gadgets(oracle_lib, P, d, mid2):
    """Mid gadgets between the main and the fast one on a toy
    set whose schedule uses every key: main (12,3) -> mid (10,2) [-> mid2
    (9,2)] -> fast (8,2) -> fast2 (11,1). The values keep their sign, and the
    schedule matches the library's and params.py's."""
    import ctypes as C
    from dataclasses import replace
    from fheicp import _lib
    from fheicp.params import TOY, sign_schedule
    kw = dict(TOY_FAST3, pbs_mid_base_log=10, pbs_mid_level=2)
    if mid2:
        kw.update(pbs_mid2_base_log=mid2[0], pbs_mid2_level=mid2[1])
    prm = replace(TOY, msg_bits=P, sign_digit_bits=d, **kw)
    dd, sched = sign_schedule(prm)
    assert dd == d and set(sched) == ({0, 1, 2, 3, 4} if mid2 else {0, 1, 2, 3}), sched
    assert oracle_lib.sign_schedule(prm.as_dict()) == sched
    out = (C.c_int32 * 64)()
    R = _lib.lib().fhe_sign_schedule(C.byref(_lib.params_struct(prm.as_dict())), out, 64)
    assert list(out[:R]) == sched
    r = oracle_lib.RefTFHE(prm.as_dict(), 4323)
    assert sorted(r.keys) == ([1, 2, 3, 4] if mid2 else [1, 2, 3])
    h = 2 ** (P - 1)
    v = np.concatenate([[-h, -h + 1, -2, -1, 0, 1, h - 2, h - 1],
                        np.random.default_rng(P + d).integers(-h, h, 120)]).astype(np.int64)
    sign = r.sign_extract(r.encrypt_ints(v, seed=400 + P))
    assert np.array_equal(r.decrypt_bits(sign), (v < 0).astype(np.int64))
    # each mid key is its own stream: a mid-gadget bootstrap on it keeps signs
    small = r.keyswitch(r.encrypt_ints(np.array([-5, 7], np.int64) << (P - 4), seed=5))
    ph = r.phase(r.pbs_gadget(small, 3, 1 << 61)).view(np.int64)
    assert list(ph > 0) == [False, True]


def test_multibit_rotation_oracle(oracle_lib):
    """The multi-bit blind rotation (group 2) in the oracle:
    an odd n (the last pair has a phantom zero coefficient), the key holds
    three GGSWs per pair, and the bootstrap's output phase equals the classic
    rotation's to within noise: both rotate the test vector by the same
    sum_i a_i s_i."""
    from dataclasses import replace
    from fheicp.params import TOY
    prm = replace(TOY, n=63, msg_bits=6, pbs_fast_base_log=15, pbs_fast_level=2, pbs_fast_group=2)
    r = oracle_lib.RefTFHE(prm.as_dict(), 77)
    assert r.bsk2.size == 3 * 32 * 3 * 2 * 3 * 256
    v = np.arange(-32, 32, dtype=np.int64)
    small = r.keyswitch(r.encrypt_ints(v, seed=9))
    tv = 1 << 61
    mb = r.phase(r.pbs_gadget(small, 1, tv)).view(np.int64)
    cl = r.phase(r.pbs_gadget(small, 0, tv)).view(np.int64)   # classic on the main (15, 2) key
    assert np.abs(mb - cl).max() < 2 ** 50
    assert np.array_equal(mb > 0, cl > 0)


@pytest.mark.parametrize("P,d", [(6, 3), (8, 4)])
def test_sign_extract_multibit_gadgets(oracle_lib, P, d):
    """Sign extraction whose fast and fast2 gadgets run the multi-bit rotation
    (the real sets' plans, on the toy set): every P-bit value keeps its sign,
    with the plan the library resolves for these groups."""
    from dataclasses import replace
    from fheicp.params import TOY, sign_plan
    prm = replace(TOY, msg_bits=P, sign_digit_bits=d, pbs_base_log=12, pbs_level=3, pbs_fast_base_log=15,
                  pbs_fast_level=2, pbs_fast_group=2, pbs_fast2_base_log=23, pbs_fast2_level=1, pbs_fast2_group=2)
    assert oracle_lib.sign_plan(prm.as_dict()) == sign_plan(prm)
    assert sign_plan(prm)[2] < P   # rounds on the multi-bit fast2 gadget
    r = oracle_lib.RefTFHE(prm.as_dict(), 4323)
    h = 2 ** (P - 1)
    v = np.arange(-h, h, dtype=np.int64)
    sign = r.sign_extract(r.encrypt_ints(v, seed=400 + P))
    assert np.array_equal(r.decrypt_bits(sign), (v < 0).astype(np.int64))


@pytest.mark.parametrize("lut_bits", [1, 3, 4])
def test_oracle_pbs_table_every_value(oracle_lib, lut_bits):
    """ref_pbs_table (the restatement of fhe_pbs_table_batch) on the TOY set:
    an arbitrary signed table, every input message, the output decrypts to
    lut[m] at the context's msg_bits."""
    from dataclasses import replace
    P_out = 8
    prm = replace(TOY, msg_bits=lut_bits + 1)
    ref = oracle_lib.RefTFHE(prm.as_dict(), 99)
    M = 1 << lut_bits
    m = np.arange(M, dtype=np.int64)
    lut = np.random.default_rng(lut_bits).integers(-(2 ** (P_out - 1)), 2 ** (P_out - 1), M)
    small = ref.keyswitch(ref.encrypt_ints(m, seed=5))
    ref.with_msg_bits(P_out)
    out = ref.pbs_table(small, lut, lut_bits)
    assert np.array_equal(ref.decrypt_ints(out), lut)
    # the multi-bit table bootstrap (fhe_pbs_table_gadget_batch on a
    # multi-bit gadget): the same table through ref_pbs_table_gadget
    prm_mb = replace(prm, pbs_fast_base_log=15, pbs_fast_level=2, pbs_fast_group=2)
    ref_mb = oracle_lib.RefTFHE(prm_mb.as_dict(), 99)
    small = ref_mb.keyswitch(ref_mb.encrypt_ints(m, seed=6))
    ref_mb.with_msg_bits(P_out)
    out_mb = ref_mb.pbs_table(small, lut, lut_bits, gadget=1)
    assert np.array_equal(ref_mb.decrypt_ints(out_mb), lut)


def test_oracle_threshold_restatement(oracle_lib):
    """RefTFHE.threshold (fhe_threshold_batch): [acc >= T] for accumulators
    around T and at the ends of the P-bit range, on the TOY set."""
    P = TOY.msg_bits
    ref = oracle_lib.RefTFHE(TOY.as_dict(), 7)
    T = 5
    acc = np.array([-(2 ** (P - 2)), T - 2, T - 1, T, T + 1, 2 ** (P - 2)], dtype=np.int64)
    bit = ref.threshold(ref.encrypt_ints(acc, seed=3), T)
    assert np.array_equal(ref.decrypt_bits(bit), (acc >= T).astype(np.int64))


@pytest.mark.parametrize("beta,lvl", [(3, 5), (4, 4), (2, 8), (7, 4)])
def test_keyswitch_digits_zero_mean(oracle_lib, beta, lvl):
    """The key switch's digits (tfhe_ref.c decompose_ks, the same rule in
    k_ks_digits and k_keyswitch): they recompose the input rounded to
    lvl * beta bits modulo 2^64, lie in [-B/2, B/2], and are zero-mean with
    E[d^2] = (B^2 + 2) / 12, the noise model's factor (fheicp.params): the
    [-B/2, B/2) digits' mean of -1/2 would put a key-dependent bias
    0.5 * sum(KSK noise) on every key switch (measured 7% above the model's
    sigma on one (3, 5) key before this rule)."""
    from oracle.tfhe_ref import decompose_ks
    rng = np.random.default_rng(beta * 10 + lvl)
    xs = [int(x) for x in rng.integers(0, 2 ** 63, 20000, dtype=np.uint64) * 2 + rng.integers(0, 2, 20000)]
    prec = beta * lvl
    B = 1 << beta
    ds = np.array([decompose_ks(x, beta, lvl) for x in xs])
    assert ds.min() >= -B // 2 and ds.max() <= B // 2
    for x, d in zip(xs[:2000], ds[:2000]):
        want = (((x >> (63 - prec)) + 1) >> 1) << (64 - prec)
        got = sum(int(d[l]) << (64 - (l + 1) * beta) for l in range(lvl))
        assert got % 2 ** 64 == want % 2 ** 64
    assert abs(ds.mean()) < 0.02
    assert abs((ds.astype(float) ** 2).mean() / ((B * B + 2) / 12) - 1) < 0.02


def test_keyswitch_uses_the_rounded_key(toy_ref):
    """The key switch's definition (tfhe_ref.c keyswitch1, k_server.h
    ks_round): every KSK word rounded to the nearest multiple
    of 2^R, R = params.ks_round_bits (40 at lwe_noise_bits = 46: 3 byte planes
    on the matrix cores). Restated here in Python integers on 3 TOY
    ciphertexts, bit-exact; the exact key gives a different result that
    differs only far below the key-switch noise."""
    from fheicp.params import ks_round_bits
    from oracle.tfhe_ref import decompose_ks
    p = TOY
    R = ks_round_bits(p)
    assert R == 40 and ks_round_bits(params_for_bits(16)) == 40
    M = 2 ** 64
    rnd = lambda x: ((x + (1 << (R - 1))) >> R << R) % M
    big, n, KL = p.k * p.N, p.n, p.ks_level
    ksk = toy_ref.ksk.reshape(big, KL, n + 1)
    ct = toy_ref.encrypt_ints(np.array([-77, 0, 91], np.int64), seed=12)
    got = toy_ref.keyswitch(ct)
    for c in range(ct.shape[0]):
        out = [0] * n + [int(ct[c, big])]
        exact = list(out)
        for i in range(big):
            d = decompose_ks(int(ct[c, i]), p.ks_base_log, KL)
            for l in range(KL):
                if d[l]:
                    row = ksk[i, l]
                    for t in range(n + 1):
                        out[t] = (out[t] - int(d[l]) * rnd(int(row[t]))) % M
                        exact[t] = (exact[t] - int(d[l]) * int(row[t])) % M
        assert [int(x) for x in got[c]] == out
        assert exact != out
        diff = [((a - b + M // 2) % M) - M // 2 for a, b in zip(out, exact)]
        assert max(abs(x) for x in diff) < 2 ** (R + 10)


def test_oracle_sign_entry_points_under_sanitizers(tmp_path):
    """ref_sign_extract / ref_sign_extract3 pass short key arrays
    to ref_sign_extract_keys, which reads one slot per gadget (NGAD - 1). The
    oracle source and oracle/asan_driver.c are compiled together under
    -fsanitize=address,undefined (gcc, no OpenMP) and both entry points run on
    the TOY set: exact sign bits and no sanitizer report."""
    import shutil
    import subprocess
    from pathlib import Path
    if shutil.which("gcc") is None:
        pytest.skip("no gcc")
    ora = Path(__file__).resolve().parents[1] / "oracle"
    exe = tmp_path / "drv"
    subprocess.run(["gcc", "-O2", "-g", "-std=c11", "-fsanitize=address,undefined", "-fno-omit-frame-pointer",
                    "-fno-sanitize-recover=all", "-Wno-unknown-pragmas", "-o", str(exe),
                    str(ora / "asan_driver.c"), str(ora / "tfhe_ref.c"), "-lm"], check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "0 wrong sign bits" in r.stdout
    assert "Sanitizer" not in r.stderr, r.stderr
