"""GPU parity: the HIP kernels (through the C ABI) against the exact CPU oracle.

Bit-exact: key material, encryptions, linear combinations, key switching,
and every decrypted value. After a bootstrap the GPU's f64-FFT rounding
differs from the oracle's exact Karatsuba product by a bounded phase error,
checked against a tolerance well inside the decision margin.
"""
from dataclasses import replace

import numpy as np
import pytest
import torch

from fheicp.params import TOY, SchemeParams, params_for_bits
from fheicp.engine import Engine, u64

pytestmark = pytest.mark.gpu

REAL16 = params_for_bits(16)


def signed(x):
    return np.asarray(x, dtype=np.uint64).view(np.int64)


@pytest.fixture(scope="module")
def toy(need_gpu, oracle_lib):
    eng = Engine(TOY, 0)
    eng.keygen(1234)
    ref = oracle_lib.RefTFHE(TOY.as_dict(), 1234)
    return eng, ref


@pytest.fixture(scope="module")
def toy_k1(need_gpu, oracle_lib):
    """k = 1, N = 256: kN = 256 mask words, so k_encrypt_linear's wave 0 owns
    words only on lanes 0-31 (the weights' v_readlane broadcast still reads
    lanes 32-63: ADVICE r04)."""
    P = replace(TOY, k=1)
    eng = Engine(P, 0)
    eng.keygen(4321)
    ref = oracle_lib.RefTFHE(P.as_dict(), 4321)
    return eng, ref


@pytest.fixture(scope="module")
def real(need_gpu, oracle_lib):
    eng = Engine(REAL16, 0)
    eng.keygen(777)
    ref = oracle_lib.RefTFHE(REAL16.as_dict(), 777)
    return eng, ref


@pytest.mark.parametrize("which", ["toy", "real"])
def test_keygen_bit_exact(which, request):
    eng, ref = request.getfixturevalue(which)
    keys = eng.export_keys()
    assert np.array_equal(keys["s_small"], ref.s_small)
    assert np.array_equal(keys["s_big"], ref.s_big)
    assert np.array_equal(keys["ksk"], ref.ksk)
    assert np.array_equal(keys["bsk"], ref.bsk)


@pytest.mark.parametrize("which", ["toy", "real"])
def test_encrypt_decrypt_bit_exact(which, request):
    eng, ref = request.getfixturevalue(which)
    P = eng.msg_bits
    rng = np.random.default_rng(5)
    v = rng.integers(-(2 ** (P - 1)), 2 ** (P - 1), 300)
    v[:4] = [-(2 ** (P - 1)), 2 ** (P - 1) - 1, 0, -1]
    ct = eng.encrypt(v, seed=99, id0=1000)
    ct_ref = ref.encrypt_ints(v, seed=99, id0=1000)
    assert np.array_equal(u64(ct).reshape(ct_ref.shape), ct_ref)
    assert np.array_equal(eng.decrypt(ct).cpu().numpy(), v)
    assert np.array_equal(ref.decrypt_ints(ct_ref), v)


@pytest.mark.parametrize("which", ["toy", "real"])
def test_linear_and_keyswitch_bit_exact(which, request):
    eng, ref = request.getfixturevalue(which)
    P = eng.msg_bits
    rng = np.random.default_rng(6)
    B, D = 40, 16
    x = rng.integers(-8, 8, (B, D))
    w = rng.integers(-31, 32, D)
    cst = int(rng.integers(-100, 100))
    ct = eng.encrypt(x, seed=3)
    ct_ref = ref.encrypt_ints(x, seed=3)
    lin = eng.linear(ct, B, D, w, cst)
    lin_ref = ref.linear(ct_ref, B, D, w, cst)
    assert np.array_equal(u64(lin), lin_ref)
    half = 2 ** (P - 1)
    expect = (x @ w + cst + half) % (2 * half) - half   # arithmetic mod 2^P
    assert np.array_equal(eng.decrypt(lin).cpu().numpy(), expect)
    for shift, add in ((0, 0), (P - 3, 1 << 62)):
        ks = eng.keyswitch(lin, shift, add)
        sh = (lin_ref << np.uint64(shift))
        sh[:, -1] += np.uint64(add)
        ks_ref = ref.keyswitch(sh)
        assert np.array_equal(u64(ks), ks_ref), f"keyswitch shift={shift}"


@pytest.mark.parametrize("B", [1, 17, 300, 1024, 2000])
def test_keyswitch_ragged_batches_bit_exact(real, B):
    """The MFMA key switch (k_keyswitch_mfma: 128 ciphertexts x 48 columns per
    workgroup, two 16-ciphertext groups per wave, a 4-deep load ring, K split
    over S workgroups: S = 20, 20, 8, 3 and 1 for these batches) on batches
    that leave idle waves and half-empty groups: bit-exact against the
    oracle's key switch on the rounded KSK."""
    eng, ref = real
    P = eng.msg_bits
    rng = np.random.default_rng(60 + B)
    v = rng.integers(-(2 ** (P - 1)), 2 ** (P - 1), B)
    ct = eng.encrypt(v, seed=61, id0=7 * B)
    ct_ref = ref.encrypt_ints(v, seed=61, id0=7 * B)
    eng.profile(True)
    ks = eng.keyswitch(ct, 2, 1 << 61)
    eng.profile(False)
    sh = ct_ref << np.uint64(2)
    sh[:, -1] += np.uint64(1 << 61)
    assert np.array_equal(u64(ks), ref.keyswitch(sh))
    # three byte planes of the rounded KSK, three column blocks per workgroup
    assert eng.kernel_name("keyswitch") == "k_keyswitch_mfma<3, 3>"


def test_keyswitch_valu_variant_bit_exact(need_gpu, oracle_lib, monkeypatch):
    """The VALU split-K key switch (k_keyswitch, the path for parameter sets
    the i8 matrix cores cannot take; FHEICP_KS_VARIANT=1 forces it) reads the
    same rounded KSK words (ks_round) and its colsum: bit-exact against the
    oracle, like the MFMA form."""
    monkeypatch.setenv("FHEICP_KS_VARIANT", "1")
    eng = Engine(TOY, 0)
    eng.keygen(4242)
    ref = oracle_lib.RefTFHE(TOY.as_dict(), 4242)
    v = np.random.default_rng(62).integers(-128, 128, 70)
    ct = eng.encrypt(v, seed=63)
    sh = ref.encrypt_ints(v, seed=63) << np.uint64(3)
    sh[:, -1] += np.uint64(1 << 60)
    assert np.array_equal(u64(eng.keyswitch(ct, 3, 1 << 60)), ref.keyswitch(sh))
    eng.profile(True)
    eng.keyswitch(ct, 0, 0)
    eng.profile(False)
    assert eng.kernel_name("keyswitch") == "k_keyswitch"


def test_pbs_matches_oracle_toy(toy):
    eng, ref = toy
    rng = np.random.default_rng(7)
    v = rng.integers(-128, 128, 24)
    ct = eng.encrypt(v, seed=11)
    small = eng.keyswitch(ct, 0, 0)
    tv = 1 << 61
    out = eng.pbs(small, tv)
    out_ref = ref.pbs_const(u64(small), tv)
    ph = signed(u64(eng.phase(out)))
    ph_ref = signed(ref.phase(out_ref))
    # sign of the bootstrapped phase follows the input phase half-torus
    expect = np.where(v >= 0, tv, -tv)
    assert np.all(np.abs(ph - expect) < 2 ** 52)
    assert np.all(np.abs(ph_ref - expect) < 2 ** 52)
    # GPU f64 FFT vs exact product. Mask words diverge as soon as one gadget
    # digit rounds the other way (a +-1 digit adds a whole random BSK row),
    # but the phases must agree to within noise level.
    assert np.abs(ph - ph_ref).max() < 2 ** 48


def test_bit_extract_toy(toy):
    eng, ref = toy
    P = eng.msg_bits
    rng = np.random.default_rng(8)
    v = rng.integers(-(2 ** (P - 1)), 2 ** (P - 1), 64)
    v[:3] = [-(2 ** (P - 1)), 2 ** (P - 1) - 1, 0]
    ct = eng.encrypt(v, seed=12)
    ref_ct, sign = eng.bit_extract(ct)
    assert np.array_equal(eng.decrypt(ref_ct).cpu().numpy(), v)
    assert np.array_equal(eng.decrypt_bits(sign).cpu().numpy(), (v < 0).astype(np.int64))
    # oracle on a few, bit-exact decrypts and close phases
    ct_ref = ref.encrypt_ints(v[:4], seed=12)
    r2, s2 = ref.bit_extract(ct_ref)
    assert np.array_equal(ref.decrypt_ints(r2), v[:4])
    d = signed(u64(eng.phase(ref_ct[:4].contiguous())) - ref.phase(r2))
    assert np.abs(d).max() < 2 ** (64 - P - 4)


def test_bit_extract_real_params(real):
    eng, ref = real
    P = eng.msg_bits
    rng = np.random.default_rng(9)
    v = rng.integers(-(2 ** (P - 1)), 2 ** (P - 1), 256)
    v[:4] = [-(2 ** (P - 1)), 2 ** (P - 1) - 1, 0, -1]
    ct = eng.encrypt(v, seed=21)
    ref_ct, sign = eng.bit_extract(ct)
    got = eng.decrypt(ref_ct).cpu().numpy()
    assert np.array_equal(got, v)
    assert np.array_equal(eng.decrypt_bits(sign).cpu().numpy(), (v < 0).astype(np.int64))
    # refreshed = sum of P bit ciphertexts: noise ~ sqrt(P) * sigma_pbs
    # (DESIGN.md §3.5), still inside the Delta/2 decoding margin
    ph = signed(u64(eng.phase(ref_ct)))
    err = ph - (v.astype(np.int64) << (64 - P))
    assert np.abs(err).max() < 2 ** (63 - P)
    assert np.std(err.astype(np.float64)) < 2 ** 45.5


def test_single_pbs_real_vs_oracle(real):
    eng, ref = real
    v = np.array([-30000, -12000, 12000, 30000], dtype=np.int64)  # |phase| >> KS+MS noise
    ct = eng.encrypt(v, seed=31)
    small = eng.keyswitch(ct, 0, 0)
    out = eng.pbs(small, 1 << 62)
    out_ref = ref.pbs_const(u64(small), 1 << 62)
    ph = signed(u64(eng.phase(out)))
    ph_ref = signed(ref.phase(out_ref))
    assert np.abs(ph - ph_ref).max() < 2 ** 48
    assert np.array_equal(ph > 0, v >= 0)


def test_topk_matches_stable_sort(need_gpu):
    eng = Engine(TOY, 0)
    rng = np.random.default_rng(10)
    for B, k in ((1000, 10), (37, 50), (5000, 1), (0, 3)):
        acc = rng.integers(-20, 20, B)   # many ties
        below = (rng.random(B) < 0.3).astype(np.int64)
        oa, oi = eng.topk(eng.to_dev(acc), eng.to_dev(below), k, base_idx=100)
        keep = [(i, int(acc[i])) for i in range(B) if not below[i]]
        keep.sort(key=lambda x: x[1], reverse=True)     # Python stable sort
        exp = keep[:k]
        got_i = oi.cpu().numpy()
        got_a = oa.cpu().numpy()
        assert [int(i) - 100 for i in got_i[:len(exp)]] == [i for i, _ in exp]
        assert [int(a) for a in got_a[:len(exp)]] == [a for _, a in exp]
        assert np.all(got_i[len(exp):] == -1)


def _need_ab():
    from fheicp import _lib
    if not _lib.ab_build():
        pytest.skip("A/B-only kernel shape: run with FHEICP_LIB=<tools/build_variant.sh ab -DFHEICP_AB build>")


@pytest.mark.parametrize("variant", ["2", "3"])
def test_bit_extract_real_params_other_kernels(need_gpu, oracle_lib, monkeypatch, variant):
    """The other blind-rotation kernels (FHEICP_BR_VARIANT=2: two waves per
    ciphertext, shipped for gadget levels >= 4; 3: four, A/B builds only)
    give the same results as the default (v4)."""
    if variant == "3":
        _need_ab()
    monkeypatch.setenv("FHEICP_BR_VARIANT", variant)
    eng = Engine(REAL16, 0)
    eng.keygen(777)
    P = eng.msg_bits
    v = np.random.default_rng(19).integers(-(2 ** (P - 1)), 2 ** (P - 1), 128)
    ref_ct, sign = eng.bit_extract(eng.encrypt(v, seed=22))
    assert np.array_equal(eng.decrypt(ref_ct).cpu().numpy(), v)
    assert np.array_equal(eng.decrypt_bits(sign).cpu().numpy(), (v < 0).astype(np.int64))


@pytest.mark.parametrize("P,dbits", [(8, 3), (8, 4), (7, 4), (5, 4), (4, 4)])
def test_sign_toy_all_values_vs_oracle(need_gpu, oracle_lib, P, dbits):
    """Digit sign extraction (fhe_sign_batch) with 3- and 4-bit digits: every
    toy value, each branch shape (full digits, a 3-bit leftover digit at P=7,
    a single leftover bit at P=5, the top chunk alone at P=4), and the GPU
    sign ciphertexts' phases track the oracle's restatement."""
    prm = replace(TOY, msg_bits=P, sign_digit_bits=dbits)
    eng = Engine(prm, 0)
    eng.keygen(1234)
    ref = oracle_lib.RefTFHE(prm.as_dict(), 1234)
    v = np.arange(-(2 ** (P - 1)), 2 ** (P - 1), dtype=np.int64)
    sign = eng.sign(eng.encrypt(v, seed=41))
    assert np.array_equal(eng.decrypt_bits(sign).cpu().numpy(), (v < 0).astype(np.int64))
    h = 2 ** (P - 1)
    sel = np.array([0, 1, h - 1, h, h + 1, 2 * h - 1])
    s_ref = ref.sign_extract(ref.encrypt_ints(v[sel], seed=41, id0=0))
    assert np.array_equal(ref.decrypt_bits(s_ref), (v[sel] < 0).astype(np.int64))
    d = signed(u64(eng.phase(sign[sel].contiguous())) - ref.phase(s_ref))
    assert np.abs(d).max() < 2 ** 56
    eng.close()


TOY_FAST = dict(pbs_base_log=12, pbs_level=3, pbs_fast_base_log=8, pbs_fast_level=2)


@pytest.mark.parametrize("P,grp", [(8, 1), (16, 2), (16, 1), (19, 2), (26, 2)])
def test_fast_bsk_bit_exact(need_gpu, oracle_lib, P, grp):
    """Every bootstrapping key of a multi-gadget parameter set (toy (12,3)+(8,2);
    real P=16: (15,2) + (15,2) + (23,1); P=19: (12,3) + mid (12,3) + (15,2) +
    (23,1); P=26: (6,7) + mid0 (5,8) + mid (8,5) + mid2 (12,3) + (15,2) +
    (23,1)) is
    bit-exact against the oracle's keygen, the fast gadgets' keys as
    multi-bit keys (group 2: three GGSWs per pair) and as classic ones, the
    mid gadgets' as the planner sets them (multi-bit)."""
    prm = replace(TOY, msg_bits=P, **TOY_FAST) if P < 12 else params_for_bits(P)
    if P >= 12:
        prm = replace(prm, pbs_fast_group=grp, pbs_fast2_group=grp)
    assert prm.pbs_fast_level
    eng = Engine(prm, 0)
    eng.keygen(4321)
    ref = oracle_lib.RefTFHE(prm.as_dict(), 4321)
    assert np.array_equal(eng.export_keys()["bsk"], ref.bsk)
    assert np.array_equal(eng.export_fast_bsk(1), ref.bsk2)
    if prm.pbs_fast2_level:
        assert np.array_equal(eng.export_fast_bsk(2), ref.bsk3)
    for which in (3, 4, 5):
        if which in ref.keys:
            assert np.array_equal(eng.export_fast_bsk(which), ref.keys[which]), which
    assert (3 in ref.keys) == (P >= 17)   # multi-bit mid keys (tags 21-24) from P = 17
    assert (5 in ref.keys) == (P >= 25)   # the multi-bit mid0 key (tags 27-28) from P = 25
    eng.close()


@pytest.mark.parametrize("P,dbits,mid2,mid0", [(11, 4, None, None), (11, 3, (9, 2), None),
                                               (11, 3, (9, 2), (11, 3))])
def test_sign_toy_mid_gadgets_vs_oracle(need_gpu, oracle_lib, P, dbits, mid2, mid0):
    """Mid gadgets (toy main (12,3) [-> mid0 (11,3)] -> mid (10,2) [-> mid2
    (9,2)] -> fast (8,2) -> fast2 (11,1)): the schedule puts rounds on every
    key (with mid0, on all but the main one), the mid keys are bit-exact,
    every value keeps its sign and the phases track the oracle's six-key
    restatement."""
    from fheicp.params import sign_schedule
    kw = dict(TOY_FAST3, pbs_mid_base_log=10, pbs_mid_level=2)
    if mid2:
        kw.update(pbs_mid2_base_log=mid2[0], pbs_mid2_level=mid2[1])
    if mid0:
        kw.update(pbs_mid0_base_log=mid0[0], pbs_mid0_level=mid0[1])
    prm = replace(TOY, msg_bits=P, sign_digit_bits=dbits, **kw)
    want = {5, 1, 2, 3, 4} if mid0 else {0, 1, 2, 3, 4} if mid2 else {0, 1, 2, 3}
    assert set(sign_schedule(prm)[1]) == want
    eng = Engine(prm, 0)
    eng.keygen(4324)
    ref = oracle_lib.RefTFHE(prm.as_dict(), 4324)
    for which in sorted(ref.keys):
        assert np.array_equal(eng.export_fast_bsk(which), ref.keys[which]), which
    v = np.arange(-(2 ** (P - 1)), 2 ** (P - 1), dtype=np.int64)
    sign = eng.sign(eng.encrypt(v, seed=64))
    assert np.array_equal(eng.decrypt_bits(sign).cpu().numpy(), (v < 0).astype(np.int64))
    h = 2 ** (P - 1)
    sel = np.array([0, 1, h - 1, h, h + 1, 2 * h - 1])
    s_ref = ref.sign_extract(ref.encrypt_ints(v[sel], seed=64, id0=0))
    assert np.array_equal(ref.decrypt_bits(s_ref), (v[sel] < 0).astype(np.int64))
    # the last round is on the coarse (11,1) toy gadget (see the three-gadget test)
    dph = signed(u64(eng.phase(sign[sel].contiguous())) - ref.phase(s_ref))
    assert np.abs(dph).max() < 2 ** 61
    eng.close()


@pytest.mark.parametrize("P,dbits", [(8, 3), (11, 4)])
def test_sign_toy_fast_gadget_vs_oracle(need_gpu, oracle_lib, P, dbits):
    """Per-round gadgets on the GPU: the leading sign_precise_rounds bootstraps
    on the main key, the rest on the fast one, every value exact, and the sign
    ciphertexts' phases track the oracle's two-key restatement."""
    from fheicp.params import sign_plan, sign_rounds
    prm = replace(TOY, msg_bits=P, sign_digit_bits=dbits, **TOY_FAST)
    d, j, _ = sign_plan(prm)
    assert 0 < j < len(sign_rounds(P, d))
    eng = Engine(prm, 0)
    eng.keygen(4321)
    ref = oracle_lib.RefTFHE(prm.as_dict(), 4321)
    v = np.arange(-(2 ** (P - 1)), 2 ** (P - 1), dtype=np.int64)
    sign = eng.sign(eng.encrypt(v, seed=61))
    assert np.array_equal(eng.decrypt_bits(sign).cpu().numpy(), (v < 0).astype(np.int64))
    h = 2 ** (P - 1)
    sel = np.array([0, 1, h - 1, h, h + 1, 2 * h - 1])
    s_ref = ref.sign_extract(ref.encrypt_ints(v[sel], seed=61, id0=0))
    assert np.array_equal(ref.decrypt_bits(s_ref), (v[sel] < 0).astype(np.int64))
    dph = signed(u64(eng.phase(sign[sel].contiguous())) - ref.phase(s_ref))
    assert np.abs(dph).max() < 2 ** 56
    # imported keys: the fast key is re-encrypted with fresh randomness, the
    # signs are unchanged
    eng2 = Engine(prm, 0)
    eng2.import_keys(eng.export_keys())
    assert not np.array_equal(eng2.export_fast_bsk(), eng.export_fast_bsk())
    sign2 = eng2.sign(eng2.encrypt(v, seed=62))
    assert np.array_equal(eng2.decrypt_bits(sign2).cpu().numpy(), (v < 0).astype(np.int64))
    eng2.close()
    eng.close()


TOY_FAST3 = dict(TOY_FAST, pbs_fast2_base_log=11, pbs_fast2_level=1)


@pytest.mark.parametrize("P,dbits", [(8, 3), (11, 4)])
def test_sign_toy_three_gadgets_vs_oracle(need_gpu, oracle_lib, P, dbits):
    """Three gadgets (toy (12,3) + (8,2) + (11,1)): the plan puts rounds on
    all three keys; every value is exact and the phases track the oracle."""
    from fheicp.params import sign_plan, sign_rounds
    prm = replace(TOY, msg_bits=P, sign_digit_bits=dbits, **TOY_FAST3)
    d, j1, j2 = sign_plan(prm)
    assert 0 < j1 < j2 < len(sign_rounds(P, d))
    eng = Engine(prm, 0)
    eng.keygen(4323)
    ref = oracle_lib.RefTFHE(prm.as_dict(), 4323)
    assert np.array_equal(eng.export_fast_bsk(2), ref.bsk3)
    v = np.arange(-(2 ** (P - 1)), 2 ** (P - 1), dtype=np.int64)
    sign = eng.sign(eng.encrypt(v, seed=63))
    assert np.array_equal(eng.decrypt_bits(sign).cpu().numpy(), (v < 0).astype(np.int64))
    h = 2 ** (P - 1)
    sel = np.array([0, 1, h - 1, h, h + 1, 2 * h - 1])
    s_ref = ref.sign_extract(ref.encrypt_ints(v[sel], seed=63, id0=0))
    assert np.array_equal(ref.decrypt_bits(s_ref), (v[sel] < 0).astype(np.int64))
    # the last round runs on the coarse (11,1) toy gadget: the two outputs'
    # noise (sigma ~2^58) differs wherever a rounding decision of the gadget
    # decomposition flips, so they agree within the noise, inside the 2^62
    # decryption margin
    dph = signed(u64(eng.phase(sign[sel].contiguous())) - ref.phase(s_ref))
    assert np.abs(dph).max() < 2 ** 61
    eng.close()


@pytest.mark.parametrize("P,dbits,fast", [(16, 0, True), (16, 3, True), (16, 0, "classic"), (19, 0, True),
                                          (19, 0, False), (21, 0, True), (21, 0, False), (25, 0, True),
                                          (26, 0, True)])
def test_sign_real_params(need_gpu, P, dbits, fast):
    """Real parameters at the C2/C4 (P=16: 4-bit digits, and 3-bit forced),
    C3 (P=21: 3-bit) and C5 (P=26: six gadgets, the first round on the
    multi-bit mid0 (5,8); P=25: mid0 (6,7)) widths,
    with (fast; multi-bit fast gadgets) and
    without the per-round fast gadgets, and with the fast gadgets on the
    classic rotation ("classic"), boundaries included."""
    prm = params_for_bits(P, fast=bool(fast))
    if fast == "classic":
        prm = replace(prm, pbs_fast_group=1, pbs_fast2_group=1)
    eng = Engine(replace(prm, sign_digit_bits=dbits), 0)
    eng.keygen(900 + P)
    rng = np.random.default_rng(P)
    h = 2 ** (P - 1)
    v = rng.integers(-h, h, 1024)
    v[:8] = [-h, -h + 1, -2, -1, 0, 1, h - 2, h - 1]
    sign = eng.sign(eng.encrypt(v, seed=P))
    assert np.array_equal(eng.decrypt_bits(sign).cpu().numpy(), (v < 0).astype(np.int64))
    eng.close()


def test_sign_every_width(need_gpu):
    """Every accumulator width the parameter table supports (P = 2..27), each
    with its params_for_bits gadgets and sign plan (single gadget, (23,1) or
    (15,2) fast rounds; v4 32- and 64-bit and v2 kernels): the boundary values
    and a random sample keep their exact sign."""
    from fheicp.params import sign_plan
    rng = np.random.default_rng(2027)
    for P in range(2, 28):
        prm = params_for_bits(P)
        eng = Engine(prm, 0)
        eng.keygen(3000 + P)
        h = 2 ** (P - 1)
        v = np.concatenate([[-h, -h + 1, -2, -1, 0, 1, h - 2, h - 1] if P > 2 else [-2, -1, 0, 1],
                            rng.integers(-h, h, 248)]).astype(np.int64)
        sign = eng.sign(eng.encrypt(v, seed=P))
        got = eng.decrypt_bits(sign).cpu().numpy()
        assert np.array_equal(got, (v < 0).astype(np.int64)), (P, sign_plan(prm))
        eng.close()


def test_pbs_lut_real_vs_oracle(real):
    """4-slot staircase bootstrap on the real parameters, against the oracle."""
    eng, ref = real
    D = np.array([0, 1, 2, 3], dtype=np.uint64)
    msg = (D << np.uint64(61)) + np.uint64(1 << 60)
    ct = eng.to_dev(msg.view(np.int64))
    enc = eng.encrypt(np.zeros(4, np.int64), seed=51)        # encryptions of 0 ...
    enc[:, -1] += ct                                          # ... shifted to the raw phases
    small = eng.keyswitch(enc, 0, 0)
    out = eng.pbs_lut(small, 0, 1 << 48, 2)
    out_ref = ref.pbs_lut(u64(small), 0, 1 << 48, 2)
    ph = signed(u64(eng.phase(out)))
    assert np.abs(ph - signed(ref.phase(out_ref))).max() < 2 ** 46
    assert np.abs(ph - (D.astype(np.int64) << 48)).max() < 2 ** 46


@pytest.mark.parametrize("g,fl", [("4", "0"), ("4", "1"), ("2", "0"), ("2", "1"), ("1", "0")])
def test_v4_workgroup_shapes(need_gpu, monkeypatch, g, fl):
    """Every v4 workgroup shape (FHEICP_V4_G ciphertexts per workgroup, s_barrier
    or per-ciphertext LDS hand-offs FHEICP_V4_FL) gives the exact sign and
    refreshed value on the real parameters, with a batch that is not a multiple
    of the workgroup (B = 1023: the last workgroup runs padding ciphertexts)."""
    if (g, fl) != ("4", "0"):
        _need_ab()
    monkeypatch.setenv("FHEICP_V4_G", g)
    monkeypatch.setenv("FHEICP_V4_FL", fl)
    eng = Engine(REAL16, 0)
    eng.keygen(777)
    h = 2 ** 15
    v = np.random.default_rng(23).integers(-h, h, 1023)
    v[:6] = [-h, -1, 0, 1, h - 1, -h + 1]
    sign = eng.sign(eng.encrypt(v, seed=24))
    assert np.array_equal(eng.decrypt_bits(sign).cpu().numpy(), (v < 0).astype(np.int64))
    ref_ct, sign2 = eng.bit_extract(eng.encrypt(v[:64], seed=25))
    assert np.array_equal(eng.decrypt(ref_ct).cpu().numpy(), v[:64])
    eng.close()


def test_pbs_table_every_value_real(real):
    """fhe_pbs_table_batch on the real parameters: an arbitrary 3-bit table
    (a requantisation-like map with signed outputs) over every input, 64
    times each, decrypts exactly; a 4-bit table over every input decrypts
    exactly and its phases track the oracle's ref_pbs_table."""
    eng, ref = real
    P = eng.msg_bits
    try:
        for lut_bits, reps in ((3, 64), (4, 1)):
            M = 1 << lut_bits
            lut = np.random.default_rng(lut_bits).integers(-(2 ** (P - 1)), 2 ** (P - 1), M)
            lut[0], lut[-1] = -(2 ** (P - 1)), 2 ** (P - 1) - 1
            m = np.tile(np.arange(M, dtype=np.int64), reps)
            eng.set_msg_bits(lut_bits + 1)          # input encoding: padding bit + lut_bits
            small = eng.keyswitch(eng.encrypt(m, seed=70 + lut_bits), 0, 0)
            eng.set_msg_bits(P)
            out = eng.pbs_table(small, lut, lut_bits)
            assert np.array_equal(eng.decrypt(out).cpu().numpy(), lut[m])
            if lut_bits == 4:
                ref.with_msg_bits(P)
                # the same gadget (fhe_pbs_table_gadget: (15,2) multi-bit here)
                o_ref = ref.pbs_table(u64(small)[:4], lut, lut_bits, gadget=eng.table_gadget())
                assert np.array_equal(ref.decrypt_ints(o_ref), lut[m[:4]])
                d = signed(u64(eng.phase(out[:4].contiguous())) - ref.phase(o_ref))
                assert np.abs(d).max() < 2 ** 48
    finally:
        eng.set_msg_bits(P)


def test_threshold_batch_real(real):
    """fhe_threshold_batch: [acc >= T] (batch_operations.py:278) for
    accumulators at and around T and at the ends of the 16-bit range; the
    accumulator ciphertext is left unchanged; the oracle's restatement
    decrypts to the same bits."""
    eng, ref = real
    P = eng.msg_bits
    T = 1234
    h = 2 ** (P - 2)
    acc = np.concatenate([[T - 2, T - 1, T, T + 1, -h, h - 1, 0, -1],
                          np.random.default_rng(77).integers(-h, h, 504)]).astype(np.int64)
    ct = eng.encrypt(acc, seed=78)
    before = u64(ct).copy()
    bit = eng.threshold(ct, T)
    assert np.array_equal(u64(ct), before)
    assert np.array_equal(eng.decrypt_bits(bit).cpu().numpy(), (acc >= T).astype(np.int64))
    b_ref = ref.threshold(u64(ct)[:4], T)
    assert np.array_equal(ref.decrypt_bits(b_ref), (acc[:4] >= T).astype(np.int64))


@pytest.mark.parametrize("which", ["toy", "real", "toy_k1"])
def test_encrypt_linear_fused_bit_exact(which, request):
    """fhe_encrypt_linear_batch (the fused client encryption + leveled dot of
    fhe_compare_batch / fhe_score_batch, packed features: DESIGN.md §3.2) is
    bit-identical to fhe_encrypt_packed_batch followed by
    fhe_linear_packed_batch, and both to the oracle's textbook GLWE encryption
    + product + sample extraction; GLWEs equal the oracle's word for word. D
    covers a count that is not a multiple of anything (37), the compare
    path's 16, and more features than N (two GLWEs per row); the last case
    draws weights over the whole int64 range (the MAC's general high-word
    term, |w| >= 2^31) and is checked word for word only (its message wraps)."""
    eng, ref = request.getfixturevalue(which)
    rng = np.random.default_rng(11)
    N = eng.params.N
    for B, D in ((5, 37), (64, 16), (3, N + 44), (4, 70)):
        x = rng.integers(-32, 32, (B, D))
        wide = D == 70
        w = rng.integers(-2 ** 63, 2 ** 63 - 1, D) if wide else rng.integers(-127, 128, D)
        cst = int(rng.integers(-1000, 1000))
        fused = u64(eng.encrypt_linear(x, w, cst, seed=8, id0=77))
        glwe = eng.encrypt_packed(x, seed=8, id0=77)
        glwe_ref = ref.encrypt_packed(x, seed=8, id0=77)
        assert np.array_equal(u64(glwe).reshape(glwe_ref.shape), glwe_ref), (B, D)
        two = u64(eng.linear_packed(glwe, D, w, cst))
        assert np.array_equal(fused, two), (B, D)
        lin_ref = ref.linear_packed(glwe_ref, D, w, cst)
        assert np.array_equal(fused, lin_ref), (B, D)
        if wide:
            continue
        half = 2 ** (eng.msg_bits - 1)
        assert np.array_equal(ref.decrypt_ints(lin_ref), (x @ w + cst + half) % (2 * half) - half)


def test_pbs_table_every_multibit_gadget(need_gpu, oracle_lib):
    """The table bootstrap on every multi-bit gadget of the P = 26 set (mid0
    (5,8), mid (8,5), mid2 (12,3) on the 48-bit k_blind_rotate_mb64, fast
    (15,2) and fast2 (23,1) on the 32-bit k_blind_rotate_mb, each with the
    table test vector and that gadget's key) and on the classic main gadget:
    a 3-bit table over every input, 16 times each, decrypts exactly at an
    output width the gadget's noise carries (>= 8 sigma at half a step:
    26 bits on (5,8) and (6,7), 24 on (8,5), 20 on (12,3), 16 on (15,2), 10
    on (23,1)); the
    default gadget is the most precise multi-bit one (mid0); the launched
    instantiation is the BrTvLut one; on mid0 and fast the phases of four
    outputs agree with the oracle's ref_pbs_table_gadget to noise level."""
    p = params_for_bits(26)
    eng = Engine(p, 0)
    eng.keygen(8026)
    ref = None
    P = p.msg_bits
    assert eng.table_gadget() == 5
    lut_bits, M = 3, 8
    m = np.tile(np.arange(M, dtype=np.int64), 16)
    eng.set_msg_bits(lut_bits + 1)
    small = eng.keyswitch(eng.encrypt(m, seed=81), 0, 0)
    buckets = {1: "fast", 2: "fast2", 3: "mid", 4: "mid2", 5: "mid0"}
    out_bits = {5: 26, 3: 24, 4: 20, 1: 16, 2: 10, 0: 26}
    for gad in (5, 3, 4, 1, 2, 0):
        Po = out_bits[gad]
        lut = np.random.default_rng(26 + gad).integers(-(2 ** (Po - 1)), 2 ** (Po - 1), M)
        eng.set_msg_bits(Po)
        eng.profile(True)
        out = eng.pbs_table(small, lut, lut_bits, gadget=gad)
        eng.profile(False)
        assert np.array_equal(eng.decrypt(out).cpu().numpy(), lut[m]), gad
        if gad:
            name = eng.kernel_name(f"blind_rotate_{buckets[gad]}")
            assert name.endswith("BrTvLut>") and ("mb64<" in name) == (gad in (3, 4, 5)), (gad, name)
            eng.profile_read(f"blind_rotate_{buckets[gad]}")
        if gad in (5, 1):
            if ref is None:   # the oracle's keys of the two gadgets checked (and the main one) only
                keep = replace(p, pbs_mid_base_log=0, pbs_mid_level=0, pbs_mid_group=0, pbs_mid2_base_log=0,
                               pbs_mid2_level=0, pbs_mid2_group=0, pbs_fast2_base_log=0, pbs_fast2_level=0,
                               pbs_fast2_group=0)
                ref = oracle_lib.RefTFHE(keep.as_dict(), 8026)
            ref.with_msg_bits(Po)
            o_ref = ref.pbs_table(u64(small)[:4], lut, lut_bits, gadget=gad)
            assert np.array_equal(ref.decrypt_ints(o_ref), lut[m[:4]])
            d = signed(u64(eng.phase(out[:4].contiguous())) - ref.phase(o_ref))
            assert np.abs(d).max() < 2 ** 48, gad
    eng.set_msg_bits(P)
    lut = np.random.default_rng(26).integers(-(2 ** (P - 1)), 2 ** (P - 1), M)
    out = eng.pbs_table(small, lut, lut_bits)       # the default: mid0
    assert np.array_equal(eng.decrypt(out).cpu().numpy(), lut[m])
    eng.close()
