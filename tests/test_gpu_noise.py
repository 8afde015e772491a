"""GPU: the bootstrap noise that "bit-exact" rests on, per shipped
blind-rotation instance.

Every decision of the sign extraction is exact only while the noise stays
inside its margin (>= 9.2 sigma of the model, p_fail <= 2^-64 per bootstrap;
DESIGN.md §3.5). Sampling a thousand compares cannot show that, so for each
kernel instance the parameter table can select (v4 32-bit accumulators at
(15,2) and (23,1), the key-stationary v4s with 64-bit accumulators at (12,3)
and levels 4..8, and the multi-bit rotation of the fast gadgets at (15,2)
and (23,1), plus its run-time-base-log instances, and the deep gadgets on
the multi-bit rotation with 48-bit accumulators) this measures the output noise of >= 4096 bootstraps on the real
parameters and checks it against the model (fheicp.params._variances, the
same formula as fheicp.hip and oracle/tfhe_ref.c), and checks a few output
phases against the exact oracle's bootstrap of the same inputs.
"""
import math

import numpy as np
import pytest

from fheicp.engine import Engine, u64
from dataclasses import replace

from fheicp.params import SchemeParams, _variances

pytestmark = pytest.mark.gpu

# (base_log, level, group) -> the instantiation fhe_profile_kernel_name
# reports; group 2 = the multi-bit rotation, run as a fast gadget
INSTANCES = {
    (15, 2, 1): "k_blind_rotate_v4<2, true, 0, 4, false, 15>",
    (23, 1, 1): "k_blind_rotate_v4<1, true, 0, 4, false, 23>",
    (14, 2, 1): "k_blind_rotate_v4<2, true, 0, 4, false, 0>",   # run-time base log
    (22, 1, 1): "k_blind_rotate_v4<1, true, 0, 4, false, 0>",
    (12, 3, 1): "k_blind_rotate_v4s<3, false, 0, 0>",
    # level 3 with L * beta <= 31: the 64-bit kernel too (no 32-bit level-3 instance ships)
    (10, 3, 1): "k_blind_rotate_v4s<3, false, 0, 0>",
    (10, 4, 1): "k_blind_rotate_v4s<4, false, 0, 0>",
    (8, 5, 1): "k_blind_rotate_v4s<5, false, 0, 0>",
    (7, 6, 1): "k_blind_rotate_v4s<6, false, 0, 0>",
    (6, 7, 1): "k_blind_rotate_v4s<7, false, 0, 0>",
    (5, 8, 1): "k_blind_rotate_v4s<8, false, 0, 0>",
    (15, 2, 2): "k_blind_rotate_mb<2, 0, 15, BrTv>",
    (23, 1, 2): "k_blind_rotate_mb<1, 0, 23, BrTv>",
    # the multi-bit kernels with a run-time base log (other gadgets)
    (14, 2, 2): "k_blind_rotate_mb<2, 0, 0, BrTv>",
    (22, 1, 2): "k_blind_rotate_mb<1, 0, 0, BrTv>",
    # the deep gadgets on the multi-bit rotation, 48-bit accumulators
    (12, 3, 2): "k_blind_rotate_mb64<3, 0, BrTv>",
    (10, 4, 2): "k_blind_rotate_mb64<4, 0, BrTv>",
    (8, 5, 2): "k_blind_rotate_mb64<5, 0, BrTv>",
    (7, 6, 2): "k_blind_rotate_mb64<6, 0, BrTv>",
    (6, 7, 2): "k_blind_rotate_mb64<7, 0, BrTv>",
    (5, 8, 2): "k_blind_rotate_mb64<8, 0, BrTv>",
    # level 2 with L * beta > 31 also takes the 48-bit kernel (level 1 would
    # need beta >= 32, which fhe_ctx_create refuses for multi-bit gadgets)
    (16, 2, 2): "k_blind_rotate_mb64<2, 0, BrTv>",
}
COUNT = 4096
TV = 1 << 61


def signed(x):
    return np.asarray(x, dtype=np.uint64).view(np.int64)


@pytest.mark.parametrize("gadget", list(INSTANCES))
def test_bootstrap_noise_vs_model(need_gpu, oracle_lib, gadget):
    beta, lvl, grp = gadget
    if grp == 1:
        prm = SchemeParams(pbs_base_log=beta, pbs_level=lvl, msg_bits=16)
    else:   # a fast gadget of a set whose main gadget is (15, 2)
        prm = SchemeParams(msg_bits=16, pbs_fast_base_log=beta, pbs_fast_level=lvl, pbs_fast_group=2)
    g = 0 if grp == 1 else 1
    bucket = "blind_rotate_main" if g == 0 else "blind_rotate_fast"
    eng = Engine(prm, 0)
    seed = 5000 + 10 * beta + lvl + 100 * (grp - 1)
    eng.keygen(seed)
    # inputs at phase +-2^62: far from the 0 / 2^63 boundaries, so the key
    # and modulus switch noise never flips the rotation's half of the torus
    sgn = np.where(np.arange(COUNT) % 2 == 0, 1, -1).astype(np.int64)
    v = sgn * (1 << 14)
    small = eng.keyswitch(eng.encrypt(v, seed=17), 0, 0)
    eng.profile(True)
    out = eng.pbs_gadget(small, g, TV)
    eng.profile(False)
    assert eng.kernel_name(bucket) == INSTANCES[gadget]
    prof = eng.profile_read(bucket)
    assert prof["items"] == COUNT
    print(f"gadget {gadget}: {prof['total_ms'] / prof['launches'] * 1024 / COUNT:.3f} ms per 1024 bootstraps")
    ph = signed(u64(eng.phase(out)))
    err = (ph - sgn * TV).astype(np.float64) / 2.0 ** 64
    sigma = float(np.sqrt(np.mean(err ** 2)))   # RMS: a bias would count too
    sigma_model = math.sqrt(_variances(replace(prm, pbs_base_log=beta, pbs_level=lvl), group=grp)[0])
    print(f"gadget {gadget}: sigma 2^{math.log2(sigma):.2f}, model 2^{math.log2(sigma_model):.2f}, "
          f"max |err| {np.abs(err).max() / sigma_model:.2f} model sigmas")
    assert sigma <= 1.1 * sigma_model
    # the same bootstraps in the exact oracle: phases agree to noise level
    ref = oracle_lib.RefTFHE(prm.as_dict(), seed)
    sm = u64(small)[:2]
    ph_ref = signed(ref.phase(ref.pbs_gadget(sm, g, TV)))
    assert np.abs(ph[:2] - ph_ref).max() < 8 * sigma_model * 2.0 ** 64
    assert np.array_equal(ph_ref > 0, sgn[:2] > 0)
    eng.close()


def test_multibit_digit_width_limit(need_gpu):
    """A multi-bit gadget with 32-bit digits is refused at context creation
    (the 48-bit kernel reads digits as 32-bit fields; measured before the
    check: sigma 2^-2.2 against a model of 2^-5.6 for (32, 1))."""
    from fheicp import _lib
    with pytest.raises(_lib.FheError, match="base_log <= 31"):
        Engine(SchemeParams(msg_bits=16, pbs_fast_base_log=32, pbs_fast_level=1, pbs_fast_group=2), 0)


@pytest.mark.parametrize("ks", [(3, 5), (4, 4)])
def test_keyswitch_noise_vs_model(need_gpu, ks):
    """The key switch's output noise (the second-largest fixed term of every
    sign round after the modulus switch) against the model's
    v_ks, for the shipped (3, 5) key switch (level-major i8 MFMA) and the
    former (4, 4): 4096 fresh encryptions, switched, decrypted on the host
    under the exported small key."""
    from fheicp.params import params_for_bits
    prm = replace(params_for_bits(16), ks_base_log=ks[0], ks_level=ks[1])
    eng = Engine(prm, 0)
    eng.keygen(6100 + ks[0])
    rng = np.random.default_rng(ks[0])
    v = rng.integers(-(2 ** 15), 2 ** 15, COUNT)
    small = u64(eng.keyswitch(eng.encrypt(v, seed=23), 0, 0)).reshape(COUNT, prm.n + 1)
    s = eng.export_keys()["s_small"].astype(np.uint64)
    with np.errstate(over="ignore"):
        ph = small[:, -1] - (small[:, :-1] * s[None, :]).sum(axis=1, dtype=np.uint64)
    err = signed(ph - (v.astype(np.int64).astype(np.uint64) << np.uint64(64 - 16))).astype(np.float64) / 2.0 ** 64
    sigma = float(np.sqrt(np.mean(err ** 2)))
    sigma_model = math.sqrt(_variances(prm)[1])
    print(f"key switch {ks}: sigma 2^{math.log2(sigma):.2f}, model 2^{math.log2(sigma_model):.2f}")
    assert sigma <= 1.1 * sigma_model
    assert sigma >= 0.7 * sigma_model        # the model is not vacuous either
    eng.close()
