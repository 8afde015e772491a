"""GPU: the decision noise that "bit-exact" rests on, measured round by round
inside the real sign extraction, and the failure rate at a narrowed margin.

Every threshold bit (the decision of batch_operations.py:278, reached through
predict(fhe="execute"), fhe_similarity.py:151) is exact only while each
bootstrap's rotation exponent stays inside its test-vector slot. The model
(fheicp.params._sched_worst, the same formula as fheicp.hip plan_worst and
oracle/tfhe_ref.c) gives each round's decision-noise sigma: every earlier
bootstrap's output noise amplified by 4^shift, plus the round's key switch and
modulus switch, and the plans keep >= 9.2 sigma.

fhe_sign_trace_batch runs the shipped extraction and reports every round's
rotation exponent phi (k_ms_phase: the key-switched phase switched to 2N
exactly as that round's rotation rounds it; checked here against a numpy
restatement of the oracle's rounding). tests/decision_noise_lib.py gives the
exact exponent of each round, so phi - ideal IS the decision noise:
  (a) per round of the shipped P = 16 plan (C2, C4) and the first round of
      C5's P = 26 plan, over >= 10^5 inputs: sigma against the model's;
  (b) at a deliberately narrowed margin (a noisy gadget ahead of a round), over
      >= 2 * 10^6 accumulators: the count of flipped decisions against the
      Gaussian tail at the measured sigma (the shape the 9.2-sigma
      extrapolation assumes) and against the model's rate, and every ciphertext
      without a flipped decision has the exact threshold bit.
"""
import math
import sys
from dataclasses import replace
from pathlib import Path

import numpy as np
import pytest
import torch

sys.path.insert(0, str(Path(__file__).resolve().parent))
import decision_noise_lib as DL  # noqa: E402
from fheicp.engine import Engine, u64  # noqa: E402
from fheicp.params import (_tuniform_var, params_for_bits, sign_digit_bits, sign_round_ops,  # noqa: E402
                           sign_round_sigmas, sign_schedule, gadget_of)

pytestmark = pytest.mark.gpu


def _trace(eng, v, sched=None, rounds=0, seed=11, ct=None):
    """Encrypt v (fresh, unless ct is given), run the traced extraction,
    return (phases [R][count] int64 on the host, sign bits or None)."""
    if ct is None:
        ct = eng.encrypt(v, seed=seed)
    sign, ph = eng.sign_trace(ct, sched=sched, rounds=rounds)
    bits = eng.decrypt_bits(sign).cpu().numpy() if sign is not None else None
    return ph.cpu().numpy().astype(np.int64) & 0xFFFFFFFF, bits


def _round_table(p, v, phases, sched, input_var=0.0, rounds=None):
    """Per round: measured mean / RMS of the decision noise (torus units)
    against the model sigma (with the input's own noise amplified)."""
    P, N = p.msg_bits, p.N
    d, _ = sign_schedule(p)
    ops = sign_round_ops(P, d, N)
    model = sign_round_sigmas(p, sched)
    out = []
    for r in range(len(phases) if rounds is None else rounds):
        ideal = DL.ideal_index(v, ops[r], P, N)
        err = DL.centred(phases[r], ideal, N).astype(np.float64) / (2 * N)
        sh, ml, sig = model[r]
        sig = math.sqrt(sig ** 2 + input_var * 4.0 ** sh)
        out.append(dict(round=r, gadget=sched[r], shift=sh, margin_log2=ml, model_log2=math.log2(sig),
                        meas_log2=math.log2(math.sqrt(np.mean(err ** 2))), ratio=math.sqrt(np.mean(err ** 2)) / sig,
                        mean_sig=float(np.mean(err)) / sig, max_sig=float(np.abs(err).max()) / sig,
                        margin_sig=2.0 ** ml / sig, flips=int(np.sum(
                            DL.tv_decode(phases[r], ops[r], N) != DL.tv_decode(ideal, ops[r], N)))))
    return out


def _print_table(title, rows):
    print(f"\n{title}")
    for t in rows:
        print(f"  round {t['round']} gadget {t['gadget']} shift {t['shift']:2d}: sigma 2^{t['meas_log2']:.2f} "
              f"(model 2^{t['model_log2']:.2f}, ratio {t['ratio']:.3f}), mean {t['mean_sig']:+.3f} sigma, "
              f"max |err| {t['max_sig']:.2f} sigma, margin {t['margin_sig']:.2f} model sigma, flips {t['flips']}")


def test_ms_phase_kernel_matches_numpy(need_gpu):
    """k_ms_phase (the trace's exponent) equals the numpy restatement of the
    oracle's modulus switch on the same key-switched ciphertexts, for the
    classic and the multi-bit rotation (round 0 of two plans)."""
    p = params_for_bits(16)
    eng = Engine(p, 0)
    eng.keygen(7101)
    s = eng.export_keys()["s_small"]
    rng = np.random.default_rng(1)
    v = rng.integers(-(1 << 15), 1 << 15, 2048)
    d, sched = sign_schedule(p)
    op = sign_round_ops(16, d, p.N)[0]
    for g in sorted({0, sched[0]}):
        ct = eng.encrypt(v, seed=5)
        small = u64(eng.keyswitch(ct.clone(), op["shift"], op["add"])).reshape(len(v), p.n + 1)
        phases, _ = _trace(eng, v, sched=[g] + list(sched[1:]), rounds=1, ct=ct)
        want = DL.ms_phase_numpy(small, s, p.N, gadget_of(p, g)[2] if g else 1)
        assert np.array_equal(phases[0], want), g
    eng.close()


def test_decision_noise_per_round_p16(need_gpu):
    """(a) Every round of the shipped P = 16 plan (C2 and the C4 shards),
    >= 10^5 uniformly drawn accumulators through the real extraction: each
    round's decision-noise sigma within [0.75, 1.1] x the model's, zero mean,
    no decision anywhere near its margin, every threshold bit exact."""
    p = params_for_bits(16)
    eng = Engine(p, 0)
    eng.keygen(7102)
    rng = np.random.default_rng(2)
    count = 1 << 17
    v = rng.integers(-(1 << 15), 1 << 15, count)
    _, sched = sign_schedule(p)
    phases, bits = _trace(eng, v)
    assert np.array_equal(bits, (v < 0).astype(np.int64))
    # fresh inputs: their own noise (TUniform(17), 2^-46.6) x 2^12 is < 2^-34: omitted
    rows = _round_table(p, v, phases, sched)
    _print_table(f"decision noise, P = 16 plan {sched}, {count} accumulators", rows)
    for t in rows:
        assert 0.75 <= t["ratio"] <= 1.1, t
        assert abs(t["mean_sig"]) < 0.05, t
        assert t["flips"] == 0 and t["max_sig"] < 0.75 * t["margin_sig"], t
    eng.close()


def test_decision_noise_first_round_c5(need_gpu):
    """(a) The first round of C5's P = 26 plan (mid0, multi-bit (5,8)): the
    input is the reference's leveled circuit itself (k_encrypt_linear at
    D = 768, n_bits = 8 ranges), so its noise sum_j w_j e_j, amplified by
    2^22, is in the prediction. >= 10^5 accumulators, sigma within
    [0.75, 1.1] x the model's, no decision near its margin."""
    p = params_for_bits(26)
    eng = Engine(p, 0)
    eng.keygen(7103)
    rng = np.random.default_rng(3)
    count, D = 1 << 17, 768
    x = rng.integers(-128, 128, (count, D))
    w = rng.integers(-127, 128, D)
    cst = int(rng.integers(-(1 << 20), 1 << 20))
    v = x @ w + cst
    assert np.abs(v).max() < (1 << 25)
    ct = eng.encrypt_linear(torch.from_numpy(x).to(eng.device), torch.from_numpy(w).to(eng.device), cst, seed=9)
    _, sched = sign_schedule(p)
    phases, _ = _trace(eng, v, rounds=1, ct=ct)
    input_var = float(np.sum(w.astype(np.float64) ** 2)) * _tuniform_var(p.glwe_noise_bits) / 2.0 ** 128
    rows = _round_table(p, v, phases, sched, input_var=input_var, rounds=1)
    _print_table(f"decision noise, P = 26 plan {sched}, round 0 only, {count} accumulators "
                 f"(input noise 2^{0.5 * math.log2(input_var):.2f} x 2^22)", rows)
    t = rows[0]
    assert 0.75 <= t["ratio"] <= 1.1, t
    assert abs(t["mean_sig"]) < 0.05, t
    assert t["flips"] == 0 and t["max_sig"] < 0.75 * t["margin_sig"], t
    eng.close()


def _narrowed(fast2, count, chunk, seed):
    """The P = 11 extraction on the shipped key set with fast2 = `fast2`
    (multi-bit) on every round: round 1 decides on v << 7 carrying round 0's
    output noise x 2^7 at margin 2^-5, the narrowed decision."""
    p = replace(params_for_bits(16), msg_bits=11, pbs_fast2_base_log=fast2[0], pbs_fast2_level=fast2[1])
    eng = Engine(p, 0)
    eng.keygen(seed)
    d = sign_digit_bits(p)
    assert d == 4
    ops = sign_round_ops(11, d, p.N)
    R = len(ops)
    sched = [2] * R
    rng = np.random.default_rng(seed)
    v_all, ph_all, bits_all = [], [], []
    for i in range(count // chunk):
        v = rng.integers(-(1 << 10), 1 << 10, chunk)
        phases, bits = _trace(eng, v, sched=sched, seed=1000 + i)
        v_all.append(v)
        ph_all.append(phases)
        bits_all.append(bits)
        torch.cuda.synchronize()
        print(f"  chunk {i + 1}/{count // chunk}", flush=True)
    eng.close()
    return p, ops, sched, np.concatenate(v_all), np.concatenate(ph_all, axis=1), np.concatenate(bits_all)


def _flip_stats(p, ops, sched, v, phases, bits):
    """Observed decision flips (censored after a ciphertext's first), their
    Gaussian prediction at the measured per-round (mean, sd) and at the model
    sigma, and the threshold bits of the ciphertexts without a flip."""
    N = p.N
    model = sign_round_sigmas(p, sched)
    alive = np.ones(len(v), bool)
    obs, lam_meas, lam_model, rows = 0, 0.0, 0.0, []
    for r, op in enumerate(ops):
        ideal = DL.ideal_index(v, op, p.msg_bits, N)
        e = DL.centred(phases[r], ideal, N).astype(np.float64)
        flip = DL.tv_decode(phases[r], op, N) != DL.tv_decode(ideal, op, N)
        ea = e[alive]
        mu, sd = float(ea.mean()), float(ea.std())
        dist = DL.boundary_distances(op, N)
        pm = DL.flip_probability(ideal[alive], op, N, mu, sd, dist)
        pmod = DL.flip_probability(ideal[alive], op, N, 0.0, model[r][2] * 2 * N, dist)
        k = int(np.sum(flip & alive))
        rows.append(dict(round=r, shift=model[r][0], sd_meas_log2=math.log2(sd / (2 * N)),
                         sd_model_log2=math.log2(model[r][2]), margin_meas=2.0 ** model[r][1] * 2 * N / sd,
                         margin_model=2.0 ** model[r][1] / model[r][2], flips=k, pred_meas=float(pm.sum()),
                         pred_model=float(pmod.sum())))
        obs += k
        lam_meas += float(pm.sum())
        lam_model += float(pmod.sum())
        alive &= ~flip
    wrong = bits != (v < 0)
    return obs, lam_meas, lam_model, rows, alive, wrong


def _check_poisson(obs, lam_meas, lam_model, tail=1e-4):
    from scipy.stats import poisson
    assert poisson.cdf(obs, lam_meas) > tail and poisson.sf(obs - 1, lam_meas) > tail, (obs, lam_meas)
    assert obs <= poisson.ppf(1 - tail, lam_model), (obs, lam_model)


@pytest.mark.parametrize("fast2,count", [((23, 1), 1 << 21), ((22, 1), 1 << 19)])
def test_flip_rate_at_narrowed_margin(need_gpu, fast2, count):
    """(b) A schedule whose narrowest decision the model puts at 4.37 sigma
    ((23,1) noise x 2^7 at a 2^-5 margin) and, for a count-rich check, 3.41
    sigma ((22,1)): the flipped decisions over >= 2 * 10^6 (resp. 2^19)
    accumulators fall in the Poisson band of the Gaussian tail at the measured
    sigma, never above the model's band, and a ciphertext whose decisions all
    held has the exact threshold bit."""
    p, ops, sched, v, phases, bits = _narrowed(fast2, count, 1 << 18, 7200 + fast2[0])
    obs, lam_meas, lam_model, rows, alive, wrong = _flip_stats(p, ops, sched, v, phases, bits)
    print(f"\nnarrowed margin, fast2 {fast2}, {count} accumulators, P = 11, schedule {sched}:")
    for t in rows:
        print(f"  round {t['round']} shift {t['shift']}: sd 2^{t['sd_meas_log2']:.3f} (model 2^{t['sd_model_log2']:.3f}), "
              f"margin {t['margin_meas']:.2f} measured / {t['margin_model']:.2f} model sigma: flips {t['flips']}, "
              f"Gaussian at measured sd {t['pred_meas']:.1f}, at model sigma {t['pred_model']:.1f}")
    print(f"  total flips {obs}: predicted {lam_meas:.1f} (measured sd), {lam_model:.1f} (model); "
          f"wrong threshold bits {int(wrong.sum())}, all of them after a flipped decision: "
          f"{bool(not np.any(wrong & alive))}")
    assert not np.any(wrong & alive)
    _check_poisson(obs, lam_meas, lam_model)
