"""CPU: parameter selection / noise model, and the sharded search merge over a
2-rank gloo group (the N > 1 path of bench.py and search, without a GPU)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from fheicp.params import (PBS_GADGETS, TOY, params_for_bits, noise_report, sign_digit_bits, sign_pbs_count,
                           sign_plan, sign_precise_rounds, sign_rounds, sign_schedule)
from fheicp.search import sharded_topk


@pytest.mark.parametrize("pmax,beta,lvl", PBS_GADGETS)
def test_gadget_table_has_margin(pmax, beta, lvl):
    from fheicp.params import SchemeParams, _cheapest_plan
    # the table's gadget with its cheapest fast / mid gadgets (params_for_bits
    # may still pick the next, more precise main gadget when that is cheaper)
    p = _cheapest_plan(SchemeParams(pbs_base_log=beta, pbs_level=lvl, msg_bits=pmax))
    assert params_for_bits(pmax).pbs_level in (lvl, lvl + 1)
    # >= 9.2 sigma at the decision margin  <=>  p_fail <= 2^-64 per PBS, for
    # the digit sign extraction (1/16 margin) and the single-bit one (1/4)
    for method in ("digits", "bits"):
        r = noise_report(p, method)
        assert r["margin_sigmas"] > 9.2, (method, r)
        assert r["log2_pfail_per_pbs"] < -64
    # and the next width up would not be (the table is tight)
    if pmax < 27:
        assert noise_report(p.with_msg_bits(pmax + 1))["margin_sigmas"] < 9.2


def _param_sets():
    for P in range(2, 28):
        for fast in (True, False):
            p = params_for_bits(P, fast=fast)
            if fast and p.pbs_fast2_level:   # also the two-gadget variant
                q = p.__class__(**{**p.as_dict(), "pbs_fast2_base_log": 0, "pbs_fast2_level": 0})
                for d in (0, 3, 4):
                    yield q.__class__(**{**q.as_dict(), "sign_digit_bits": d})
            for d in (0, 3, 4):
                yield p.with_msg_bits(P).__class__(**{**p.as_dict(), "sign_digit_bits": d})
            if fast and p.pbs_fast_level:   # the same gadgets on the classic rotation
                yield p.__class__(**{**p.as_dict(), "pbs_fast_group": 1, "pbs_fast2_group": 1})
    for P in range(2, 17):
        yield TOY.with_msg_bits(P)


def test_sign_digits_match_oracle_and_library(oracle_lib):
    """Digit width and PBS count: params.py, the C library (host-only call) and
    the oracle restatement resolve every parameter set identically."""
    from fheicp import _lib
    L = _lib.lib()
    for p in _param_sets():
        d = p.as_dict()
        cp = _lib.params_struct(d)
        assert sign_digit_bits(p) == oracle_lib.sign_digit_bits(d) == L.fhe_sign_digit_bits(cp), d
        assert sign_pbs_count(p) == oracle_lib.sign_pbs_count(d) == L.fhe_sign_pbs_count(cp), d
        assert sign_precise_rounds(p) == oracle_lib.sign_precise_rounds(d) == L.fhe_sign_precise_rounds(cp), d
        import ctypes as C
        dd, j1, j2 = C.c_int32(), C.c_int32(), C.c_int32()
        assert L.fhe_sign_plan(cp, C.byref(dd), C.byref(j1), C.byref(j2)) == 0
        assert sign_plan(p) == oracle_lib.sign_plan(d) == (dd.value, j1.value, j2.value), d
        sched = (C.c_int32 * 64)()
        R = L.fhe_sign_schedule(cp, sched, 64)
        assert sign_schedule(p)[1] == oracle_lib.sign_schedule(d) == list(sched[:R]), d
    # 4-bit digits at the configs' widths (with the (3, 5) key switch, C5's
    # P = 26 too; it took 3-bit digits with the (4, 4) one)
    assert [sign_digit_bits(params_for_bits(P)) for P in (16, 17, 21, 26)] == [4, 4, 4, 4]
    assert sign_pbs_count(16) == 7
    assert noise_report(params_for_bits(16))["digit_bits"] == 4


def test_fast_gadget_plan():
    """Per-round gadgets: params_for_bits adds the
    cheapest set of fast gadgets (by BR_COST, classic or multi-bit rotation)
    for the sign rounds whose noise is barely amplified; only the leading
    rounds, whose output is shifted up the most, stay on the precise gadget,
    and every round keeps 9.2 sigma with the fewest main, then fast, rounds."""
    from fheicp.params import _plan_worst, plan_cost
    F, F2 = (15, 2, 2), (23, 1, 2)
    # (round 4: the multi-bit rounds' modulus switch rounds each pair's active
    # exponent once, 3/4 of the classic variance, so P = 9 now runs on (23,1)
    # alone and P = 13 needs two (15,2) rounds instead of three)
    want = {4: (F2, None, (4, 0, 1)), 8: (F2, None, (4, 0, 3)), 9: (F2, None, (4, 0, 4)), 12: (F, F2, (4, 0, 1)),
            13: (F, F2, (4, 0, 2)), 16: (F, F2, (4, 0, 3))}
    for P, (fg, fg2, (d, j1, j2)) in want.items():
        p = params_for_bits(P)
        assert p.pbs_mid_level == 0, P
        assert (p.pbs_fast_base_log, p.pbs_fast_level, p.pbs_fast_group) == fg, P
        got2 = (p.pbs_fast2_base_log, p.pbs_fast2_level, p.pbs_fast2_group) if p.pbs_fast2_level else None
        assert got2 == fg2, P
        R = len(sign_rounds(P, d))
        assert sign_plan(p) == (d, j1, j2 if fg2 else R), P
        assert _plan_worst(p, d, j1, j2) >= 9.2
        assert j1 == 0 or _plan_worst(p, d, j1 - 1, R) < 9.2
        assert fg2 is None or j2 == j1 or _plan_worst(p, d, j1, j2 - 1) < 9.2
        assert R == sign_pbs_count(p)
        assert plan_cost(p) < plan_cost(params_for_bits(P, fast=False))
    # the headline width keeps its 4-bit digits, with no bootstrap on the
    # classic (15,2) gadget since the (3, 5) key switch: three on its
    # multi-bit form, four on multi-bit (23,1)
    assert sign_plan(params_for_bits(16)) == (4, 0, 3)
    assert sign_plan(params_for_bits(19, fast=False)) == (4, 9, 9)
    # from P = 17 a mid gadget joins (test_mid_gadget_plan)
    assert params_for_bits(17).pbs_mid_level
    assert params_for_bits(3).pbs_fast_level == 0


def test_mid_gadget_plan():
    """Mid gadgets: from P = 17 the plan adds one or two
    gadgets between the main and the fast one, on the multi-bit rotation with
    48-bit accumulators (k_blind_rotate_mb64), 0.72-0.78x the classic time at
    the same gadget (BR_COST, measured). The schedule walks main -> mid -> mid2
    -> fast -> fast2, each gadget on the fewest rounds for which the next one
    on all the rest keeps every decision at 9.2 sigma, and the plan is cheaper
    than the same gadgets without mids. A multi-bit mid at the main gadget's
    own level takes the first round wherever its (3x key) noise allows."""
    from dataclasses import replace
    from fheicp.params import _sched_worst, plan_cost, sign_schedule
    M3, M4, M5, M6 = (12, 3, 2), (10, 4, 2), (8, 5, 2), (7, 6, 2)
    want = {17: (M3, None), 19: (M3, None), 20: (M4, None), 21: (M4, M3), 22: (M5, M3), 23: (M5, M3),
            24: (M6, M4), 25: (M4, M3), 26: (M5, M3), 27: (M6, M4)}
    for P, (m1, m2) in want.items():
        p = params_for_bits(P)
        assert (p.pbs_mid_base_log, p.pbs_mid_level, p.pbs_mid_group) == m1, P
        got2 = (p.pbs_mid2_base_log, p.pbs_mid2_level, p.pbs_mid2_group) if p.pbs_mid2_level else None
        assert got2 == m2, P
        d, sched = sign_schedule(p)
        assert len(sched) == sign_pbs_count(p) and _sched_worst(p, d, sched) >= 9.2, P
        lad = [g for g in (0, 5, 3, 4, 1, 2) if g in sched]
        assert sched == sorted(sched, key=lad.index), P   # ladder order
        for i in range(len(lad) - 1):                      # each gadget on its fewest rounds
            c = sched.index(lad[i + 1])
            start = sched.index(lad[i])
            if c > start:
                fewer = sched[:c - 1] + [lad[i + 1]] * (len(sched) - c + 1)
                assert _sched_worst(p, d, fewer) < 9.2, (P, i)
        nomid = replace(p, pbs_mid_base_log=0, pbs_mid_level=0, pbs_mid2_base_log=0, pbs_mid2_level=0,
                        pbs_mid_group=0, pbs_mid2_group=0, pbs_mid0_base_log=0, pbs_mid0_level=0,
                        pbs_mid0_group=0)
        assert plan_cost(p) < plan_cost(nomid), P
        classic = replace(p, pbs_mid_group=0, pbs_mid2_group=0, pbs_mid0_group=0)
        assert plan_cost(p) < plan_cost(classic), P
    # C5's width: the first round on the mid0 gadget, multi-bit (5,8) (the
    # classic main (6,7) key is made, never launched; 2.6 % cheaper than
    # that round on it), 2 mid (8,5) and 2 mid2 (12,3) multi-bit, 4 fast,
    # 4 fast2; P = 25 the same with a (6,7) mid0
    p26 = params_for_bits(26)
    assert (p26.pbs_base_log, p26.pbs_level, p26.pbs_mid_base_log, p26.pbs_mid_level,
            p26.pbs_mid2_base_log, p26.pbs_mid2_level) == (6, 7, 8, 5, 12, 3)
    assert (p26.pbs_mid0_base_log, p26.pbs_mid0_level, p26.pbs_mid0_group) == (5, 8, 2)
    assert sign_schedule(p26)[1] == [5, 3, 3, 4, 4] + [1] * 4 + [2] * 4
    assert plan_cost(p26) < 0.975 * plan_cost(replace(p26, pbs_mid0_base_log=0, pbs_mid0_level=0,
                                                      pbs_mid0_group=0))
    p25 = params_for_bits(25)
    assert (p25.pbs_mid0_base_log, p25.pbs_mid0_level, p25.pbs_mid0_group) == (6, 7, 2)
    assert sign_schedule(p25)[1][0] == 5
    # mid0 is added only where it makes the plan cheaper: no width below 25
    assert not any(params_for_bits(P).pbs_mid0_level for P in range(2, 25))
    # the headline width runs every round on the multi-bit fast gadgets: the
    # main (15, 2) key is made but never launched
    assert sign_schedule(params_for_bits(16))[1] == [1, 1, 1, 2, 2, 2, 2]
    # the headline width has no mid gadget; C3's (P = 21) takes the (10,4)
    # gadget, whose quieter first bootstrap allows 4-bit digits (10 bootstraps
    # instead of 13), on the multi-bit rotation for its first round (the
    # classic (10,4) main key is made, never launched), then 2 x mb (12,3),
    # 3 x mb (15,2) and 4 x mb (23,1) (4 and 3 before round 4)
    assert params_for_bits(16).pbs_mid_level == 0
    p21 = params_for_bits(21)
    assert (p21.pbs_base_log, p21.pbs_level) == (10, 4)
    assert sign_schedule(p21) == (4, [3, 4, 4, 1, 1, 1, 2, 2, 2, 2])


def test_multibit_modswitch_variance():
    """The multi-bit modulus switch (DESIGN.md §4.5, pbs1_mb / mb_rotate): the
    phase error of a rotation by the active subset's exponent, each exponent
    switched from its exact sum, simulated over random masks and binary keys
    at the real n = 887, 2N = 2048: its variance matches params._ms_var
    (group 2, 3/4 of the classic one per pair) within 3%, and the classic
    per-coefficient rounding matches group 1."""
    from fheicp.params import _ms_var, params_for_bits
    p = params_for_bits(16)
    rng = np.random.default_rng(5)
    T, n, twoN = 4000, p.n, 2 * p.N
    A = rng.integers(0, 2 ** 63, (T, n + 1), dtype=np.uint64) * np.uint64(2) + rng.integers(0, 2, (T, n + 1)).astype(np.uint64)
    s = rng.integers(0, 2, (T, n)).astype(np.int64)

    def sw(x):  # round(x 2N / 2^64) mod 2N, and the rounding error in units of the torus
        r = ((x >> np.uint64(52)) + np.uint64(1)) >> np.uint64(1)
        err = (r.astype(np.float64) - x.astype(np.float64) * twoN / 2.0 ** 64)
        return r % twoN, (err + twoN / 2) % twoN - twoN / 2

    _, eb = sw(A[:, n])
    _, e = sw(A[:, :n])
    classic = eb - (e * s).sum(1)
    m = n // 2
    a1, a2 = A[:, 0:2 * m:2], A[:, 1:2 * m:2]
    s1, s2 = s[:, 0:2 * m:2], s[:, 1:2 * m:2]
    _, e1 = sw(a1)
    _, e2 = sw(a2)
    with np.errstate(over="ignore"):
        _, e12 = sw(a1 + a2)
    pair = np.where((s1 == 1) & (s2 == 1), e12, np.where(s1 == 1, e1, np.where(s2 == 1, e2, 0.0)))
    lone = e[:, n - 1] * s[:, n - 1] if n % 2 else 0.0
    mb = eb - pair.sum(1) - lone
    v1, v2 = classic.var() / twoN ** 2, mb.var() / twoN ** 2
    assert abs(v1 / _ms_var(p, 1) - 1) < 0.05, v1 / _ms_var(p, 1)
    assert abs(v2 / _ms_var(p, 2) - 1) < 0.05, v2 / _ms_var(p, 2)
    assert 0.7 < _ms_var(p, 2) / _ms_var(p, 1) < 0.8


def test_multibit_noise_model():
    """The multi-bit term of the noise model (group 2) is the same formula in
    params.py, the C library and the oracle (through the plans they resolve),
    and its factors: 3x key noise, 3x FFT error, half the 2^32 roundings."""
    from dataclasses import replace
    from fheicp.params import SchemeParams, _variances
    for b, lv in ((15, 2), (23, 1)):
        p = SchemeParams(pbs_base_log=b, pbs_level=lv)
        v1, v2 = _variances(p)[0], _variances(p, group=2)[0]
        assert 1.05 < v2 / v1 < 1.8, (b, lv, v2 / v1)
    # a plan whose fast gadget flips to classic when the group changes differs
    q = params_for_bits(20)
    assert q.pbs_fast_group == 2 and q.pbs_fast2_group == 2
    assert sign_schedule(replace(q, pbs_fast_group=1, pbs_fast2_group=1))[1] != sign_schedule(q)[1]


def test_sign_digit_bits_validation():
    with pytest.raises(ValueError):
        sign_digit_bits(params_for_bits(16).__class__(sign_digit_bits=5))


def test_params_for_bits_limits():
    assert params_for_bits(11).pbs_level == 2
    assert params_for_bits(21, fast=False).pbs_level == 3   # the table's gadget
    assert params_for_bits(21).pbs_level == 4               # the cheaper plan's main gadget
    with pytest.raises(ValueError):
        params_for_bits(28)


def cpu_topk(acc, below, k, base_idx):
    """Reference top-k for the test: Python stable sort, (acc desc, idx asc)."""
    a = acc.tolist()
    b = below.tolist() if below is not None else [0] * len(a)
    keep = [(i, a[i]) for i in range(len(a)) if not b[i]]
    keep.sort(key=lambda x: x[1], reverse=True)
    keep = keep[:k]
    oa = torch.full((k,), -(2 ** 63), dtype=torch.int64)
    oi = torch.full((k,), -1, dtype=torch.int64)
    for j, (i, v) in enumerate(keep):
        oa[j] = v
        oi[j] = i + base_idx
    return oa, oi


def _worker(rank, world, port, acc_all, below_all, k, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.distributed.init_process_group("gloo", rank=rank, world_size=world)
    n = len(acc_all) // world
    acc = torch.tensor(acc_all[rank * n:(rank + 1) * n])
    below = torch.tensor(below_all[rank * n:(rank + 1) * n])
    oa, oi = sharded_topk(acc, below, k, rank * n, cpu_topk, world)
    q.put((rank, oa.tolist(), oi.tolist()))
    torch.distributed.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("world,k", [(2, 10), (2, 37), (4, 5)])
def test_sharded_topk_equals_global(world, k):
    rng = np.random.default_rng(world * 100 + k)
    n = 64 * world
    acc_all = rng.integers(-15, 15, n).tolist()          # many ties across shards
    below_all = (rng.random(n) < 0.4).astype(np.int64).tolist()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, acc_all, below_all, k, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = [q.get(timeout=120) for _ in ps]
    for p in ps:
        p.join(timeout=60)
    ga, gi = cpu_topk(torch.tensor(acc_all), torch.tensor(below_all), k, 0)
    for _, oa, oi in res:
        assert oa == ga.tolist() and oi == gi.tolist()


def _proc_worker(rank, world, port, store_dir, query, cases, q):
    import sys as _s
    from pathlib import Path as _P
    root = _P(__file__).resolve().parents[1]
    for p in (str(root / "fhe-icp_amd"), str(root)):
        if p not in _s.path:
            _s.path.insert(0, p)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.distributed.init_process_group("gloo", rank=rank, world_size=world)
    from batch_operations import BatchConfig, BatchProcessor
    from encrypted_storage import EncryptedDocumentStore
    cfg = BatchConfig(fhe="disable", input_dim=16, n_bits=6, seed=21, show_progress=False,
                      key_manager_default=False)
    p = BatchProcessor(storage=EncryptedDocumentStore(store_dir), config=cfg)
    res = [p.search_vector(np.asarray(query), k, t) for k, t in cases]
    q.put((rank, res, p.fhe_model.model.quant_params.to_dict()))
    torch.distributed.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_processor_sharded_search_gloo(tmp_path, monkeypatch, world):
    """BatchProcessor.search_vector under torch.distributed (gloo, 2 and 3
    ranks, a ragged 301-document store with duplicated documents): each rank
    scores its contiguous range, one all-gather merges the top-k, and every
    rank returns batch_operations.py:268-284's result (float >=, stable sort
    desc, slice), restated by the oracle over the whole store."""
    from encrypted_storage import EncryptedDocument, EncryptedDocumentStore
    from oracle import quant_ref as Q
    monkeypatch.setattr(EncryptedDocument, "allowed_dims", (16, 128, 256))
    qv, docs = Q.make_corpus(16, 301, seed=77)
    docs[5] = docs[200]
    docs[150] = docs[151]                       # ties across the rank boundary
    store = EncryptedDocumentStore(str(tmp_path))
    ids = [f"d{i:03d}" for i in range(len(docs))]
    store.save_many([EncryptedDocument(doc_id=ids[i], content_hash=f"{i:064x}", timestamp="2025-01-01T00:00:00",
                                       encrypted_embedding=docs[i], metadata={}) for i in range(len(docs))])
    cases = [(10, 0.5), (400, -100.0), (3, 100.0), (1, 0.0)]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_proc_worker, args=(r, world, port, str(tmp_path), qv.tolist(), cases, q))
          for r in range(world)]
    for p in ps:
        p.start()
    res = [q.get(timeout=180) for _ in ps]
    for p in ps:
        p.join(timeout=60)
    qp = Q.QuantizedLinearParams.from_json(res[0][2])
    for _, got, qd in res:
        assert qd == res[0][2]
        for (k, t), g in zip(cases, got):
            want = [(ids[i], s) for i, s in Q.search(qp, qv, docs, k, t)]
            assert g == want, (k, t)


@pytest.mark.parametrize("beta,lvl", [(12, 3), (10, 4), (8, 5), (7, 6), (6, 7), (5, 8)])
def test_offset_digits_equal_sequential(beta, lvl):
    """The deep v4s kernels re-extract each level's digit as
    ((r' >> i beta) & (B - 1)) - B/2 from r' = r + sum_i (B/2) B^i, r the
    rounded top L*beta bits; the other kernels and the oracle use the
    sequential balanced decomposition (sign-extend beta bits, subtract,
    next). Both are the digit representation of r mod B^L in [-B/2, B/2), so
    they agree on every input: checked here on random words, near-ties and
    the top of the range (numpy uint64, mod-2^64 like the kernels)."""
    rng = np.random.default_rng(beta * 10 + lvl)
    x = rng.integers(0, 2 ** 63, 200_000, dtype=np.uint64) * np.uint64(2) + rng.integers(0, 2, 200_000, dtype=np.uint64)
    prec = lvl * beta
    x[:2000] = (np.arange(2000, dtype=np.uint64) << np.uint64(64 - prec - 1))   # rounding ties
    x[2000:4000] = np.uint64(2 ** 64 - 1) - np.arange(2000, dtype=np.uint64)
    r = ((x >> np.uint64(63 - prec)) + np.uint64(1)) >> np.uint64(1)
    B = np.uint64(1 << beta)
    seq = np.zeros((lvl, x.size), np.int64)
    rr = r.copy()
    for i in range(lvl):
        low = ((rr >> np.uint64(i * beta)) & (B - np.uint64(1))).astype(np.int64)
        d = np.where(low >= (1 << (beta - 1)), low - (1 << beta), low)
        seq[lvl - 1 - i] = d
        rr = rr - (d.astype(np.uint64) << np.uint64(i * beta))      # mod 2^64
    coff = np.uint64(sum(1 << (i * beta + beta - 1) for i in range(lvl)))
    rp = r + coff
    for lv in range(lvl):
        off = ((rp >> np.uint64((lvl - 1 - lv) * beta)) & (B - np.uint64(1))).astype(np.int64) - (1 << (beta - 1))
        assert np.array_equal(off, seq[lv]), (beta, lvl, lv)


def test_two_word_torus_rounding_equals_split():
    """The 64-bit-accumulator kernels (br_v4.h Acc<false>::from_f64) read
    round(z 2^64) mod 2^64 as h 2^32 + rint(r 2^32), h = rint(F) and r = F - h
    for F = (z - rint(z)) 2^32, with both roundings done by adding 1.5 2^52
    and reading mantissa bits; wave_fft.h f64_to_torus (the form it replaces)
    splits round(v) mod 2^64 through floor. Restated in numpy on random
    magnitudes, exact ties and tiny values: the two agree bit for bit."""
    rng = np.random.default_rng(7)
    z = rng.standard_normal(300_000) * np.exp2(rng.integers(-70, 40, 300_000))
    z[:1000] = (np.arange(1000) - 500 + 0.5) * 2.0 ** -64             # ties at 2^-64
    z[1000:2000] = (np.arange(1000) - 500 + 0.5) * 2.0 ** -20
    z[2000:2010] = [0.0, -0.0, 0.5, -0.5, 1.5, -2.5, 2.0 ** 30, -(2.0 ** 30), 2.0 ** 60, 2.0 ** -1074]
    M = 6755399441055744.0
    bits = lambda a: a.view(np.uint64)
    F = np.ldexp(z - np.rint(z), 32)
    t1 = F + M
    t2 = np.ldexp(F - (t1 - M), 32) + M
    new = ((bits(t1) & np.uint64(0xFFFFFFFF)) << np.uint64(32)) + (bits(t2) - np.uint64(0x4338000000000000))
    v = np.ldexp(z, 64)                                               # f64_to_torus(v)
    m = np.rint(v * 2.0 ** -64)
    r = np.rint(v - m * 2.0 ** 64)        # exact for these |v| (numpy has no fma; m 2^64 is exact)
    hi = np.floor(r * 2.0 ** -32)
    lo = r - hi * 2.0 ** 32
    hu = np.where(hi >= 2.0 ** 31, hi - 2.0 ** 32, hi).astype(np.int64).astype(np.uint64) & np.uint64(0xFFFFFFFF)
    old = (hu << np.uint64(32)) + lo.astype(np.uint64)
    assert np.array_equal(new, old)


@pytest.mark.parametrize("P", [3, 5, 11, 15, 16, 21, 26])
def test_sign_round_ops_clear_simulation(P):
    """fheicp.params.sign_round_ops (the bookkeeping the decision-noise GPU
    test measures against) run in the clear on exact phases: every round's
    exact exponent is the centre of its slot on the 2N grid, the test vector
    read there clears exactly the bits the next round assumes cleared, and the
    last round's output is [v < 0]; the shifts and margins are sign_rounds'."""
    import sys
    sys.path.insert(0, str(__import__("pathlib").Path(__file__).resolve().parent))
    import decision_noise_lib as DL
    from fheicp.params import sign_round_ops
    p = params_for_bits(P)
    d = sign_digit_bits(p)
    N = p.N
    ops = sign_round_ops(P, d, N)
    if P >= 4:
        assert [(o["shift"]) for o in ops] == [sh for sh, _ in sign_rounds(P, d)]
    assert len(ops) == sign_pbs_count(p)
    rng = np.random.default_rng(P)
    v = np.arange(-(1 << (P - 1)), 1 << (P - 1), dtype=np.int64) if P <= 16 else \
        rng.integers(-(1 << (P - 1)), 1 << (P - 1), 200000)
    delta = np.uint64(1 << (64 - P))
    M = v.view(np.uint64) * delta
    sign = None
    for r, op in enumerate(ops):
        with np.errstate(over="ignore"):
            assert np.array_equal(M, DL.v_cur(v, op).view(np.uint64) * delta), r
        ideal = DL.ideal_index(v, op, P, N)
        x = DL.tv_decode(ideal, op, N)
        base = np.uint64(op["tv"][0])
        with np.errstate(over="ignore"):
            dlt = base - x if op["mode"] == 1 else x
            M = M - dlt
        if r == len(ops) - 1:
            sign = dlt
        # the margin: the nearest slot boundary is 2^(ml) of the torus away
        if P >= 4:
            ml = sign_rounds(P, d)[r][1]
            d_lo, d_hi = DL.boundary_distances(op, N)
            assert min(d_lo[ideal].min(), d_hi[ideal].min()) == (2 * N) >> (-ml)
    assert np.array_equal(sign >> np.uint64(63), (v < 0).astype(np.uint64))
