"""GPU: edge cases of the compare path that the reference's search loop meets
(batch_operations.py:268-284), on the C2 model of the golden fixture
(tests/golden/quant_golden.json, 16-dim, n_bits=6, P = 16):

- an empty batch and ragged batches that leave a workgroup's four ciphertext
  slots part-filled (the `c < count` guards of k_blind_rotate_v4 / _mb) or a
  last workgroup of the key switch partial: accumulators and threshold bits
  equal the fixture's prefix, whatever the batch size;
- thresholds at both ends of the accumulator range (every document below, none
  below): the sign extraction's decision at the edges of the P-bit width;
- top_k larger than the documents kept, top_k = 0, and top_k over a batch
  where nothing passes: the (score desc, index asc) order of the reference's
  stable sort, padded with index -1.
"""
import json
from pathlib import Path

import numpy as np
import pytest
import torch

from oracle import quant_ref as Q

pytestmark = pytest.mark.gpu

GOLD = json.loads((Path(__file__).parent / "golden" / "quant_golden.json").read_text())
MIN_SIM = 0.5


@pytest.fixture(scope="module")
def c2(need_gpu):
    from fheicp.model import FheLinearModel, QuantParams
    g = GOLD["C2"]
    m = FheLinearModel(QuantParams.from_dict(g["params"]))
    m.compile(key_seed=202, device=0)
    q, docs = Q.make_corpus(g["config"]["dim"], g["config"]["docs"], seed=g["corpus_seed"])
    dev = m.engine.device
    qx = m.quantize_dev(torch.from_numpy(docs).to(dev), torch.from_numpy(q).to(dev))
    yield m, g, qx
    m.engine.close()


def _ref_topk(acc, below, k, scale):
    """batch_operations.py:278-284: keep score >= t, stable sort desc, slice."""
    keep = [(i, float(scale * np.float64(a))) for i, (a, b) in enumerate(zip(acc, below)) if not b]
    keep.sort(key=lambda x: x[1], reverse=True)
    return keep[:k]


@pytest.mark.parametrize("B", [0, 1, 3, 5, 7, 63, 65, 257])
def test_ragged_batches_equal_golden_prefix(c2, B):
    from fheicp.model import threshold_int
    m, g, qx = c2
    T = threshold_int(m.qparams, MIN_SIM)
    acc, below = m.encrypted_acc(qx[:B].contiguous(), T)
    assert tuple(acc.shape) == (B,) and tuple(below.shape) == (B,)
    want = np.asarray(g["acc"][:B], dtype=np.int64)
    assert np.array_equal(acc.cpu().numpy(), want)
    assert np.array_equal(below.cpu().numpy(), (want < T).astype(np.int64))


def test_threshold_at_both_ends_of_the_range(c2):
    m, g, qx = c2
    lo, hi = m.qparams.acc_range()
    want = np.asarray(g["acc"][:129], dtype=np.int64)
    sub = qx[:129].contiguous()
    # T = hi + 1: every accumulator is below; T = lo: none is
    acc, below = m.encrypted_acc(sub, hi + 1)
    assert np.array_equal(acc.cpu().numpy(), want)
    assert below.cpu().numpy().tolist() == [1] * 129
    acc, below = m.encrypted_acc(sub, lo)
    assert np.array_equal(acc.cpu().numpy(), want)
    assert below.cpu().numpy().tolist() == [0] * 129
    # T at the smallest and largest accumulator of the batch: the decision
    # flips exactly there
    for T in (int(want.min()), int(want.max()), int(want.max()) + 1):
        _, below = m.encrypted_acc(sub, T)
        assert np.array_equal(below.cpu().numpy(), (want < T).astype(np.int64))


@pytest.mark.parametrize("B,k", [(3, 10), (5, 0), (65, 64), (257, 300), (1024, 1024)])
def test_topk_sizes(c2, B, k):
    from fheicp.model import threshold_int
    m, g, qx = c2
    T = threshold_int(m.qparams, MIN_SIM)
    acc, below = m.encrypted_acc(qx[:B].contiguous(), T)
    oa, oi = m.engine.topk(acc, below, k)
    assert tuple(oi.shape) == (k,)
    s = np.float64(m.qparams.out_scale)
    ref = _ref_topk(acc.cpu().tolist(), below.cpu().tolist(), k, s)
    ia, ii = oa.cpu().tolist(), oi.cpu().tolist()
    got = [(int(i), float(s * np.float64(a))) for a, i in zip(ia, ii) if i >= 0]
    assert got == ref
    # the entries past the kept documents are padding
    assert all(i == -1 for i in ii[len(ref):])
    # and the ranking equals the fixture's where the fixture's top-10 applies
    if B == 1024 and k >= 10:
        assert [(i, sc) for i, sc in got[:10]] == [(int(i), float(sc)) for i, sc in g["topk"]]


def test_topk_nothing_passes(c2):
    m, g, qx = c2
    lo, hi = m.qparams.acc_range()
    acc, below = m.encrypted_acc(qx[:100].contiguous(), hi + 1)
    oa, oi = m.engine.topk(acc, below, 10)
    assert oi.cpu().tolist() == [-1] * 10
