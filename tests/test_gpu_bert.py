"""GPU: the embedding stage's encoder (include/fhe_bert.h)
against the fp32 torch BERT the reference runs (bert_embeddings.py:102-158).

The reference loads 'bert-base-uncased' by name (a download the offline image
does not have), so the check uses a randomly initialised transformers
BertModel of the same architecture (seeded; real-weight parity is unpinned)
on synthetic token ids at the reference's max_length of 100, batch 8, with
torch's fp32 forward on the host as the reference.

Tolerances, stated per arithmetic (TOL):
  f32 (default; the reference's arithmetic, f32 MFMA, another summation
  order): last hidden state relative RMS <= 1e-5 on the unpadded tokens,
  pooled max |diff| <= 2e-4, cosine >= 1 - 1e-9.
  bf16 (opt-in): about 3x the errors observed at round 3 (rel RMS 4.3e-3,
  min cosine 0.999989, pooled max |diff| 1.67e-2): rel RMS <= 1.3e-2,
  cosine >= 0.99997, pooled max |diff| <= 0.05.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

B, S = 8, 100
TOL = {"f32": {"rel_rms": 1e-5, "cos": 1 - 1e-9, "max": 2e-4},
       "bf16": {"rel_rms": 1.3e-2, "cos": 0.99997, "max": 0.05}}


@pytest.fixture(scope="module")
def model(need_gpu):
    from transformers import BertConfig, BertModel
    torch.manual_seed(1234)
    return BertModel(BertConfig(), add_pooling_layer=False).eval()


@pytest.fixture(scope="module", params=["f32", "bf16"])
def bert(request, model):
    from fheicp.bert import GpuBert
    return model, GpuBert(model=model, device=0, precision=request.param)


def _inputs(seed=0):
    g = torch.Generator().manual_seed(seed)
    ids = torch.randint(1000, 30000, (B, S), generator=g)
    ids[:, 0] = 101                                          # [CLS]
    lens = torch.randint(12, S + 1, (B,), generator=g)
    lens[0] = S
    mask = (torch.arange(S)[None, :] < lens[:, None]).to(torch.int64)
    ids[torch.arange(B), lens - 1] = 102                     # [SEP]
    ids = torch.where(mask.bool(), ids, torch.zeros_like(ids))   # [PAD] = 0
    tt = torch.zeros_like(ids)
    tt[1, 30:60] = 1                                          # a second segment in one row
    return ids, mask, tt


def _pool(hid, mask, mode):
    if mode == "mean":
        am = mask.unsqueeze(-1).to(hid.dtype)
        return (hid * am).sum(1) / am.sum(1)
    if mode == "cls":
        return hid[:, 0, :]
    return hid.max(dim=1)[0]


def test_bert_forward_vs_fp32(bert):
    m, g = bert
    tol = TOL[g.precision]
    ids, mask, tt = _inputs()
    with torch.no_grad():
        ref = m(input_ids=ids, attention_mask=mask, token_type_ids=tt).last_hidden_state.double()
    hid = g.forward(ids, mask, tt, pooling="none").cpu().double()
    valid = mask.bool()
    err = (hid - ref)[valid]
    rel_rms = float(err.pow(2).mean().sqrt() / ref[valid].pow(2).mean().sqrt())
    print(f"[{g.precision}] last_hidden_state: rel RMS {rel_rms:.3e}, max |diff| {float(err.abs().max()):.3e}")
    assert rel_rms <= tol["rel_rms"]
    for mode in ("mean", "cls", "max"):
        want = _pool(ref, mask, mode)
        got = g.forward(ids, mask, tt, pooling=mode).cpu().double()
        cos = torch.nn.functional.cosine_similarity(got, want, dim=1)
        mx = float((got - want).abs().max())
        print(f"[{g.precision}] {mode}: min cosine {float(cos.min()):.10f}, max |diff| {mx:.3e}")
        assert float(cos.min()) >= tol["cos"] and mx <= tol["max"], mode
        # the GPU's own pooling of its hidden state (fp32, same kernel inputs)
        np.testing.assert_allclose(got.numpy(), _pool(hid, mask, mode).numpy(), rtol=1e-5, atol=1e-5)


def test_precision_is_fixed_before_weights(model):
    """fhe_bert_set_precision only before the first tensor (the weights are
    stored in the selected type), and unknown precisions are refused."""
    import ctypes as C
    from fheicp import _lib
    from fheicp.bert import GpuBert
    g = GpuBert(model=model, device=0)
    assert g.precision == "f32" and g.provenance == "hip-bert-f32"
    L = _lib.lib()
    assert L.fhe_bert_get_precision(g._h) == 0
    assert L.fhe_bert_set_precision(g._h, 1) == -3          # FHE_E_STATE: weights already loaded
    with pytest.raises(ValueError):
        GpuBert(model=model, device=0, precision="fp16")
    h = C.c_void_p()
    from fheicp.bert import BertConfigC, _cfg_dict
    assert L.fhe_bert_create(C.byref(BertConfigC(**_cfg_dict(model.config))), 0, C.byref(h)) == 0
    assert L.fhe_bert_set_precision(h, 7) == -1
    assert L.fhe_bert_set_precision(h, 1) == 0 and L.fhe_bert_get_precision(h) == 1
    L.fhe_bert_destroy(h)


def test_bert_padding_invariance(bert):
    """Masked keys contribute nothing: a sequence's pooled mean embedding does
    not depend on how far its batch is padded."""
    _, g = bert
    ids, mask, tt = _inputs(1)
    short = int(mask[3].sum())
    a = g.forward(ids[3:4, :short], mask[3:4, :short], tt[3:4, :short]).cpu().numpy()
    b = g.forward(ids, mask, tt).cpu().numpy()[3:4]
    np.testing.assert_allclose(a, b, rtol=0, atol=2e-5 if g.precision == "bf16" else 2e-6)


def test_bert_embedder_mirror(bert, tmp_path):
    """fhe-icp_amd/bert_embeddings.BertEmbedder: the default is the
    reference's torch fp32 forward (no HIP encoder, provenance None);
    gpu_encoder=True runs libfheicp's encoder in the handle's precision,
    against the same class on device='cpu' with a local WordPiece
    vocabulary: same shapes, pooled embeddings within TOL."""
    from transformers import BertTokenizer
    from bert_embeddings import BertEmbedder
    m, g = bert
    words = ["the", "cat", "sat", "on", "mat", "a", "feline", "rested", "rug", "dogs", "are", "great", "pets",
             "machine", "learning", "is", "fascinating", "."]
    vf = tmp_path / "vocab.txt"
    vf.write_text("\n".join(["[PAD]", "[UNK]", "[CLS]", "[SEP]", "[MASK]"] + words) + "\n")
    tok = BertTokenizer(vocab_file=str(vf))
    texts = ["The cat sat on the mat.", "A feline rested on the rug.", "Dogs are great pets.",
             "Machine learning is fascinating.", "the cat"]
    import copy
    dflt = BertEmbedder(model=copy.deepcopy(m), tokenizer=tok, device="cuda", max_length=100)
    assert dflt.gpu is None and dflt.provenance is None
    gpu = BertEmbedder(model=m, tokenizer=tok, device="cuda", max_length=100, gpu_encoder=True,
                       gpu_precision=g.precision)
    assert gpu.provenance == f"hip-bert-{g.precision}"
    cpu = BertEmbedder(model=m, tokenizer=tok, device="cpu", max_length=100)
    tol = TOL[g.precision]["max"]
    for pooling in ("mean", "cls", "max"):
        a = gpu.get_embeddings_batch(texts, batch_size=2, pooling=pooling)
        b = cpu.get_embeddings_batch(texts, batch_size=2, pooling=pooling)
        assert a.shape == b.shape == (len(texts), 768) and a.dtype == np.float32
        assert np.abs(a - b).max() <= tol, pooling
        d = dflt.get_embeddings_batch(texts, batch_size=2, pooling=pooling)   # torch fp32 on the GPU
        assert np.abs(d - b).max() <= 2e-4, pooling
    e = gpu.get_embedding(texts[0])
    assert e.shape == (768,)
    assert abs(gpu.compute_similarity(e, cpu.get_embedding(texts[0])) - 1.0) < 5e-4
    with pytest.raises(ValueError):
        gpu.get_embedding(texts[0], pooling="median")
