"""GPU: the embedding stage's PCA (fhe_pca_transform)
against a reducer fitted here with sklearn (dimension_reduction.py:67-72), and
the quantized pair features that come out of it.

The reference's transform is float32 BLAS with an unspecified summation
order, so the bar is float32 rounding: the GPU result (f64 accumulation,
rounded once to float32) is within 1 ulp of the exactly rounded f64 product
and within 1e-5 (relative to the row's norm) of sklearn's own float32 output.
BERT's weights are not available offline, so the inputs are synthetic
768-dim rows: parity against a real BERT run is unpinned.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("D", [8, 16, 128])
def test_pca_transform_vs_sklearn(need_gpu, D):
    from sklearn.decomposition import PCA
    from fheicp.pca import GpuPCA
    rng = np.random.default_rng(D)
    basis = rng.standard_normal((32, 768)).astype(np.float32)
    train = (rng.standard_normal((2000, 32)).astype(np.float32) @ basis + 0.1 * rng.standard_normal(
        (2000, 768)).astype(np.float32)).astype(np.float32)
    pca = PCA(n_components=D, random_state=42).fit(train)
    X = (rng.standard_normal((777, 32)).astype(np.float32) @ basis).astype(np.float32)
    g = GpuPCA.from_sklearn(pca, 0)
    got = g.transform(X)
    ref32 = pca.transform(X)
    assert got.dtype == np.float32 and got.shape == (777, D)
    exact = (X.astype(np.float64) - pca.mean_.astype(np.float32).astype(np.float64)) @ \
        pca.components_.astype(np.float32).astype(np.float64).T
    ulp = np.spacing(np.abs(exact).astype(np.float32))
    assert np.all(np.abs(got.astype(np.float64) - exact) <= ulp)
    scale = np.linalg.norm(exact, axis=1, keepdims=True)
    assert np.max(np.abs(got - ref32) / scale) < 1e-5
    # a single query row and the device form agree with the batch
    np.testing.assert_array_equal(g.transform(X[5]), got[5:6])
    np.testing.assert_array_equal(g.transform_dev(torch.from_numpy(X[:7]).cuda()).cpu().numpy(), got[:7])
    g.close()


def test_pca_then_encrypted_compare(need_gpu):
    """Reduced on the GPU, stored as float32, searched encrypted: the
    accumulators equal the clear restatement on those same reduced vectors."""
    from sklearn.decomposition import PCA
    from oracle import quant_ref as Q
    from fheicp.model import FheLinearModel
    from fheicp.pca import GpuPCA
    rng = np.random.default_rng(3)
    train = rng.standard_normal((1000, 768)).astype(np.float32)
    pca = PCA(n_components=16, random_state=42).fit(train)
    g = GpuPCA.from_sklearn(pca, 0)
    docs = g.transform(rng.standard_normal((300, 768)).astype(np.float32))
    q = g.transform(rng.standard_normal((1, 768)).astype(np.float32))[0]
    docs /= np.linalg.norm(docs, axis=1, keepdims=True)
    q /= np.linalg.norm(q)
    X, y = Q.prepare_training_data(16, 1000, seed=11)
    m = FheLinearModel.fit(X, y, 6)
    m.compile(key_seed=12, device=0)
    qx = m.quantize_dev(torch.from_numpy(docs).cuda(), torch.from_numpy(q).cuda())
    acc, _ = m.encrypted_acc(qx, 0)
    oq = Q.QuantizedLinearParams.from_json(m.qparams.to_dict())
    assert np.array_equal(acc.cpu().numpy(), Q.accumulate(oq, Q.quantize_input(oq, Q.pair_features(q, docs))))
    g.close()


def test_reducer_contract_at_quantizer_boundaries(need_gpu, tmp_path):
    """The contract of BatchConfig.gpu_reducer, at a quantizer rounding
    boundary (dimension_reduction.py:67-72 feeding batch_operations.py:226,
    :273): the GPU PCA and sklearn's float32 PCA differ in the last float32
    bits, and a query that puts a rounding boundary of the input quantizer
    between the two values of a feature makes the quantized inputs (hence the
    accumulator) differ. So a store reduced by one is never scored against
    vectors from the other: the processor refuses the mix, and within the GPU
    reducer every score equals the oracle on the GPU-reduced vectors."""
    from sklearn.decomposition import PCA
    from oracle import quant_ref as Q
    from batch_operations import GPU_REDUCER, REDUCER_KEY, BatchConfig, BatchProcessor
    from encrypted_storage import EncryptedDocument, EncryptedDocumentStore
    from fheicp.pca import GpuPCA
    rng = np.random.default_rng(9)
    train = rng.standard_normal((1500, 768)).astype(np.float32)
    pca = PCA(n_components=16, random_state=42).fit(train)
    g = GpuPCA.from_sklearn(pca, 0)
    X = rng.standard_normal((400, 768)).astype(np.float32)
    got, ref32 = g.transform(X), pca.transform(X).astype(np.float32)
    diff = np.argwhere(got != ref32)
    assert len(diff) > 0                                  # the reducers differ in the last bits
    i, j = map(int, diff[0])
    a, b = sorted((float(ref32[i, j]), float(got[i, j])))
    Xt, yt = Q.prepare_training_data(16, 1000, seed=11)
    qp = Q.fit_quantized_linear(Xt, yt, 6)
    # a query component that puts the quantizer boundary (k + 1/2 - zp) s between q_j a and q_j b
    k = int(np.floor(0.5 * (qp.qx_max + qp.qx_min))) + 3
    boundary = (k + 0.5 - qp.zp_x) * qp.s_x
    qj = boundary / (0.5 * (a + b))
    query = np.zeros(16, np.float64)
    query[j] = qj
    fa = Q.quantize_input(qp, Q.pair_features(query, ref32[i][None, :]))
    fb = Q.quantize_input(qp, Q.pair_features(query, got[i][None, :]))
    assert fa[0, j] != fb[0, j]                           # one quantization level apart
    # the processor: GPU-reduced documents are tagged, a CPU-reduced query is refused
    class Emb:
        def get_embedding(self, t):
            return X[int(t.split()[1])]

        def get_embeddings_batch(self, ts):
            return np.stack([self.get_embedding(t) for t in ts])
    store = EncryptedDocumentStore(str(tmp_path))
    cfg = BatchConfig(fhe="execute", input_dim=16, n_bits=6, seed=11, key_seed=12, gpu_reducer=True,
                      show_progress=False, key_manager_default=False)
    p = BatchProcessor(embedder=Emb(), reducer=g, storage=store, config=cfg)
    texts = [f"doc {r}" for r in range(64)]
    p.encrypt_documents(texts, doc_ids=[f"d{r}" for r in range(64)])
    assert all(store.index[f"d{r}"]["metadata"][REDUCER_KEY] == GPU_REDUCER for r in range(64))
    res = p.search_similar("doc 70", top_k=5, min_similarity=-100.0)
    oq = Q.QuantizedLinearParams.from_json(p.fhe_model.model.quant_params.to_dict())
    assert res == Q.search(oq, got[70], got[:64], 5, -100.0, doc_ids=[f"d{r}" for r in range(64)])
    cpu = BatchProcessor(embedder=Emb(), reducer=pca, storage=store,
                         config=BatchConfig(fhe="disable", input_dim=16, n_bits=6, seed=11, show_progress=False,
                                            key_manager_default=False))
    with pytest.raises(ValueError, match="reducers"):
        cpu.search_similar("doc 70", top_k=5, min_similarity=-100.0)
    g.close()
