#!/usr/bin/env python3
"""Generate tests/golden/*.json from the oracles (run from the repo root).

quant_golden.json — per BASELINE config (C1..C5): frozen quantized-model
parameters (seeded synthetic training, fhe_similarity.py:34-94 semantics) and
seeded q_x / accumulator / score / top-k vectors at reduced corpus sizes, plus
the one deterministic known-answer test the reference holds
(/root/reference/test_fhe.py:13-60, y = 2x, n_bits = 8, x = 7).

tfhe_golden.json — spec-conformance digests of the FHEICP-TFHE v1 streams on
the TOY parameter set: SHA-256 of the key material and of a few encryptions.

These pin the oracle against regressions; the reference itself pins nothing
at this boundary, so beyond the test_fhe.py KAT the clear
path is "parity unpinned" against a real Concrete-ML run.
"""
import hashlib
import json
import sys
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(REPO))

from oracle import quant_ref as Q  # noqa: E402

CONFIGS = {
    "C1": {"dim": 8, "n_bits": 4, "docs": 2},
    "C2": {"dim": 16, "n_bits": 6, "docs": 1024},
    "C3": {"dim": 32, "n_bits": 8, "docs": 512},
    "C4": {"dim": 16, "n_bits": 6, "docs": 512},
    "C5": {"dim": 768, "n_bits": 8, "docs": 64},
}
TOP_K = 10
MIN_SIM = 0.5


def quant_golden():
    out = {}
    for i, (name, c) in enumerate(CONFIGS.items()):
        X, y = Q.prepare_training_data(c["dim"], 1000, seed=1234 + i)
        qp = Q.fit_quantized_linear(X, y, c["n_bits"])
        q, docs = Q.make_corpus(c["dim"], c["docs"], seed=4321 + i)
        Xp = Q.pair_features(q, docs)
        qx = Q.quantize_input(qp, Xp)
        acc = Q.accumulate(qp, qx)
        scores = Q.dequantize(qp, acc)
        top = Q.search(qp, q, docs, TOP_K, MIN_SIM)
        qc, dc = Q.make_corpus(c["dim"], 16, seed=999 + i, clip_set=True)
        Xc = Q.pair_features(qc, dc)
        lo, hi = Q.acc_bounds(qp)
        out[name] = {
            "config": c, "train_seed": 1234 + i, "corpus_seed": 4321 + i, "clip_seed": 999 + i,
            "params": qp.to_json(),
            "acc_bounds": [lo, hi], "msg_bits": Q.message_bits(qp),
            "threshold_T": Q.threshold_int(qp, MIN_SIM, lo, hi),
            "query": [float(v) for v in q], "docs_head": [[float(v) for v in row] for row in docs[:4]],
            "qx_head": qx[:4].tolist(), "acc": acc.tolist(), "scores": [float(s) for s in scores],
            "topk": [[int(i_), float(s)] for i_, s in top],
            "clip_qx": Q.quantize_input(qp, Xc).tolist(),
            "clip_acc": Q.accumulate(qp, Q.quantize_input(qp, Xc)).tolist(),
        }
    # reference KAT: /root/reference/test_fhe.py:13-60
    Xk = np.array([[1], [2], [3], [4], [5], [6]], dtype=np.float32)
    yk = np.array([2, 4, 6, 8, 10, 12], dtype=np.float32)
    qk = Q.fit_quantized_linear(Xk, yk, 8)
    xk = np.array([[7]], dtype=np.float32)
    out["KAT_test_fhe"] = {
        "source": "/root/reference/test_fhe.py:13-60 (y=2x, n_bits=8, predict x=7)",
        "params": qk.to_json(),
        "q_x": Q.quantize_input(qk, xk).tolist(),
        "acc": Q.accumulate(qk, Q.quantize_input(qk, xk)).tolist(),
        "score": float(Q.predict(qk, xk)[0]),
        "note": "7 lies above the calibration max 6 and clips to q=127; the reference prints 'Expected 14.0' "
                "but only asserts |clear - FHE| < 0.01, so this value is the restatement's, unverified "
                "against a real Concrete-ML run",
    }
    return out


def sha(a) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def tfhe_golden():
    from oracle import tfhe_ref as R
    sys.path.insert(0, str(REPO / "fhe-icp_amd"))
    from fheicp.params import TOY
    R.build()
    ref = R.RefTFHE(TOY.as_dict(), 1234)
    v = np.arange(-8, 8, dtype=np.int64)
    ct = ref.encrypt_ints(v, seed=99, id0=1000)
    return {
        "params": TOY.as_dict(), "key_seed": 1234, "enc_seed": 99, "id0": 1000, "messages": v.tolist(),
        "sha256_s_small": sha(ref.s_small), "sha256_s_big": sha(ref.s_big),
        "sha256_bsk": sha(ref.bsk), "sha256_ksk": sha(ref.ksk), "sha256_ct": sha(ct),
        "ct0_head": [int(x) for x in ct[0, :4]], "ct0_body": int(ct[0, -1]),
    }


if __name__ == "__main__":
    g = REPO / "tests" / "golden"
    (g / "quant_golden.json").write_text(json.dumps(quant_golden()))
    (g / "tfhe_golden.json").write_text(json.dumps(tfhe_golden(), indent=1))
    print("wrote", g / "quant_golden.json", g / "tfhe_golden.json")
