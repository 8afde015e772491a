"""Soak run of the headline path (not part of the product; a measurement):
--steps batches of --docs fresh documents (16-dim, n_bits = 6: C2 / C4's
parameter set, 7 bootstraps per compare), each batch encrypted with fresh
session randomness, its accumulators and threshold bits compared with the
clear restatement of the reference path (oracle/quant_ref.py: fit, quantize,
accumulate; batch_operations.py:226, :278). Prints one progress line per
batch and a JSON summary: the count of wrong accumulators and wrong
threshold bits over all compares (the exactness evidence at
scale, beside the per-round decision-noise tests).

  python tools/soak.py --docs 100000 --steps 100
"""
import argparse
import json
import sys
import time
from pathlib import Path

import numpy as np
import torch

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))
sys.path.insert(0, str(REPO / "fhe-icp_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--docs", type=int, default=100_000)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--dim", type=int, default=16)
    ap.add_argument("--n-bits", type=int, default=6)
    ap.add_argument("--min-similarity", type=float, default=0.5)
    ap.add_argument("--seed", type=int, default=4321)
    ap.add_argument("--out", default="")
    args = ap.parse_args()

    from fheicp import _lib
    from fheicp.datagen import corpus, training_pairs
    from fheicp.model import FheLinearModel, threshold_int
    from fheicp.params import sign_pbs_count
    from oracle import quant_ref as Q

    _lib.lib()
    X, y = training_pairs(args.dim, 1000, seed=args.seed + 1)
    model = FheLinearModel.fit(X, y, n_bits=args.n_bits)
    model.compile(key_seed=args.seed, device=0)
    oq = Q.fit_quantized_linear(X, y, args.n_bits)
    assert oq.to_json() == model.qparams.to_dict()
    T = threshold_int(model.qparams, args.min_similarity)
    n_pbs = sign_pbs_count(model.engine.params)
    dev = torch.device("cuda", 0)

    tot = bad_acc = bad_bit = near = 0
    t0 = time.perf_counter()
    for s in range(args.steps):
        q, docs = corpus(args.dim, args.docs, seed=args.seed + 1000 + s, query_seed=args.seed + 999 - s)
        qx = model.quantize_dev(torch.from_numpy(docs).to(dev), torch.from_numpy(q).to(dev))
        acc, below = model.encrypted_acc(qx, T)
        acc_ref = Q.accumulate(oq, Q.quantize_input(oq, Q.pair_features(q, docs)))
        bit_ref = (Q.dequantize(oq, acc_ref) < args.min_similarity).astype(np.int64)
        a, b = acc.cpu().numpy(), below.cpu().numpy()
        bad_acc += int((a != acc_ref).sum())
        bad_bit += int((b != bit_ref).sum())
        near += int((np.abs(acc_ref - T) <= 16).sum())
        tot += len(acc_ref)
        print(f"step {s + 1}/{args.steps}: {tot} compares, {bad_acc} wrong accumulators, {bad_bit} wrong "
              f"threshold bits, {time.perf_counter() - t0:.1f} s", flush=True)
    out = {"compares": tot, "bootstraps": tot * n_pbs, "pbs_per_compare": n_pbs, "wrong_accumulators": bad_acc,
           "wrong_threshold_bits": bad_bit, "compares_within_16_of_threshold": near, "steps": args.steps,
           "docs_per_step": args.docs, "dim": args.dim, "n_bits": args.n_bits, "msg_bits_P": model.msg_bits,
           "seconds": round(time.perf_counter() - t0, 1),
           "note": "each step: fresh documents and fresh encryption randomness; accumulators decrypted from the "
                   "leveled circuit, threshold bits from the exact sign extraction"}
    line = json.dumps(out)
    print(line)
    if args.out:
        Path(args.out).write_text(line + "\n")
    return 0 if bad_acc == 0 and bad_bit == 0 else 1


if __name__ == "__main__":
    sys.exit(main())
