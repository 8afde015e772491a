"""Key-switch split sweep (A/B build only: tools/build_variant.sh ksab
-DFHEICP_KS_AB, FHEICP_LIB pointing at it): time fhe_keyswitch_batch on
batches of the headline parameter set for each forced K split S, and check
that every split gives the same output. Not part of the product.

  FHEICP_LIB=$PWD/fhe-icp_amd/fheicp/libfheicp_ksab.so python tools/ks_sweep.py
"""
import os
import sys
from pathlib import Path

import numpy as np
import torch

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO / "fhe-icp_amd"))


def main():
    from fheicp.engine import Engine
    from fheicp.params import params_for_bits
    eng = Engine(params_for_bits(16), 0)
    eng.keygen(5)
    for B in (1024, 6144):
        v = np.random.default_rng(B).integers(-(2 ** 15), 2 ** 15, B)
        ct = eng.encrypt(v, seed=9)
        ref = None
        for S in ("auto", 1, 2, 3, 4, 6, 8, 12):
            if S == "auto":
                os.environ.pop("FHEICP_KS_S", None)
            else:
                os.environ["FHEICP_KS_S"] = str(S)
            out = eng.keyswitch(ct, 2, 1 << 61)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(50):
                out = eng.keyswitch(ct, 2, 1 << 61)
            e1.record()
            torch.cuda.synchronize()
            same = True if ref is None else bool(torch.equal(out, ref))
            ref = out if ref is None else ref
            print(f"B={B} S={S}: {e0.elapsed_time(e1) / 50 * 1e3:.1f} us per key switch, equal={same}", flush=True)


if __name__ == "__main__":
    main()
