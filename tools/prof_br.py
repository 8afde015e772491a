#!/usr/bin/env python3
"""Profiling driver: keygen once, then R rounds of (key switch + blind
rotation) over B ciphertexts at the production parameter set. Used under
rocprofv3 (kernel trace / PMC passes); prints per-launch HIP-event timings."""
import argparse
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO / "fhe-icp_amd"), str(REPO)]

import numpy as np  # noqa: E402
import torch  # noqa: E402
from fheicp.engine import Engine  # noqa: E402
from fheicp.params import params_for_bits  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--B", type=int, default=1024)
ap.add_argument("--rounds", type=int, default=2)
ap.add_argument("--P", type=int, default=16)
ap.add_argument("--variants", default="2,3")
a = ap.parse_args()
import os
for var in a.variants.split(","):
    os.environ["FHEICP_BR_VARIANT"] = var
    eng = Engine(params_for_bits(a.P), 0)
    eng.keygen(7)
    v = np.random.default_rng(1).integers(-(2 ** (a.P - 1)), 2 ** (a.P - 1), a.B)
    ct = eng.encrypt(v, seed=3)
    eng.profile(True)
    for i in range(a.rounds):
        sm = eng.keyswitch(ct, a.P - 1 - i, 1 << 62)
        out = eng.pbs(sm, 1 << 62)
    torch.cuda.synchronize()
    br = eng.profile_read("blind_rotate")
    ks = eng.profile_read("keyswitch")
    print(f"variant={var} B={a.B} blind_rotate {br['total_ms'] / br['launches']:.3f} ms/launch "
          f"({a.B * br['launches'] / br['total_ms'] * 1e3:.0f} PBS/s), keyswitch {ks['total_ms'] / ks['launches']:.3f} ms/launch")
    eng.close()
