#!/usr/bin/env python3
"""k_encrypt_linear alone, for counter passes (tools/pmc_probe.sh): REPS
launches of B pairs x D features on the headline parameters, the tree's
own library (--repo: another worktree, for A/Bs)."""
import argparse
import sys
from pathlib import Path

ap = argparse.ArgumentParser()
ap.add_argument("--repo", default=str(Path(__file__).resolve().parents[1]))
ap.add_argument("--B", type=int, default=1024)
ap.add_argument("--D", type=int, default=16)
ap.add_argument("--reps", type=int, default=20)
a = ap.parse_args()
sys.path[:0] = [str(Path(a.repo) / "fhe-icp_amd"), a.repo]
import numpy as np  # noqa: E402
import torch  # noqa: E402
from fheicp.engine import Engine  # noqa: E402
from fheicp.params import params_for_bits  # noqa: E402

eng = Engine(params_for_bits(16), 0)
eng.keygen(7)
rng = np.random.default_rng(3)
x = eng.to_dev(rng.integers(-32, 32, (a.B, a.D)))
w = rng.integers(-127, 128, a.D)
for i in range(a.reps):
    eng.encrypt_linear(x, w, 5, seed=8, id0=i * a.B)
torch.cuda.synchronize()
print("done", a.reps, "launches of", a.B)
