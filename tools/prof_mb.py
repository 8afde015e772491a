#!/usr/bin/env python3
"""Time and noise of the fast-gadget bootstraps (fhe_pbs_gadget_batch) at the
P=21 parameter set (fast (15,2), fast2 (23,1), both multi-bit),
and A/B library builds (--lib). Prints per-launch HIP-event ms
and the output noise against the model."""
import argparse
import math
import os
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO / "fhe-icp_amd"), str(REPO)]

import numpy as np  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--B", type=int, default=1024)
ap.add_argument("--reps", type=int, default=4)
ap.add_argument("--P", type=int, default=21)
ap.add_argument("--lib", default="")
ap.add_argument("--tag", default="")
ap.add_argument("--stamps", type=int, default=-1, help="A/B build: phase timestamps of this wave (FHEICP_MB_DBG); 99: wave 0 without BSK loads")
ap.add_argument("--dbg", type=int, default=0, help="A/B build: FHEICP_MB_DBG timing variant (2 no key loads, 16 no psi "
                "gathers, 32 no F reads, 48 both, 64 no F stores, 18 no loads + no psi; wrong results)")
a = ap.parse_args()
if a.dbg:
    os.environ["FHEICP_MB_DBG"] = str(a.dbg)
if a.stamps >= 0:
    os.environ["FHEICP_MB_DBG"] = str(130 if a.stamps == 99 else 128 + 256 * a.stamps)
if a.lib:
    from fheicp import _lib
    _lib.LIB_PATH = Path(a.lib).resolve()
import torch  # noqa: E402
from fheicp.engine import Engine, u64  # noqa: E402
from fheicp.params import params_for_bits, _variances  # noqa: E402
from dataclasses import replace  # noqa: E402

prm = params_for_bits(a.P)
eng = Engine(prm, 0)
eng.keygen(7)
sgn = np.where(np.arange(a.B) % 2 == 0, 1, -1).astype(np.int64)
small = eng.keyswitch(eng.encrypt(sgn * (1 << (a.P - 3)), seed=3), 0, 0)
TV = 1 << 61
for g, name in ((1, "blind_rotate_fast"), (2, "blind_rotate_fast2")):
    lv = prm.pbs_fast_level if g == 1 else prm.pbs_fast2_level
    bl = prm.pbs_fast_base_log if g == 1 else prm.pbs_fast2_base_log
    if not lv:
        continue
    out = eng.pbs_gadget(small, g, TV)   # warm-up
    eng.profile(True)
    for _ in range(a.reps):
        out = eng.pbs_gadget(small, g, TV)
    torch.cuda.synchronize()
    eng.profile(False)
    pr = eng.profile_read(name)
    ph = u64(eng.phase(out)).view(np.int64)
    err = (ph - sgn * TV).astype(np.float64) / 2.0 ** 64
    sig = math.sqrt(float(np.mean(err ** 2)))
    model = math.sqrt(_variances(replace(prm, pbs_base_log=bl, pbs_level=lv))[0])
    print(f"{a.tag} gadget ({bl},{lv}) {eng.kernel_name(name)}: {pr['total_ms'] / max(1, pr['launches']):.3f} ms "
          f"per {a.B} ({pr['launches']} launches); sigma 2^{math.log2(sig):.2f} (classic model 2^{math.log2(model):.2f}, "
          f"ratio {sig / model:.3f}); signs ok {bool(np.all((ph > 0) == (sgn > 0)))}")
    if a.stamps >= 0:
        import ctypes as C
        st = np.zeros(64 + 3 * 2048, np.uint64)
        eng._chk(eng._L.fhe_debug_v4_stamps(eng._ctx, C.c_void_p(st.ctypes.data)))
        names = (["digits", "fwd0", "F0+ld", "bar1", "mac0"] + (["bar2", "fwd1", "F1+ld", "bar3", "mac1"] if lv > 1 else [])
                 + ["bar", "inverse"])
        idx = [0, 1, 2, 3, 4, 5] + ([6, 7, 8, 9] if lv > 1 else []) + [10, 11]
        for s4 in range(4):
            row = st[s4 * 16:s4 * 16 + 16].astype(np.int64)[idx]
            print(f"   pair {100 + s4} wave {a.stamps}: total {int(row[-1] - row[0])} cycles  " +
                  " ".join(f"{n}:{int(x)}" for n, x in zip(names, np.diff(row))))
eng.close()
