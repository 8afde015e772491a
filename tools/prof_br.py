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
ap.add_argument("--variants", default="4,2")
ap.add_argument("--dbg", default="", help="comma list of FHEICP_V4_DBG values to time (v4 only; wrong results)")
ap.add_argument("--gadget", default="", help="base_log,level to override the bootstrap gadget")
ap.add_argument("--lib", default="", help="load this libfheicp build instead (tools/build_variant.sh)")
ap.add_argument("--stamps", action="store_true", help="print v4 phase timestamps (FHEICP_V4_DBG=128)")
a = ap.parse_args()
import os
if a.lib:
    from fheicp import _lib
    _lib.LIB_PATH = Path(a.lib).resolve()
runs = [(v, "0") for v in a.variants.split(",")] + [("4", d) for d in a.dbg.split(",") if d]
if a.stamps:
    runs.append(("4", "128"))
for var, dbg in runs:
    os.environ["FHEICP_BR_VARIANT"] = var
    os.environ["FHEICP_V4_DBG"] = dbg
    prm = params_for_bits(a.P, fast=False)
    if a.gadget:
        from dataclasses import replace
        gb, gl = (int(x) for x in a.gadget.split(","))
        prm = replace(prm, pbs_base_log=gb, pbs_level=gl)
    eng = Engine(prm, 0)
    eng.keygen(7)
    v = np.random.default_rng(1).integers(-(2 ** (a.P - 1)), 2 ** (a.P - 1), a.B)
    ct = eng.encrypt(v, seed=3)
    eng.profile(True)
    for i in range(a.rounds):
        sm = eng.keyswitch(ct, a.P - 1 - i, 1 << 62)
        out = eng.pbs(sm, 1 << 62)
    torch.cuda.synchronize()
    # output noise of the last bootstrap: phase - nearest of +-2^62
    ph = eng.phase(out).cpu().numpy().view(np.uint64)
    err = (ph - np.uint64(1 << 62)).view(np.int64).astype(np.float64)
    err2 = (ph + np.uint64(1 << 62)).view(np.int64).astype(np.float64)
    e = np.where(np.abs(err) < np.abs(err2), err, err2)
    from fheicp.params import _variances
    print(f"gadget=({prm.pbs_base_log},{prm.pbs_level}) output noise log2 std {np.log2(e.std() / 2.0 ** 64):.2f} "
          f"(model {0.5 * np.log2(_variances(prm)[0]):.2f}) "
          f"(max |e| 2^{np.log2(np.abs(e).max() / 2.0 ** 64):.2f} of the torus)")
    br = eng.profile_read("blind_rotate")
    ks = eng.profile_read("keyswitch")
    if dbg == "128":
        import ctypes as C
        st = np.zeros(64 + 3 * 2048, np.uint64)
        eng._chk(eng._L.fhe_debug_v4_stamps(eng._ctx, C.c_void_p(st.ctypes.data)))
        names = ["start", "digits", "fwd0", "F0+mac0", "bar1", "mac0x", "bar2", "fwd1", "F1+mac1", "bar3",
                 "mac1x", "bar4", "inverse", "acc"]
        for s4 in range(4):
            row = st[s4 * 16:s4 * 16 + 14].astype(np.int64)
            d = np.diff(row)
            rt = int(st[s4 * 16 + 15]) - int(st[s4 * 16 + 14])   # s_memrealtime: 100 MHz
            clk = (row[-1] - row[0]) / (rt * 10.0) if rt > 0 else 0.0
            print("step", 100 + s4, "total", int(row[-1] - row[0]), f"realtime_ns {rt * 10} (shader clock ~{clk:.2f} GHz)",
                  " ".join(f"{n}:{int(x)}" for n, x in zip(names[1:], d)))
    if dbg == "128":
        gg = int(os.environ.get("FHEICP_V4_G", "2"))
        nwg = min(2048, (a.B + gg - 1) // gg)
        sp = st[64:64 + 3 * nwg].reshape(nwg, 3).astype(np.int64)
        t0 = sp[:, 0].min()
        start, end = (sp[:, 0] - t0) * 10, (sp[:, 1] - t0) * 10   # ns at 100 MHz
        dur = end - start
        hw = sp[:, 2]
        cu = (hw >> 8) & 0xF; sh = (hw >> 12) & 1; se = (hw >> 13) & 0x7
        print(f"workgroups {nwg}: span {end.max() / 1e6:.3f} ms (RTC @100MHz); start min/med/max "
              f"{start.min() / 1e6:.3f}/{np.median(start) / 1e6:.3f}/{start.max() / 1e6:.3f} ms; "
              f"duration min/med/max {dur.min() / 1e6:.3f}/{np.median(dur) / 1e6:.3f}/{dur.max() / 1e6:.3f} ms")
        late = int((start > 0.1 * end.max()).sum())
        print(f"  workgroups starting after 10% of the span: {late}; distinct (se, sh, cu): "
              f"{len(set(zip(se.tolist(), sh.tolist(), cu.tolist())))}")
    print(f"variant={var} dbg={dbg} G={os.environ.get('FHEICP_V4_G', '4')} A64={os.environ.get('FHEICP_V4_A64', '0')} B={a.B} blind_rotate {br['total_ms'] / br['launches']:.3f} ms/launch "
          f"({a.B * br['launches'] / br['total_ms'] * 1e3:.0f} PBS/s), keyswitch {ks['total_ms'] / ks['launches']:.3f} ms/launch")
    eng.close()
