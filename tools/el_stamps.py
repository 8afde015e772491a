#!/usr/bin/env python3
"""Phase timing of k_encrypt_linear in an A/B build (tools/build_variant.sh
stamps -DFHEICP_AB): 1024 pairs x D features, per wave index the median
s_memtime spans of mask generation, noise blocks, barrier wait, MAC loop and
epilogue, and the workgroups' start / end spread on s_memrealtime (100 MHz).
Usage: python tools/el_stamps.py --lib fhe-icp_amd/fheicp/libfheicp_stamps.so"""
import argparse
import ctypes as C
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO / "fhe-icp_amd"), str(REPO)]

import numpy as np  # noqa: E402
import torch  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--lib", required=True)
ap.add_argument("--B", type=int, default=1024)
ap.add_argument("--D", type=int, default=16)
ap.add_argument("--reps", type=int, default=20)
a = ap.parse_args()
from fheicp import _lib  # noqa: E402
_lib.LIB_PATH = Path(a.lib).resolve()
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
st = np.zeros(1024 * 4 * 10, np.uint64)
eng._chk(eng._L.fhe_debug_el_stamps(eng._ctx, C.c_void_p(st.ctypes.data)))
st = st.reshape(1024, 4, 10).astype(np.int64)[:min(a.B, 1024)]
names = ["mask", "noise", "barrier", "mac", "epilogue"]
print(f"B={a.B} D={a.D}: median s_memtime cycles per phase (last launch)")
for wv in range(4):
    d = np.diff(st[:, wv, 1:7], axis=1)
    print(f"  wave {wv}: " + "  ".join(f"{n} {int(np.median(d[:, i]))}" for i, n in enumerate(names)),
          f" total {int(np.median(st[:, wv, 6] - st[:, wv, 1]))}")
t0 = st[:, :, 0].min()
start = (st[:, 0, 0] - t0) * 10.0  # ns
end = (st[:, :, 7].max(axis=1) - t0) * 10.0
print(f"  workgroup start (ns from first): p0 {np.percentile(start, 0):.0f} p50 {np.percentile(start, 50):.0f} "
      f"p90 {np.percentile(start, 90):.0f} max {start.max():.0f}")
print(f"  workgroup end   (ns from first start): p10 {np.percentile(end, 10):.0f} p50 {np.percentile(end, 50):.0f} "
      f"max {end.max():.0f}")
dur = end - start
print(f"  workgroup duration ns: p10 {np.percentile(dur, 10):.0f} p50 {np.percentile(dur, 50):.0f} max {dur.max():.0f}")
hist = np.histogram(start, bins=8)
print("  start histogram:", hist[0].tolist(), "edges ns", [int(e) for e in hist[1]])
cyc = st[:, :, 6] - st[:, :, 1]
print(f"  wave cycles start->end: p10 {np.percentile(cyc, 10):.0f} p50 {np.percentile(cyc, 50):.0f} max {cyc.max():.0f}")
# placement: HW_ID bits wave 3:0, simd 5:4, cu 11:8, sh 12, se 15:13 (gfx9 layout); XCC_ID low 4 bits
hw, xcc = st[:, :, 8], st[:, :, 9] & 15
simd = (hw >> 4) & 3
cu = (xcc << 8) | (((hw >> 13) & 7) << 5) | (((hw >> 12) & 1) << 4) | ((hw >> 8) & 15)
keys = cu * 4 + simd
uniq, counts = np.unique(keys, return_counts=True)
occ = dict(zip(uniq.tolist(), counts.tolist()))
print(f"  distinct CUs {len(np.unique(cu))}, SIMDs {len(uniq)}; waves per SIMD histogram",
      dict(zip(*np.unique(counts, return_counts=True))))
wg_cu = cu[:, 0]
_, per_cu = np.unique(wg_cu, return_counts=True)
print("  workgroups per CU histogram", dict(zip(*np.unique(per_cu, return_counts=True))))
wmax = np.array([max(occ[int(k)] for k in keys[i]) for i in range(len(keys))])
for m in sorted(set(wmax.tolist())):
    sel = wmax == m
    print(f"  workgroups whose busiest SIMD holds {m} waves: {sel.sum()}, median cycles {np.median(cyc[sel].max(axis=1)):.0f}, "
          f"median ns {np.median(dur[sel]):.0f}")
print("  per-XCC median ns:", {int(x): int(np.median(dur[xcc[:, 0] == x])) for x in np.unique(xcc[:, 0])})
print("  SIMD of wave index w (rows) histogram over workgroups:")
for wv in range(4):
    print(f"    wave {wv}:", dict(zip(*[x.tolist() for x in np.unique(simd[:, wv], return_counts=True)])))
print("  first CUs: workgroup -> (simd, slot) of waves 0..3")
for c in np.unique(wg_cu)[:6]:
    rows = np.nonzero(wg_cu == c)[0]
    print(f"    cu {int(c):5d}:", "; ".join(f"b{int(b)} " + ",".join(f"{int(simd[b, w])}/{int(hw[b, w] & 15)}" for w in range(4))
                                     for b in rows))
