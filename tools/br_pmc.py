#!/usr/bin/env python3
"""Per-kernel PMC figures of the bench's blind-rotation kernels, keyed on the
sha256 of the libfheicp.so they were measured on (bench.py reads them only
for that exact build).

Inputs: rocprofv3 counter_collection.csv files of separate --pmc passes over
`bench.py --steps 1 --warmup 0 --no-cpu-baseline` (tools/pmc_bench.sh):
  f64   SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU
  fetch FETCH_SIZE
  write WRITE_SIZE
  grbm  GRBM_GUI_ACTIVE GRBM_COUNT (the clock each kernel held)
and the kernel-trace csv of the same command for the per-launch durations.
Recipe (MI355X_MICROARCH.md, HBM/rocprofv3): SQ_INSTS_* count wave64
instructions, so f64 FLOPs = 64 x (2 FMA + ADD + MUL); FETCH_SIZE/WRITE_SIZE
are KiB from separate passes and gfx950's FETCH_SIZE counts half the bytes of
wide coalesced reads: hbm_bytes = (2 FETCH_SIZE + WRITE_SIZE) x 1024.
Entries are keyed "kernel@cts" (several configs merge into one file with
--merge); f64_flops_per_ct scales to any batch of the same kernel.
Usage: br_pmc.py --lib LIB --cts N --f64 CSV --fetch CSV --write CSV [--trace CSV] [--merge JSON] --out JSON
"""
import argparse
import collections
import csv
import hashlib
import json


def kname(s: str) -> str:
    s = s.strip()
    if s.startswith("void "):
        s = s[5:]
    return s.split("(")[0]


def per_kernel(path, match=("k_blind_rotate", "k_keyswitch", "k_encrypt_linear")):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(path)):
        n = kname(r["Kernel_Name"])
        if any(m in n for m in match):
            acc[n][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {n: {c: (sum(v) / len(v), len(v)) for c, v in cs.items()} for n, cs in acc.items()}


def grbm_clock(path, xcds=8):
    """Per kernel: GRBM_GUI_ACTIVE per dispatch (summed over the XCDs) over
    the dispatch's own duration in that pass -> the clock the kernel held,
    MHz. The counter window is a few microseconds longer than the dispatch,
    so for a kernel of tens of microseconds this is an upper bound; for the
    millisecond blind rotations it is the clock."""
    d = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != "GRBM_GUI_ACTIVE":
            continue
        n = kname(r["Kernel_Name"])
        dur_us = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3
        if dur_us > 0:
            d[n].append((float(r["Counter_Value"]), dur_us))
    out = {}
    for n, v in d.items():
        us = sum(t for _, t in v) / len(v)
        mhz = sum(g for g, _ in v) / xcds / sum(t for _, t in v)
        out[n] = {"grbm_gui_active_per_launch": sum(g for g, _ in v) / len(v), "grbm_window_us": us}
        # below a millisecond the counter window's few extra microseconds
        # dominate: kept as an upper bound only
        out[n]["clock_mhz" if us >= 1000 else "clock_mhz_upper_bound"] = mhz
    return out


def trace_ms(path):
    d = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        n = kname(r["Kernel_Name"])
        d[n].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6)
    return {n: (sum(v) / len(v), len(v)) for n, v in d.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", required=True)
    ap.add_argument("--cts", type=int, required=True, help="ciphertexts per launch of the measured command")
    ap.add_argument("--f64", required=True)
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--trace", default="")
    ap.add_argument("--grbm", default="", help="counter csv of a GRBM_GUI_ACTIVE GRBM_COUNT pass")
    ap.add_argument("--command", default="python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline")
    ap.add_argument("--out", required=True)
    ap.add_argument("--merge", default="", help="an earlier br_pmc.json of the same library to extend")
    a = ap.parse_args()
    f64, fetch, write = per_kernel(a.f64), per_kernel(a.fetch), per_kernel(a.write)
    tr = trace_ms(a.trace) if a.trace else {}
    clk = grbm_clock(a.grbm) if a.grbm else {}
    sha = hashlib.sha256(open(a.lib, "rb").read()).hexdigest()
    out = {"lib_sha256": sha, "commands": [], "kernels": {}}
    if a.merge:
        try:
            old = json.load(open(a.merge))
            if old.get("lib_sha256") == sha:
                out["commands"] = old.get("commands", [])
                out["kernels"] = old.get("kernels", {})
        except (OSError, ValueError):
            pass
    out["commands"].append({"command": a.command, "cts_per_launch": a.cts})
    # the blind-rotation kernels run whole workgroups of 4 ciphertexts, so
    # their work per launch is (f64 FLOPs per padded ciphertext) x ceil(cts/4)*4
    padded = (a.cts + 3) // 4 * 4
    for n, c in f64.items():
        fma, add, mul = (c.get(f"SQ_INSTS_VALU_{x}_F64", (0.0, 0))[0] for x in ("FMA", "ADD", "MUL"))
        flops = 64.0 * (2 * fma + add + mul)
        e = {"cts_per_launch": a.cts, "launches": c.get("SQ_INSTS_VALU_FMA_F64", (0, 0))[1],
             "f64_insts_per_launch": {"fma": fma, "add": add, "mul": mul},
             "valu_insts_per_launch": c.get("SQ_INSTS_VALU", (0.0, 0))[0],
             "f64_flops_per_launch": flops, "f64_flops_per_ct": flops / padded, "command": a.command}
        if n in fetch and n in write:
            fk, wk = fetch[n]["FETCH_SIZE"][0], write[n]["WRITE_SIZE"][0]
            e.update(fetch_size_kib=fk, write_size_kib=wk, hbm_bytes_per_launch=(2 * fk + wk) * 1024)
        if n in tr:
            e["avg_launch_ms"], e["trace_launches"] = tr[n]
        if n in clk:
            e.update({k: round(v, 1) for k, v in clk[n].items()})
        out["kernels"][f"{n}@{a.cts}"] = e
    s = json.dumps(out, indent=1)
    open(a.out, "w").write(s + "\n")
    print(s)


if __name__ == "__main__":
    main()
