#!/usr/bin/env python3
"""Average per-dispatch counter values of the blind-rotation kernel from
gpurun_out/pmc*/pmc_counter_collection.csv (tools/pmc_br.sh)."""
import csv
import glob
import sys

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
match = sys.argv[2] if len(sys.argv) > 2 else "blind_rotate"
vals = {}
for f in sorted(glob.glob(f"{d}/pmc*/pmc_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        if match in r["Kernel_Name"]:
            vals.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
for k, v in vals.items():
    print(f"{k:28s} {sum(v) / len(v):.4g}  (n={len(v)})")
