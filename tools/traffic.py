#!/usr/bin/env python3
"""Per-launch HBM traffic of the blind-rotation kernel from rocprofv3 PMC csvs.

Recipe (MI355X_MICROARCH.md §HBM, cdna_hip_programming.md §7): FETCH_SIZE and
WRITE_SIZE are in KiB and must come from separate passes; on gfx950
FETCH_SIZE counts half the bytes of wide coalesced reads, so
    hbm_bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024
Usage: traffic.py <fetch_counters.csv> <write_counters.csv> [out.json]
"""
import csv
import json
import os
import sys


def per_launch(path, counter, match="k_blind_rotate"):
    rows = [r for r in csv.DictReader(open(path)) if match in r["Kernel_Name"] and r["Counter_Name"] == counter]
    if not rows:
        raise SystemExit(f"no {counter} rows for {match} in {path}")
    vals = [float(r["Counter_Value"]) for r in rows]
    names = sorted({r["Kernel_Name"].split("(")[0] for r in rows})
    return sum(vals) / len(vals), len(vals), names


def main():
    fetch, nf, names = per_launch(sys.argv[1], "FETCH_SIZE")
    write, nw, _ = per_launch(sys.argv[2], "WRITE_SIZE")
    out = {
        "kernel": ", ".join(names),
        "fetch_size_kib_raw": fetch,
        "write_size_kib": write,
        "launches": [nf, nw],
        "hbm_bytes_per_launch": (2 * fetch + write) * 1024,
        "recipe": "(2*FETCH_SIZE + WRITE_SIZE) * 1024, separate --pmc passes (gfx950 FETCH_SIZE half-count)",
    }
    # what was measured (gadget, kernel build), from $TRAFFIC_META (JSON)
    out.update(json.loads(os.environ.get("TRAFFIC_META", "{}")))
    s = json.dumps(out, indent=2)
    print(s)
    if len(sys.argv) > 3:
        open(sys.argv[3], "w").write(s + "\n")


if __name__ == "__main__":
    main()
