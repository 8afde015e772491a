#!/bin/bash
# SQ stall / issue counters of the blind-rotation kernels over one headline
# bench step (two --pmc passes, each its own run) and a per-kernel summary:
# gpurun_out/pmc_sq/summary.txt. $LIB (optional) = an A/B build to load.
set -u -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out/pmc_sq${TAG:-}; mkdir -p "$OUT"; cd "$R"; export TMPDIR=/tmp
CMD="$R/bench.py --steps 1 --warmup 0 --no-cpu-baseline ${BENCH_ARGS:-}"
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -s KILL 180 rocprofv3 --pmc $grp -d "$OUT/p$i" -o pmc --output-format csv -- python3 $CMD > "$OUT/p$i.log" 2>&1 || { echo "pass $i failed"; exit 1; }
done
python3 - "$OUT" > "$OUT/summary.txt" <<'PY'
import csv, glob, sys, collections
d = sys.argv[1]
vals = collections.defaultdict(lambda: collections.defaultdict(list))
dur = collections.defaultdict(list)
for f in sorted(glob.glob(f"{d}/p*/**/*counter_collection.csv", recursive=True)):
    for r in csv.DictReader(open(f)):
        if "blind_rotate" in r["Kernel_Name"]:
            k = r["Kernel_Name"].split("(")[0]
            vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
            dur[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6)
for k, cs in vals.items():
    m = {c: sum(v) / len(v) for c, v in cs.items()}
    print(k, f"(pmc-run ms ~{sum(dur[k]) / len(dur[k]):.3f})")
    for c, v in sorted(m.items()):
        print(f"   {c:24s} {v:.5g}")
    w = m.get("SQ_WAVES", 0)
    if w and m.get("SQ_WAVE_CYCLES"):
        wc = m["SQ_WAVE_CYCLES"]
        print(f"   wait_any/wave_cycles {m.get('SQ_WAIT_ANY', 0) / wc:.3f}  active_valu/wave_cycles {m.get('SQ_ACTIVE_INST_VALU', 0) / wc:.3f}"
              f"  active_lds/wave_cycles {m.get('SQ_ACTIVE_INST_LDS', 0) / wc:.3f}  valu insts/wave {m.get('SQ_INSTS_VALU', 0) / w:.0f}")
    if m.get("GRBM_GUI_ACTIVE"):
        ms = sum(dur[k]) / len(dur[k])
        print(f"   GRBM_GUI_ACTIVE/ms = {m['GRBM_GUI_ACTIVE'] / ms / 1e3:.0f} MHz (if per-kernel)")
PY
cat "$OUT/summary.txt"
