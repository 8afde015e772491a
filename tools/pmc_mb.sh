#!/bin/bash
# Counter passes over tools/prof_mb.py (fast-gadget bootstraps, P=21 set),
# classic (FHEICP_MB=0) and multi-bit (FHEICP_MB=1).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out/pmc_mb; mkdir -p "$OUT"; cd "$R"; export TMPDIR=/tmp
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM_WR"; do
  i=$((i+1))
  for mb in 0 1; do
    FHEICP_MB=$mb timeout -k 10 120 rocprofv3 --pmc $grp -d "$OUT/mb${mb}_pmc$i" -o pmc --output-format csv -- python3 "$R/tools/prof_mb.py" --reps 1 > "$OUT/mb${mb}_pmc$i.log" 2>&1 || { echo "pmc$i mb$mb failed"; exit 1; }
  done
done
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
d = sys.argv[1]
for mb in (0, 1):
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in sorted(glob.glob(f"{d}/mb{mb}_pmc*/**/*counter_collection.csv", recursive=True)):
        for r in csv.DictReader(open(f)):
            if "blind_rotate" in r["Kernel_Name"]:
                k = r["Kernel_Name"].split("(")[0]
                vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, cs in vals.items():
        print(f"mb={mb} {k}")
        for c, v in sorted(cs.items()):
            print(f"   {c:24s} {sum(v)/len(v):.4g}")
PY
