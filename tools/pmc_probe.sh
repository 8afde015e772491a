#!/bin/bash
# Counter passes (each its own run) over one command, summarised per kernel:
# tools/pmc_probe.sh TAG REGEX -- CMD...  -> gpurun_out/pmc_TAG/summary.txt
# (REGEX selects the kernels of the summary; the passes: HBM bytes, L2 hit/miss,
# SQ issue/wait counters)
set -u -o pipefail
TAG=$1; RE=$2; shift 3
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out/pmc_$TAG; mkdir -p "$OUT"; cd "$R"; export TMPDIR=/tmp
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" \
           "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp -d "$OUT/p$i" -o pmc --output-format csv -- "$@" > "$OUT/p$i.log" 2>&1 || echo "pass $i ($grp) failed" >> "$OUT/summary.txt"
done
python3 - "$OUT" "$RE" >> "$OUT/summary.txt" <<'PY'
import csv, glob, sys, re, collections
d, rx = sys.argv[1], re.compile(sys.argv[2])
vals = collections.defaultdict(lambda: collections.defaultdict(list))
dur = collections.defaultdict(list)
for f in sorted(glob.glob(f"{d}/p*/**/*counter_collection.csv", recursive=True)):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0]
        if not rx.search(k):
            continue
        vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
        dur[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6)
for k, cs in vals.items():
    print(k, f"(pmc-run avg {sum(dur[k]) / len(dur[k]):.4f} ms over {len(dur[k])} records)")
    for c, v in sorted(cs.items()):
        print(f"   {c:28s} {sum(v) / len(v):.6g}   (n={len(v)})")
PY
