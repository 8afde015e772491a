#!/bin/bash
# L1 (TCP) and L2 (TCC) passes over the blind rotation: how much of the BSK
# stream the vector L1 serves and what reaches L2 (one counter block per pass).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p "$OUT"; cd "$R"; export TMPDIR=/tmp
V=${VARIANTS:-4}
i=0
for grp in "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $grp -d "$OUT/pmc_cache$i" -o pmc --output-format csv -- python3 "$R/tools/prof_br.py" --rounds 1 --variants "$V" > "$OUT/pmc_cache$i.log" 2>&1 || { echo "cache$i failed"; exit 1; }
done
