#!/bin/bash
# FETCH_SIZE and WRITE_SIZE passes (separate, per the gfx950 recipe) over the
# bench's blind-rotation geometry; writes gpurun_out/br_traffic.json.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p "$OUT"; cd "$R"; export TMPDIR=/tmp
V=${VARIANTS:-2}
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc_fetch" -o pmc --output-format csv -- python3 "$R/tools/prof_br.py" --rounds 2 --variants "$V" > "$OUT/pmc_fetch.log" 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc_write" -o pmc --output-format csv -- python3 "$R/tools/prof_br.py" --rounds 2 --variants "$V" > "$OUT/pmc_write.log" 2>&1 || exit 1
python3 tools/traffic.py "$(ls "$OUT"/pmc_fetch/*counter_collection.csv "$OUT"/pmc_fetch/*/*counter_collection.csv 2>/dev/null | head -n1)" \
  "$(ls "$OUT"/pmc_write/*counter_collection.csv "$OUT"/pmc_write/*/*counter_collection.csv 2>/dev/null | head -n1)" "$OUT/br_traffic.json"
