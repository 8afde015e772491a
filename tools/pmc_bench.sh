#!/bin/bash
# PMC passes over the headline bench command (one per counter group, each its
# own run, as the gfx950 recipe requires) and the per-kernel summary bench.py
# reads: gpurun_out/pmc_bench/br_pmc.json (copy it to profiles/br_pmc.json).
# Extra bench.py arguments (another config) go in $BENCH_ARGS; $CTS is the
# ciphertexts per launch (the documents per GPU of that run); a run for another
# config merges into the same file (entries keyed kernel@cts); $PMC_ENV names
# an environment prefix of the command in the record (e.g. "FHEICP_PIPE=0 ").
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=${PMC_OUT:-$R/gpurun_out/pmc_bench}; mkdir -p "$OUT"; cd "$R"; export TMPDIR=/tmp
rm -rf "$OUT/f64" "$OUT/fetch" "$OUT/write" "$OUT/grbm" "$OUT/trace"   # csvof reads the first file of each pass
CMD="$R/bench.py --steps 1 --warmup 0 --no-cpu-baseline ${BENCH_ARGS:-}"
csvof() { ls "$1"/*counter_collection.csv "$1"/*/*counter_collection.csv 2>/dev/null | head -n1; }
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU \
  -d "$OUT/f64" -o pmc --output-format csv -- python3 $CMD > "$OUT/f64.log" 2>&1 || exit 1
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d "$OUT/fetch" -o pmc --output-format csv -- python3 $CMD > "$OUT/fetch.log" 2>&1 || exit 1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d "$OUT/write" -o pmc --output-format csv -- python3 $CMD > "$OUT/write.log" 2>&1 || exit 1
# the clock the kernels hold (GRBM_GUI_ACTIVE over each dispatch, summed over the 8 XCDs)
timeout -s KILL 300 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT -d "$OUT/grbm" -o pmc --output-format csv -- python3 $CMD > "$OUT/grbm.log" 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} > "$OUT/trace.log" 2>&1 || exit 1
python3 tools/br_pmc.py --lib fhe-icp_amd/fheicp/libfheicp.so --cts "${CTS:-1024}" --f64 "$(csvof "$OUT/f64")" \
  --fetch "$(csvof "$OUT/fetch")" --write "$(csvof "$OUT/write")" --grbm "$(csvof "$OUT/grbm")" \
  --trace "$(ls "$OUT"/trace/*kernel_trace.csv "$OUT"/trace/*/*kernel_trace.csv 2>/dev/null | head -n1)" \
  --command "${PMC_ENV:-}python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline ${BENCH_ARGS:-}" \
  --merge "${PMC_MERGE:-$OUT/br_pmc.json}" --out "$OUT/br_pmc.json" > "$OUT/br_pmc.log" 2>&1
