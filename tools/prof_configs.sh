#!/bin/bash
# Kernel trace (rocprofv3 --kernel-trace --stats) of the C5 and C3 bench lines,
# so the deep v4s kernels' HIP-event averages in the JSON line can be checked
# against rocprof's: gpurun_out/prof_cfg/{c5,c3}/run_kernel_stats.csv + .json.
set -u -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out/prof_cfg; mkdir -p "$OUT"; cd "$R"; export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/c5" -o run --output-format csv -- python3 "$R/bench.py" \
  --docs 1000 --dim 768 --n-bits 8 --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/c5.json" 2> "$OUT/c5.err" || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/c3" -o run --output-format csv -- python3 "$R/bench.py" \
  --docs 10000 --dim 32 --n-bits 8 --steps 1 --warmup 1 --no-cpu-baseline > "$OUT/c3.json" 2> "$OUT/c3.err" || exit 1
