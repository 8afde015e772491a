#!/bin/bash
# Round-2 measurement pass after the multi-bit / key-stationary kernels:
# smoke, the PMC passes + kernel trace of the headline bench, the bench
# itself and the other configs (the GPU suite runs separately).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p "$OUT"; cd "$R"
step() { echo "== $1 $(date +%T)" >> "$OUT/steps.log"; }
step smoke; timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/r02b_smoke.log" 2>&1 || exit 1
step pmc; bash tools/pmc_bench.sh || exit 1
cp "$OUT/pmc_bench/br_pmc.json" profiles/br_pmc.json
step bench; timeout -k 10 600 python bench.py > "$OUT/r02b_bench.json" 2> "$OUT/r02b_bench.err" || exit 1
step configs; bash tools/bench_configs.sh || exit 1
step done
