#!/bin/bash
# Round-2 GPU pass: the whole -m gpu suite (incl. the per-config and noise
# tests), smoke, the PMC passes of the headline bench, the bench itself.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p "$OUT"; cd "$R"
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -s > "$OUT/r02_tests.log" 2>&1 || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/r02_smoke.log" 2>&1 || exit 1
bash tools/pmc_bench.sh || exit 1
cp "$OUT/pmc_bench/br_pmc.json" profiles/br_pmc.json
timeout -k 10 600 python bench.py > "$OUT/r02_bench.json" 2> "$OUT/r02_bench.err" || exit 1
bash tools/bench_configs.sh || exit 1
