#!/bin/bash
# round 3: the GPU suite, then the headline, C3, C4-shard and C5 bench lines
set -u -o pipefail
T=${1:-r03f}
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p "$OUT"; cd "$R"
timeout -k 10 900 python -u -m pytest tests/ -m gpu -v -s -p no:cacheprovider --timeout 400 --timeout-method thread \
  > "$OUT/${T}_tests.log" 2>&1
echo "suite rc=$?" >> "$OUT/${T}_steps.log"
timeout -k 10 300 python bench.py > "$OUT/${T}_bench.json" 2> "$OUT/${T}_bench.err" || exit 1
timeout -k 10 400 python bench.py --docs 10000 --dim 32 --n-bits 8 --steps 2 > "$OUT/${T}_c3_bench.json" 2> "$OUT/${T}_c3.err" || exit 1
timeout -k 10 400 python bench.py --docs 1000 --dim 768 --n-bits 8 --steps 2 > "$OUT/${T}_c5_bench.json" 2> "$OUT/${T}_c5.err" || exit 1
timeout -k 10 300 python bench.py --docs 12500 --dim 16 --n-bits 6 --steps 2 > "$OUT/${T}_c4_bench.json" 2> "$OUT/${T}_c4.err" || exit 1
