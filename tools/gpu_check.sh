#!/bin/bash
# One GPU pass (tools/gpu_check.sh TAG [configs]): the whole -m gpu suite,
# the headline bench, and with "configs" the C3 / C4-shard / C5 lines;
# outputs gpurun_out/TAG_*.
set -u -o pipefail
T=${1:-r03}
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p "$OUT"; cd "$R"
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -v -s -p no:cacheprovider --timeout 400 --timeout-method thread \
  > "$OUT/${T}_tests.log" 2>&1 || exit 1
timeout -k 10 300 python bench.py > "$OUT/${T}_bench.json" 2> "$OUT/${T}_bench.err" || exit 1
if [ "${2:-}" = configs ]; then
  timeout -k 10 400 python bench.py --docs 10000 --dim 32 --n-bits 8 --steps 2 > "$OUT/${T}_c3_bench.json" 2> "$OUT/${T}_c3.err" || exit 1
  timeout -k 10 300 python bench.py --docs 12500 --dim 16 --n-bits 6 --steps 2 > "$OUT/${T}_c4_bench.json" 2> "$OUT/${T}_c4.err" || exit 1
  timeout -k 10 400 python bench.py --docs 1000 --dim 768 --n-bits 8 --steps 2 > "$OUT/${T}_c5_bench.json" 2> "$OUT/${T}_c5.err" || exit 1
fi
