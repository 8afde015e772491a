#!/bin/bash
# round 3: BERT tests, noise tests (mb64 timing), the GPU suite, headline + embed bench
set -u -o pipefail
T=${1:-r03d}
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p "$OUT"; cd "$R"
timeout -k 10 600 python -u -m pytest tests/test_gpu_bert.py -x -v -s -p no:cacheprovider --timeout 300 --timeout-method thread \
  > "$OUT/${T}_bert_tests.log" 2>&1
echo "bert rc=$?" >> "$OUT/${T}_steps.log"
timeout -k 10 900 python -u -m pytest tests/ -m gpu -v -s -p no:cacheprovider --timeout 400 --timeout-method thread \
  --deselect tests/test_gpu_bert.py > "$OUT/${T}_tests.log" 2>&1
echo "suite rc=$?" >> "$OUT/${T}_steps.log"
timeout -k 10 300 python bench.py > "$OUT/${T}_bench.json" 2> "$OUT/${T}_bench.err" || exit 1
timeout -k 10 300 python bench.py --mode embed --steps 5 > "$OUT/${T}_embed_bench.json" 2> "$OUT/${T}_embed.err" || exit 1
