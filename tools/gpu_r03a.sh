#!/bin/bash
# round 3, first GPU pass: the new -m gpu tests, then the headline bench
set -u -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p "$OUT"; cd "$R"
timeout -k 10 700 python -u -m pytest -x -v -p no:cacheprovider --timeout 400 --timeout-method thread \
  tests/test_gpu_sharded.py tests/test_gpu_dropin.py tests/test_gpu_noise.py -k "sharded or dropin or gadget4 or gadget5" \
  > "$OUT/r03a_tests.log" 2>&1 || exit 1
timeout -k 10 300 python bench.py > "$OUT/r03a_bench.json" 2> "$OUT/r03a_bench.err" || exit 1
