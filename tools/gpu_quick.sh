#!/bin/bash
# a quick kernel check: the noise tests (per-instance timing), the parity
# tests, then the headline bench line
set -u -o pipefail
T=${1:-quick}
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p "$OUT"; cd "$R"
timeout -k 10 600 python -u -m pytest tests/test_gpu_noise.py tests/test_gpu_parity.py -x -v -s -p no:cacheprovider \
  --timeout 300 --timeout-method thread > "$OUT/${T}_noise.log" 2>&1 || exit 1
timeout -k 10 300 python bench.py > "$OUT/${T}_bench.json" 2> "$OUT/${T}_bench.err" || exit 1
