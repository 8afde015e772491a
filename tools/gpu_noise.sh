#!/bin/bash
# the bootstrap / key-switch noise tests (per-instance timing lines) alone
set -u -o pipefail
T=${1:-noise}
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p "$OUT"; cd "$R"
timeout -k 10 600 python -u -m pytest tests/test_gpu_noise.py -v -s -p no:cacheprovider --timeout 300 --timeout-method thread \
  > "$OUT/${T}_noise.log" 2>&1
