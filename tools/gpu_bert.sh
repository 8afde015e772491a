#!/bin/bash
# the BERT encoder: tolerance tests, then the embed bench line
set -u -o pipefail
T=${1:-bert}
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p "$OUT"; cd "$R"
timeout -k 10 300 python -u -m pytest tests/test_gpu_bert.py -x -v -s -p no:cacheprovider --timeout 200 --timeout-method thread \
  > "$OUT/${T}_bert_tests.log" 2>&1 || exit 1
timeout -k 10 300 python bench.py --mode embed --steps 5 > "$OUT/${T}_embed_bench.json" 2> "$OUT/${T}_embed.err" || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$R"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/${T}_prof" -o run --output-format csv -- python3 bench.py --mode embed --steps 3 > "$OUT/${T}_prof.log" 2>&1 || exit 1
