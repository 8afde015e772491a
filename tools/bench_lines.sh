#!/bin/bash
# The bench lines of tools/closing_r05.sh alone (C2, C3, C4 shard, C5, embed),
# for a rerun on another box with the committed profiles/br_pmc.json of this
# build: tools/bench_lines.sh TAG -> gpurun_out/TAG_*.json
set -u -o pipefail
T=${1:-bench}
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p "$OUT"; cd "$R"
timeout -k 10 600 python bench.py > "$OUT/${T}_bench.json" 2> "$OUT/${T}_bench.err" || exit 1
timeout -k 10 400 python bench.py --docs 10000 --dim 32 --n-bits 8 --steps 2 > "$OUT/${T}_c3_bench.json" 2> "$OUT/${T}_c3.err" || exit 1
timeout -k 10 300 python bench.py --docs 12500 --dim 16 --n-bits 6 --steps 2 > "$OUT/${T}_c4_bench.json" 2> "$OUT/${T}_c4.err" || exit 1
timeout -k 10 400 python bench.py --docs 1000 --dim 768 --n-bits 8 --steps 2 > "$OUT/${T}_c5_bench.json" 2> "$OUT/${T}_c5.err" || exit 1
timeout -k 10 300 python bench.py --mode embed --steps 5 > "$OUT/${T}_embed_bench.json" 2> "$OUT/${T}_embed.err" || exit 1
