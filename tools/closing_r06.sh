#!/bin/bash
# Closing pass on one GPU, in parts that each fit one gpurun call
# (tools/closing_r06.sh TAG PART, outputs gpurun_out/TAG_*, copied to
# profiles/ by hand):
#   tests  the whole -m gpu suite and smoke();
#   pmc    the PMC passes of the headline, C3 (one stream), C5 and the table
#          bootstrap (tools/pmc_r03.sh: br_pmc.json keyed on this build's
#          sha256, every record with the clock its kernel held; installed as
#          profiles/br_pmc.json for the bench lines), then the bench lines of
#          C2 (headline), C3, C4 (one shard), C5 and --mode lut;
#   extra  the corpus line, the embedding stage in f32 (default) and bf16,
#          the SQ counters of the headline kernels, a 2-rank gloo run of the
#          N > 1 (C4, 100k docs) path started the driver's way without a
#          launcher, and the rocprofv3 kernel summary of the f32 embed line.
set -u -o pipefail
T=${1:-r06end}; PART=${2:-tests}
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p "$OUT"; cd "$R"
step() { echo "== $1 $(date +%T)" >> "$OUT/${T}_steps.log"; }
if [ "$PART" = tests ]; then
  step tests; timeout -k 10 1000 python -u -m pytest tests/ -m gpu -v -p no:cacheprovider --timeout 400 --timeout-method thread > "$OUT/${T}_tests.log" 2>&1 || exit 1
  step smoke; timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/${T}_smoke.log" 2>&1 || exit 1
elif [ "$PART" = pmc ]; then
  step pmc; bash tools/pmc_r03.sh > "$OUT/${T}_pmc.log" 2>&1 || exit 1
  cp "$OUT/pmc_r03/br_pmc.json" profiles/br_pmc.json
  step bench; timeout -k 10 600 python bench.py > "$OUT/${T}_bench.json" 2> "$OUT/${T}_bench.err" || exit 1
  step c3; timeout -k 10 400 python bench.py --docs 10000 --dim 32 --n-bits 8 --steps 2 > "$OUT/${T}_c3_bench.json" 2> "$OUT/${T}_c3.err" || exit 1
  step c4; timeout -k 10 300 python bench.py --docs 12500 --dim 16 --n-bits 6 --steps 2 > "$OUT/${T}_c4_bench.json" 2> "$OUT/${T}_c4.err" || exit 1
  step c5; timeout -k 10 400 python bench.py --docs 1000 --dim 768 --n-bits 8 --steps 4 > "$OUT/${T}_c5_bench.json" 2> "$OUT/${T}_c5.err" || exit 1
  step lut; timeout -k 10 300 python bench.py --mode lut --steps 20 --warmup 3 > "$OUT/${T}_lut_bench.json" 2> "$OUT/${T}_lut.err" || exit 1
elif [ "$PART" = extra ]; then
  step corpus; timeout -k 10 300 python bench.py --mode corpus --steps 5 > "$OUT/${T}_corpus_bench.json" 2> "$OUT/${T}_corpus.err" || exit 1
  step embed; timeout -k 10 300 python bench.py --mode embed --steps 5 > "$OUT/${T}_embed_bench.json" 2> "$OUT/${T}_embed.err" || exit 1
  step embed_bf16; timeout -k 10 300 python bench.py --mode embed --embed-precision bf16 --steps 5 > "$OUT/${T}_embed_bf16_bench.json" 2> "$OUT/${T}_embed_bf16.err" || exit 1
  step sq; TAG=_$T bash tools/pmc_sq.sh > /dev/null || exit 1
  step n2; FHEICP_DIST_BACKEND=gloo timeout -k 10 500 python bench.py --gpus 2 --steps 2 --warmup 1 > "$OUT/${T}_n2.json" 2> "$OUT/${T}_n2.err" || exit 1
  cd /tmp && export TMPDIR=/tmp && cd "$R"
  step prof_embed; timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/${T}_prof_embed" -o run --output-format csv -- python3 bench.py --mode embed --steps 3 --no-cpu-baseline > "$OUT/${T}_prof_embed.log" 2>&1 || exit 1
fi
step "done $PART"
