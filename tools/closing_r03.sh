#!/bin/bash
# Closing pass on one GPU (tools/closing_r03.sh TAG (r03end the last), outputs gpurun_out/TAG_*,
# copied to profiles/ by hand): the whole -m gpu suite, smoke, the PMC passes
# of the headline, C3 (one stream) and C5 (tools/pmc_r03.sh; br_pmc.json keyed
# on this build's sha256, installed for the bench lines that follow), the
# bench lines of C2 (headline), C3, C4 (one shard), C5 and the embedding
# stage, the SQ counters of the headline and C5 kernels, and a 2-rank gloo
# rehearsal of the N > 1 (C4, 100k docs) path.
set -u -o pipefail
T=${1:-r03end}
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p "$OUT"; cd "$R"
step() { echo "== $1 $(date +%T)" >> "$OUT/${T}_steps.log"; }
step tests; timeout -k 10 900 python -u -m pytest tests/ -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread > "$OUT/${T}_tests.log" 2>&1 || exit 1
step smoke; timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/${T}_smoke.log" 2>&1 || exit 1
step pmc; bash tools/pmc_r03.sh > "$OUT/${T}_pmc.log" 2>&1 || exit 1
cp "$OUT/pmc_r03/br_pmc.json" profiles/br_pmc.json
step bench; timeout -k 10 600 python bench.py > "$OUT/${T}_bench.json" 2> "$OUT/${T}_bench.err" || exit 1
step c3; timeout -k 10 400 python bench.py --docs 10000 --dim 32 --n-bits 8 --steps 2 > "$OUT/${T}_c3_bench.json" 2> "$OUT/${T}_c3.err" || exit 1
step c4; timeout -k 10 300 python bench.py --docs 12500 --dim 16 --n-bits 6 --steps 2 > "$OUT/${T}_c4_bench.json" 2> "$OUT/${T}_c4.err" || exit 1
step c5; timeout -k 10 400 python bench.py --docs 1000 --dim 768 --n-bits 8 --steps 2 > "$OUT/${T}_c5_bench.json" 2> "$OUT/${T}_c5.err" || exit 1
step embed; timeout -k 10 300 python bench.py --mode embed --steps 5 > "$OUT/${T}_embed_bench.json" 2> "$OUT/${T}_embed.err" || exit 1
step sq; bash tools/pmc_sq.sh > /dev/null || exit 1
step sq_c5; TAG=_c5 BENCH_ARGS="--docs 1000 --dim 768 --n-bits 8" bash tools/pmc_sq.sh > /dev/null || exit 1
step n2; FHEICP_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 2 --warmup 1 > "$OUT/${T}_n2.json" 2> "$OUT/${T}_n2.err" || exit 1
step done
