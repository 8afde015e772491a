#!/bin/bash
# Closing pass on one GPU (tools/closing_pass.sh TAG, outputs gpurun_out/TAG_*,
# copied to profiles/ by hand): the whole -m gpu suite, smoke, the PMC
# passes + kernel trace of the headline bench (profiles/br_pmc.json keyed on
# this build's sha256), the bench itself, the other configs, the SQ counters
# and a 2-rank gloo rehearsal of the N > 1 (C4, 100k docs) path.
set -u -o pipefail
T=${1:-r02f}
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p "$OUT"; cd "$R"
step() { echo "== $1 $(date +%T)" >> "$OUT/steps.log"; }
step tests; timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > "$OUT/${T}_tests.log" 2>&1 || exit 1
step smoke; timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/${T}_smoke.log" 2>&1 || exit 1
step pmc; bash tools/pmc_bench.sh || exit 1
cp "$OUT/pmc_bench/br_pmc.json" profiles/br_pmc.json
step bench; timeout -k 10 600 python bench.py > "$OUT/${T}_bench.json" 2> "$OUT/${T}_bench.err" || exit 1
step configs; bash tools/bench_configs.sh || exit 1
step sq; bash tools/pmc_sq.sh > /dev/null || exit 1
step n2; FHEICP_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 2 --warmup 1 > "$OUT/${T}_n2.json" 2> "$OUT/${T}_n2.err" || exit 1
step done
