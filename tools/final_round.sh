#!/bin/bash
# Round-end measurement on one GPU: PMC traffic of the dominant blind-rotation
# kernel (so bench.py can report it), parity tests, smoke, the headline bench,
# its rocprofv3 kernel trace, the other configs, the corpus mode and a 2-rank
# gloo rehearsal of the N > 1 path. Every GPU step has its own time limit and
# the script stops at the first failure.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p "$OUT"; cd "$R"
step() { local name=$1; shift; echo "== $name" >> "$OUT/steps.log"; "$@"; local rc=$?; echo "== $name rc=$rc" >> "$OUT/steps.log"; return $rc; }
export TRAFFIC_META='{"pbs_level": 2, "pbs_base_log": 15, "cts_per_launch": 1024, "kernel_build": "v4-a32-exact-round"}'
step traffic env VARIANTS=4 bash tools/pmc_traffic.sh || exit 1
step cache env VARIANTS=4 bash tools/pmc_cache.sh || exit 1
cp "$OUT/br_traffic.json" profiles/r01_br_traffic.json
step tests timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > "$OUT/tests.log" 2>&1 || exit 1
step smoke timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || exit 1
step bench timeout -k 10 600 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || exit 1
export TMPDIR=/tmp
step rocprof timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/prof.log" 2>&1 || exit 1
step configs bash tools/bench_configs.sh || exit 1
step corpus timeout -k 10 300 python bench.py --mode corpus --steps 2 > "$OUT/corpus.json" 2> "$OUT/corpus.err" || exit 1
step n2 env FHEICP_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 > "$OUT/n2.json" 2> "$OUT/n2.err" || exit 1
echo done >> "$OUT/steps.log"
