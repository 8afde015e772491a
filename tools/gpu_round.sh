#!/bin/bash
# One GPU session: parity tests -> smoke -> bench -> rocprofv3 kernel trace.
# Every GPU step has its own time limit; the script stops at the first failure.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p "$OUT"
cd "$R"
step() { local name=$1; shift; echo "== $name" >> "$OUT/steps.log"; "$@"; local rc=$?; echo "== $name rc=$rc" >> "$OUT/steps.log"; return $rc; }
step tests timeout -k 10 600 python -m pytest tests/ -m gpu -x -q -p no:cacheprovider > "$OUT/tests.log" 2>&1 || exit 1
step smoke timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || exit 1
step bench timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > "$OUT/bench.json" 2> "$OUT/bench.err" || exit 1
if [ "${PROFILE:-1}" = "1" ]; then
  export TMPDIR=/tmp
  step rocprof timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/prof.log" 2>&1 || exit 1
fi
echo done >> "$OUT/steps.log"
