#!/bin/bash
# PMC + kernel-trace passes of the headline, C3 (one stream: FHEICP_PIPE=0),
# C5 and the table-bootstrap (--mode lut) runs of this build, merged into one br_pmc.json keyed on its sha
# (copy gpurun_out/pmc_r03/br_pmc.json to profiles/br_pmc.json), and each
# run's rocprofv3 --stats kernel summary.
set -u -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=$R/gpurun_out/pmc_r03; mkdir -p "$O"
run() {  # tag cts args...
  local tag=$1 cts=$2; shift 2
  PMC_OUT=$O/$tag CTS=$cts BENCH_ARGS="$*" PMC_MERGE=$O/br_pmc.json bash tools/pmc_bench.sh || return 1
  cp "$O/$tag/br_pmc.json" "$O/br_pmc.json" || return 1
  cp "$(ls "$O/$tag"/trace/*kernel_stats.csv "$O/$tag"/trace/*/*kernel_stats.csv 2>/dev/null | head -n1)" "$O/${tag}_kernel_stats.csv"
  echo "$tag done" >> "$O/steps.log"
}
rm -f "$O/br_pmc.json"
run c2 1024 || exit 1
export FHEICP_PIPE=0
PMC_ENV="FHEICP_PIPE=0 " run c3 10000 --docs 10000 --dim 32 --n-bits 8 || exit 1
unset FHEICP_PIPE
run c5 1000 --docs 1000 --dim 768 --n-bits 8 || exit 1
# the table bootstrap on the multi-bit rotation (bench.py --mode lut)
run lut 1024 --mode lut || exit 1
