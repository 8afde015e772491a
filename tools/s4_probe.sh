#!/bin/bash
# Multi-bit kernel A/B (psi address reuse, psi-1 table, early key loads at
# L = 1), phase stamps of the baseline, classic v4 vs key-stationary v4s for
# the main gadget, and the SQ counters of the headline bench.
set -u -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p "$OUT"; cd "$R"
L=fhe-icp_amd/fheicp
{
for rep in 1 2; do
  timeout -k 10 120 python tools/prof_mb.py --tag base || exit 1
  for v in ${VARIANTS:-psi1 psim pre}; do
    timeout -k 10 120 python tools/prof_mb.py --tag $v --lib $L/libfheicp_$v.so || exit 1
  done
done
for w in 0 5; do
  timeout -k 10 120 python tools/prof_mb.py --tag stamps --stamps $w --lib $L/libfheicp_ab.so || exit 1
done
for s in 0 1; do
  FHEICP_V4S=$s timeout -k 10 120 python tools/prof_br.py --variants 4 --rounds 3 --P 16 --lib $L/libfheicp_ab.so 2>&1 | sed "s/^/v4s=$s /" || exit 1
done
} > "$OUT/s4_probe.txt" 2>&1 || exit 1
bash tools/pmc_sq.sh > /dev/null || exit 1
