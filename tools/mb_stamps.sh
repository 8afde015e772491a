#!/bin/bash
# phase timestamps of the multi-bit kernels (A/B build with FHEICP_AB)
set -o pipefail
for w in ${WAVES:-0 1 5}; do
  timeout -k 10 120 python tools/prof_mb.py --reps 1 --stamps $w --lib fhe-icp_amd/fheicp/libfheicp_ab.so || exit 1
done
