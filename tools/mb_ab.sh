#!/bin/bash
# classic vs multi-bit fast-gadget bootstraps (FHEICP_MB = 0 classic, 1 per-
# ciphertext products, 2 key-stationary products), and A/B builds (LIBS="name ...")
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do
  for mb in ${MBS:-0 1 2}; do
    FHEICP_MB=$mb timeout -k 10 120 python tools/prof_mb.py --tag "mb$mb" || exit 1
  done
  for name in ${LIBS}; do
    FHEICP_MB=${LIBMB:-2} timeout -k 10 120 python tools/prof_mb.py --tag "$name" --lib fhe-icp_amd/fheicp/libfheicp_$name.so || exit 1
  done
done
