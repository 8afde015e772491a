#!/bin/bash
# A/B of key-stationary variants: multi-bit fast gadgets (prof_mb, FHEICP_MB=2)
# and classic v4s (prof_br, FHEICP_V4S=1), product vs LIBS builds
set -o pipefail
for rep in 1 2; do
  for name in product ${LIBS}; do
    arg=""; [ "$name" != product ] && arg="--lib fhe-icp_amd/fheicp/libfheicp_$name.so"
    FHEICP_MB=2 timeout -k 10 120 python tools/prof_mb.py --tag "$name" $arg 2>&1 | grep -v amdgpu.ids || exit 1
    for g in 15,2 23,1; do
      FHEICP_V4S=1 timeout -k 10 120 python tools/prof_br.py --variants 4 --rounds 3 --P 16 --gadget $g $arg 2>&1 | grep "blind_rotate" | sed "s/^/$name $g /" || exit 1
    done
  done
done
