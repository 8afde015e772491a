#!/bin/bash
# classic v4 vs key-stationary v4s (FHEICP_V4S=1) for the classic gadgets
# (needs the A/B build: tools/build_variant.sh ab -DFHEICP_AB)
set -o pipefail
for rep in 1 2; do
  for g in 15,2 23,1 12,3; do
    for s in 0 1; do
      FHEICP_V4S=$s timeout -k 10 120 python tools/prof_br.py --variants 4 --rounds 3 --P 16 --gadget $g --lib fhe-icp_amd/fheicp/libfheicp_ab.so 2>&1 | grep -v amdgpu.ids | sed "s/^/v4s=$s /" || exit 1
    done
  done
done
