#!/bin/bash
# v2 against the key-stationary v4s kernels at the deep gadgets (L = 3..8):
# blind-rotation time per 1024 and output noise against the model
# (tools/prof_br.py --gadget): the libraries in $LIBS (default: an A/B
# build libfheicp_prev.so against the product library).
set -u -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"
for g in ${GADGETS:-12,3 10,4 8,5 7,6 6,7 5,8}; do
  for lib in ${LIBS:-libfheicp_prev.so libfheicp.so}; do
    [ -f fhe-icp_amd/fheicp/$lib ] || continue
    FHEICP_LIB=$R/fhe-icp_amd/fheicp/$lib timeout -k 10 120 python tools/prof_br.py --variants 4 --rounds 2 --P 26 --gadget $g 2>&1 | grep -v amdgpu.ids | sed "s/^/$lib g=$g /" || exit 1
  done
done
