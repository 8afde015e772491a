#!/bin/bash
# A/B of blind-rotation variants (timing) + the GPU parity tests on the default.
# Arguments G:FL (ciphertexts per workgroup : flag hand-offs). The library
# honours FHEICP_V4_G / FHEICP_V4_FL only in the A/B build
# (tools/build_variant.sh ab -DFHEICP_AB, then FHEICP_LIB=.../libfheicp_ab.so).
mkdir -p gpurun_out
[ -n "$NOTEST" ] || timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/ab_tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/ab_tests.log; exit 1; }
CFGS=${*:-"4:1 4:0 2:0"}
for cfg in $CFGS; do
  IFS=: read -r G F <<< "$cfg"
  FHEICP_V4_G=$G FHEICP_V4_FL=$F timeout -k 10 100 python tools/prof_br.py --variants 4 --rounds 3 --stamps 2>&1 | grep -v amdgpu.ids | sed "s/^/G=$G FL=$F /" || exit 1
done
