#!/bin/bash
# A/B builds of libfheicp.so with a compile-time switch, next to the product
# library (git-ignored): tools/build_variant.sh NAME -DFLAG ...
# -> fhe-icp_amd/fheicp/libfheicp_NAME.so, loaded by tools/prof_br.py --lib
set -e
HERE=$(cd "$(dirname "$0")/.." && pwd)
name=$1; shift
hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -Wno-unused-result "$@" \
  -o "$HERE/fhe-icp_amd/fheicp/libfheicp_$name.so" "$HERE/fhe-icp_amd/csrc/fheicp.hip" "$HERE/fhe-icp_amd/csrc/bert.hip"
