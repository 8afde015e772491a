#!/bin/bash
# VGPRs / LDS / scratch of every kernel in libfheicp's gfx950 code object
# (no GPU needed): extracts the offload bundle and reads the AMDHSA metadata.
set -e
HERE=$(cd "$(dirname "$0")" && pwd)
OUT=${1:-/tmp/fheicp_co}
mkdir -p "$OUT"
cd "$OUT"
hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared --save-temps -Wno-unused-result \
  -o libtmp.so "$HERE/../fhe-icp_amd/csrc/fheicp.hip" 2>/dev/null
S=fheicp-hip-amdgcn-amd-amdhsa-gfx950.s
python3 - "$S" "${2:-blind_rotate}" <<'PY'
import re, sys
txt = open(sys.argv[1]).read()
for m in re.finditer(r"\.amdhsa_kernel (\S+)\n(.*?)\.end_amdhsa_kernel", txt, re.S):
    name, body = m.group(1), m.group(2)
    if sys.argv[2] not in name:
        continue
    g = lambda k: (re.search(r"\." + k + r" (\d+)", body) or [None, "?"])[1]
    print(f"{name[:70]:70s} vgpr_next={g('amdhsa_next_free_vgpr')} lds={g('amdhsa_group_segment_fixed_size')} "
          f"scratch={g('amdhsa_private_segment_fixed_size')}")
PY
