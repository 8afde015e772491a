#!/bin/bash
# A/B of the multi-bit fast-gadget blind rotation (FHEICP_MB=1) against the
# classic one on the bench workloads (C2, and a 2048-doc C3 slice).
set -o pipefail
mkdir -p gpurun_out
run() {  # name env args...
  local name=$1; shift
  local envv=$1; shift
  env $envv timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > gpurun_out/$name.json 2> gpurun_out/$name.err || { echo "FAIL $name"; tail -5 gpurun_out/$name.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/$name.json'))
print('$name', d['value'], d['ms_per_step'], json.dumps(d.get('parity'))[:300])
for k,v in d['roofline'].get('kernels',{}).items(): print('   ', k, v.get('kernel'), v.get('avg_launch_ms'), v.get('launches'))
"
}
run c2_mb FHEICP_MB=1 --steps 3 --warmup 1
run c2_base FHEICP_MB=0 --steps 3 --warmup 1
run c3_mb FHEICP_MB=1 --docs 2048 --dim 32 --n-bits 8 --steps 2 --warmup 1
run c3_base FHEICP_MB=0 --docs 2048 --dim 32 --n-bits 8 --steps 2 --warmup 1
