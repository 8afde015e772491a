#!/bin/bash
# Interleaved bench A/B of library builds (tools/build_variant.sh NAME ...):
# LIBS="default name ..." ; extra bench args in $ARGS. Prints compares/s and
# the per-gadget kernel times of each run (parity flags included).
set -u -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out/lib_ab
for rep in ${REPS:-1 2}; do
  for name in ${LIBS}; do
    lib=fhe-icp_amd/fheicp/libfheicp.so; [ "$name" = default ] || lib=fhe-icp_amd/fheicp/libfheicp_$name.so
    o=gpurun_out/lib_ab/${TAG:-c2}_${name}_$rep.json
    FHEICP_LIB=$R/$lib timeout -k 10 300 python bench.py --no-cpu-baseline --steps ${STEPS:-5} --warmup 1 ${ARGS:-} > $o 2> $o.err || { echo "FAIL $name"; tail -5 $o.err; exit 1; }
    python3 -c "
import json; d=json.load(open('$o'))
p=d.get('parity',{})
print('${TAG:-c2} $name rep$rep', d['value'], d['ms_per_step'], 'parity', all(v for k,v in p.items() if isinstance(v,bool)),
      ' '.join(f\"{k}:{v.get('kernel')}={v.get('avg_launch_ms')}\" for k,v in d['roofline'].get('kernels',{}).items()),
      'leveled', d['leveled_score']['value'], d['leveled_score']['roofline']['avg_launch_ms'], d['leveled_score']['acc_equal_to_compare'])
"
  done
done
