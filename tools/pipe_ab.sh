#!/bin/bash
# Two-stream pipelined sign extraction (batches >= 2048) against one stream
# (FHEICP_PIPE=0), interleaved, on the C4 shard and C3.
set -u -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out/pipe_ab
for rep in 1 2; do
  for pipe in 0 1; do
    for cfg in "c4:--docs 12500 --dim 16 --n-bits 6" "c3:--docs 10000 --dim 32 --n-bits 8"; do
      name=${cfg%%:*}; args=${cfg#*:}
      o=gpurun_out/pipe_ab/${name}_pipe${pipe}_$rep.json
      FHEICP_PIPE=$pipe timeout -k 10 300 python bench.py --no-cpu-baseline --steps 2 --warmup 1 $args > $o 2> $o.err || { echo "FAIL $name $pipe"; tail -3 $o.err; exit 1; }
      python3 -c "
import json; d=json.load(open('$o')); p=d['parity']
print('$name pipe=$pipe rep$rep', d['value'], d['ms_per_step'], all(v for v in p.values() if isinstance(v, bool)))"
    done
  done
done
