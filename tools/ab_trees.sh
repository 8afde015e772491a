#!/bin/bash
# Interleaved bench A/B of two source trees (the current one and a git
# worktree of an earlier commit at $OLD, each with its own in-tree library
# and binding): REPS x (old, new), compares/s and the blind-rotation and
# k_encrypt_linear launch times of each run.
set -u -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out/ab_trees
for rep in ${REPS:-1 2}; do
  for t in old new; do
    d=$R; [ "$t" = old ] && d=$R/${OLD:-ab_r05}
    o=$R/gpurun_out/ab_trees/${TAG:-c2}_${t}_$rep.json
    (cd "$d" && timeout -k 10 300 python bench.py --no-cpu-baseline --steps ${STEPS:-20} --warmup 3 ${ARGS:-} > $o 2> $o.err) || { echo "FAIL $t"; tail -5 $o.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('$o').read().strip().splitlines()[-1])
p=d.get('parity',{})
print('${TAG:-c2} $t rep$rep', d['value'], d['ms_per_step'], 'parity', all(v for k,v in p.items() if isinstance(v,bool)),
      ' '.join(f\"{k}:{v.get('kernel')}={v.get('avg_launch_ms')}\" for k,v in d['roofline'].get('kernels',{}).items()),
      'leveled', d['leveled_score']['roofline']['avg_launch_ms'], 'ks_ms_total', d.get('keyswitch_ms_total'))
"
  done
done
