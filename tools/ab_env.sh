# interleaved A/B of environment knobs (FHEICP_V4_*) for the (15,2) and (23,1) kernels
# usage: ENVS="FHEICP_V4_FL=1 FHEICP_V4_G=2" bash tools/ab_env.sh
mkdir -p gpurun_out
for rep in 1 2; do
  for g in 15,2 23,1; do
    for e in NONE=0 ${ENVS}; do
      env "$e" timeout -k 10 120 python tools/prof_br.py --variants 4 --rounds 3 --P 16 --gadget $g 2>&1 | grep blind_rotate | sed "s/^/$e $g /" || exit 1
    done
  done
done
