# interleaved A/B of the product library against variant builds, for the
# (15,2) and (23,1) gadgets: LIBS="name ..." bash tools/ab_lib2.sh
mkdir -p gpurun_out
for rep in 1 2; do
  for g in 15,2 23,1; do
    for name in product ${LIBS}; do
      arg=""; [ "$name" != product ] && arg="--lib fhe-icp_amd/fheicp/libfheicp_$name.so"
      timeout -k 10 120 python tools/prof_br.py --variants 4 --rounds 3 --P 16 --gadget $g $arg 2>&1 | grep -v amdgpu.ids | sed "s/^/$name /" || exit 1
    done
  done
done
