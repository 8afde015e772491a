# interleaved A/B of the product library against tools/build_variant.sh builds
# usage: LIBS="round35" bash tools/ab_lib.sh   (P via P=..)
mkdir -p gpurun_out
for rep in 1 2; do
  for name in product ${LIBS}; do
    arg=""; [ "$name" != product ] && arg="--lib fhe-icp_amd/fheicp/libfheicp_$name.so"
    timeout -k 10 120 python tools/prof_br.py --variants 4 --rounds 3 --P ${P:-16} $arg 2>&1 | grep -v amdgpu.ids | sed "s/^/$name /" || exit 1
  done
done
