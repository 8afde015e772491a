# output noise of the v4 kernel by workgroup shape and accumulator width (P=16 gadget)
mkdir -p gpurun_out
for cfg in 4:0 2:0 1:0 2:1 1:1; do
  G=${cfg%:*}; A=${cfg#*:}
  FHEICP_V4_G=$G FHEICP_V4_A64=$A timeout -k 10 120 python tools/prof_br.py --variants 4 --rounds 2 --P 16 2>&1 | grep -v amdgpu.ids || exit 1
done
