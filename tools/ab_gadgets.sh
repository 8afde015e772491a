# blind-rotation time and output noise per bootstrap gadget (P=16 set otherwise)
mkdir -p gpurun_out
for g in ${GADGETS:-15,2 23,1 22,1 24,1 20,1 12,3}; do
  timeout -k 10 120 python tools/prof_br.py --variants 4 --rounds 3 --P 16 --gadget $g 2>&1 | grep -v amdgpu.ids || exit 1
done
