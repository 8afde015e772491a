# blind-rotation time of the u64-accumulator (12,3) kernel at 2 vs 1 ciphertexts per workgroup (P=21 set)
for rep in 1 2; do for G in 2 1; do FHEICP_V4_G=$G timeout -k 10 120 python tools/prof_br.py --variants 4 --rounds 2 --P 21 --gadget 12,3 2>&1 | grep blind_rotate | sed "s/^/G=$G /" || exit 1; done; done
