/* libfheicp development aids: NOT part of the drop-in ABI (include/fhe_icp.h).
 * Exported by every build so tools can bind them, but they work only in A/B
 * builds (tools/build_variant.sh -DFHEICP_AB; fhe_build_info() reports ab=1)
 * and return FHE_E_STATE in the shipped library. */
#ifndef FHE_ICP_DEV_H
#define FHE_ICP_DEV_H

#include "fhe_icp.h"

#ifdef __cplusplus
extern "C" {
#endif

/* A/B builds only: 4 x 16 s_memtime phase stamps of one wave of the v4 blind
 * rotation, then 2048 x {start, end, HW_ID} per workgroup (s_memrealtime),
 * recorded only when FHEICP_V4_DBG=128 (tools/prof_br.py --stamps); h_out
 * holds 64 + 6144 words. FHE_E_STATE in the shipped build. */
int fhe_debug_v4_stamps(fhe_ctx* ctx, uint64_t* h_out);

/* A/B builds only: k_encrypt_linear phase stamps, 1024 workgroups x 4 waves x
 * {s_memrealtime start, s_memtime at start / mask blocks done / noise blocks
 * done / after the barrier / MAC done / end, s_memrealtime end, HW_ID, XCC_ID}
 * (tools/el_stamps.py); h_out holds 40960 words. FHE_E_STATE in the shipped
 * build. */
int fhe_debug_el_stamps(fhe_ctx* ctx, uint64_t* h_out);

#ifdef __cplusplus
}
#endif
#endif /* FHE_ICP_DEV_H */
