/* ORACLE test infrastructure: a sanitizer driver for the exported sign
 * extraction entry points of tfhe_ref.c (tests/test_oracle_tfhe.py compiles it
 * together with tfhe_ref.c under -fsanitize=address,undefined, without OpenMP).
 * On the TOY parameter set it encrypts eight 8-bit values of both signs, runs
 * ref_sign_extract and ref_sign_extract3 (no fast gadgets: their key arrays
 * are the short forms callers pass) and checks every sign bit. Exit 0 = all
 * exact and no sanitizer report. */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

typedef struct {
  int32_t n, k, N, pbs_base_log, pbs_level, ks_base_log, ks_level, lwe_noise_bits, glwe_noise_bits, msg_bits,
      sign_digit_bits, pbs_fast_base_log, pbs_fast_level, pbs_fast2_base_log, pbs_fast2_level, pbs_fast_group,
      pbs_fast2_group, pbs_mid_base_log, pbs_mid_level, pbs_mid2_base_log, pbs_mid2_level, pbs_mid_group,
      pbs_mid2_group, pbs_mid0_base_log, pbs_mid0_level, pbs_mid0_group;
} drv_params;

size_t ref_bsk_words(const drv_params* P);
size_t ref_ksk_words(const drv_params* P);
int ref_keygen(const drv_params* P, uint64_t seed, uint64_t* s_small, uint64_t* s_big, uint64_t* bsk, uint64_t* ksk);
void ref_encrypt_ints(const drv_params* P, const uint64_t* s_big, const int64_t* v, int64_t count, uint64_t seed,
                      uint64_t id0, uint64_t* ct);
void ref_sign_extract(const drv_params* P, const uint64_t* bsk, const uint64_t* ksk, uint64_t* ct_v, int64_t count,
                      uint64_t* sign);
void ref_sign_extract3(const drv_params* P, const uint64_t* bsk, const uint64_t* bsk2, const uint64_t* bsk3,
                       const uint64_t* ksk, uint64_t* ct_v, int64_t count, uint64_t* sign);
void ref_decrypt_bits(const drv_params* P, const uint64_t* s_big, const uint64_t* ct, int64_t count, int64_t* out);

int main(void) {
  drv_params P;
  memset(&P, 0, sizeof P);
  P.n = 64; P.k = 2; P.N = 256; P.pbs_base_log = 15; P.pbs_level = 2; P.ks_base_log = 4; P.ks_level = 4;
  P.lwe_noise_bits = 46; P.glwe_noise_bits = 17; P.msg_bits = 8;
  const int64_t count = 8, W = (int64_t)P.k * P.N + 1;
  uint64_t* s_small = calloc(P.n, 8);
  uint64_t* s_big = calloc((size_t)P.k * P.N, 8);
  uint64_t* bsk = calloc(ref_bsk_words(&P), 8);
  uint64_t* ksk = calloc(ref_ksk_words(&P), 8);
  int64_t* v = calloc(count, 8);
  int64_t* bits = calloc(count, 8);
  uint64_t* ct = calloc((size_t)(count * W), 8);
  uint64_t* sign = calloc((size_t)(count * W), 8);
  ref_keygen(&P, 99, s_small, s_big, bsk, ksk);
  for (int64_t i = 0; i < count; ++i) v[i] = i * 36 - 128;  /* -128 .. 124: both signs */
  int bad = 0;
  for (int form = 0; form < 2; ++form) {
    ref_encrypt_ints(&P, s_big, v, count, 7 + form, 0, ct);
    if (form == 0) ref_sign_extract(&P, bsk, ksk, ct, count, sign);
    else ref_sign_extract3(&P, bsk, NULL, NULL, ksk, ct, count, sign);
    ref_decrypt_bits(&P, s_big, sign, count, bits);
    for (int64_t i = 0; i < count; ++i) bad += bits[i] != (v[i] < 0);
  }
  printf("asan driver: %d wrong sign bits\n", bad);
  free(s_small); free(s_big); free(bsk); free(ksk); free(v); free(bits); free(ct); free(sign);
  return bad ? 1 : 0;
}
