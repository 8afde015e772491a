/*
 * fhe_icp.h — C ABI of libfheicp.so, the MI355X (gfx950) engine behind the
 * encrypted pairwise compare of shipstone-labs/fhe-icp.
 *
 * Boundary. The reference reaches its hot path through a Concrete-ML
 * estimator object: FHESimilarityModel.model is a
 * concrete.ml.sklearn.LinearRegression (fhe_similarity.py:88-90) whose
 * .predict(X, fhe=...) is called at fhe_similarity.py:151 (fhe="execute",
 * encrypted), fhe_similarity.py:167 and batch_operations.py:233, :276
 * (clear). Everything BELOW that predict call (quantize -> encrypt -> leveled
 * dot product -> decrypt -> dequantize, concrete-python 2.10.0's runtime) is
 * replaced by the entry points below; the Python estimator in
 * fhe-icp_amd/fheicp/sklearn.py keeps the reference-facing API. The binding a
 * maintainer adds on the reference side is shown in INTEGRATION.md.
 *
 * Conventions.
 *  - Every function returns 0 on success and a negative FHE_E_* code on
 *    failure; fhe_last_error(ctx) (or NULL ctx) returns the message.
 *  - Pointers named d_* are DEVICE pointers on the context's device
 *    (caller-owned, e.g. torch tensors); pointers named h_* are host memory.
 *  - `stream` is a hipStream_t passed as void* (NULL = default stream). All
 *    launches are asynchronous on that stream unless documented otherwise.
 *  - One context per device; calls on one context must be externally
 *    serialised (same contract as the single-threaded reference callers).
 *  - Ciphertexts are little-endian u64 arrays. An LWE ciphertext of
 *    dimension d is [a_0 .. a_{d-1}, b] (d+1 words), phase = b - <a, s>
 *    modulo 2^64. "Big" ciphertexts use dimension k*N, "small" ones n.
 *  - Integer messages are encoded at Delta = 2^(64 - msg_bits).
 */
#ifndef FHE_ICP_H
#define FHE_ICP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FHE_OK 0
#define FHE_E_ARG (-1)      /* invalid argument / unsupported parameters */
#define FHE_E_DEVICE (-2)   /* HIP runtime error or no device */
#define FHE_E_STATE (-3)    /* keys not generated / imported */
#define FHE_E_NOMEM (-4)

/* Scheme parameters. After struct_size, the oracle's field
 * order (oracle/tfhe_ref.c ref_params). */
typedef struct fhe_params {
  int32_t struct_size;     /* = sizeof(fhe_params) (FHE_PARAMS_SIZE): every entry point
                              that reads a fhe_params checks it, so a binding built
                              against another version of this header (fewer or more
                              fields) fails with FHE_E_ARG instead of reading past
                              its struct or misreading fields */
  int32_t n;               /* small LWE dimension (blind-rotation length) */
  int32_t k;               /* GLWE dimension (1 or 2) */
  int32_t N;               /* polynomial size: 256, 512, 1024 or 2048 */
  int32_t pbs_base_log;    /* bootstrap gadget base log */
  int32_t pbs_level;       /* bootstrap gadget levels (1..8) */
  int32_t ks_base_log;     /* key-switch base log */
  int32_t ks_level;        /* key-switch levels */
  int32_t lwe_noise_bits;  /* TUniform bound, small LWE and KSK */
  int32_t glwe_noise_bits; /* TUniform bound, GLWE, BSK and big-key LWE */
  int32_t msg_bits;        /* P: message width of the accumulator encoding */
  int32_t sign_digit_bits; /* digit width d of fhe_sign_batch (3 or 4), or 0: the
                              widest d whose worst round keeps >= 9.2 sigma
                              (fhe_sign_digit_bits) */
  int32_t pbs_fast_base_log; /* optional second bootstrap gadget (0, 0: none). The */
  int32_t pbs_fast_level;    /* sign extraction runs its first fhe_sign_precise_rounds
                                bootstraps on (pbs_base_log, pbs_level) and the rest on
                                this cheaper one. keygen makes a second
                                bootstrapping key for it (fhe_export_fast_bsk); import
                                re-encrypts it with fresh randomness. */
  int32_t pbs_fast2_base_log; /* optional third, cheapest gadget (0, 0: none; needs the  */
  int32_t pbs_fast2_level;    /* fast one): the rounds from the plan's fast_end on use it */
  int32_t pbs_fast_group;  /* grouping factor of the fast / fast2 gadget's blind   */
  int32_t pbs_fast2_group; /* rotation: 0 or 1 = classic, one LWE coefficient per step;
                              2 = multi-bit, pairs of coefficients with three GGSWs
                              each (fhe_export_fast_bsk's layout: [pair][subset][row]
                              [component][coef]); needs N = 1024, k = 2, n <= 1023,
                              level <= 8, base_log <= 31 */
  int32_t pbs_mid_base_log;  /* optional gadgets between the main and the fast one */
  int32_t pbs_mid_level;     /* (0, 0: none; classic rotation; mid needs the fast  */
  int32_t pbs_mid2_base_log; /* gadget, mid2 needs mid): the sign plan runs the     */
  int32_t pbs_mid2_level;    /* rounds main -> mid -> mid2 -> fast -> fast2, each
                                gadget on the fewest rounds that keep every decision
                                at 9.2 sigma (fhe_sign_schedule).
                                Their keys: fhe_export_fast_bsk which = 3, 4. */
  int32_t pbs_mid_group;     /* grouping factor of the mid / mid2 gadget's blind */
  int32_t pbs_mid2_group;    /* rotation, as pbs_fast_group: 2 = multi-bit (levels
                                up to 8; 48-bit accumulators past level 2 or
                                level * base_log > 31: k_blind_rotate_mb64) */
  int32_t pbs_mid0_base_log; /* optional sixth gadget between the main and the mid */
  int32_t pbs_mid0_level;    /* one (0, 0: none; needs mid): the ladder is main ->  */
  int32_t pbs_mid0_group;    /* mid0 -> mid -> mid2 -> fast -> fast2, so a plan can run
                                its most amplified round on a multi-bit gadget as
                                precise as the classic main one (P = 26: (5,8)
                                multi-bit). Key: fhe_export_fast_bsk
                                which = 5 (stream tags 25/26, 27/28 multi-bit). */
} fhe_params;
#define FHE_PARAMS_SIZE ((int32_t)sizeof(fhe_params))

typedef struct fhe_ctx fhe_ctx;

/* ---- context -------------------------------------------------------------
 * Replaces the state Concrete builds in LinearRegression.compile()
 * (fhe_similarity.py:120: circuit + keys held on the CPU heap). device < 0
 * creates a host-only context (size queries, error strings; no kernels). */
int fhe_ctx_create(const fhe_params* params, int device, fhe_ctx** out);
void fhe_ctx_destroy(fhe_ctx* ctx);
const char* fhe_last_error(const fhe_ctx* ctx);
int fhe_get_params(const fhe_ctx* ctx, fhe_params* out);
/* Change P (msg_bits) without regenerating keys (keys do not depend on P). */
int fhe_set_msg_bits(fhe_ctx* ctx, int32_t msg_bits);

/* sizes in u64 words of the exported key material */
size_t fhe_bsk_words(const fhe_params* params);
size_t fhe_ksk_words(const fhe_params* params);
size_t fhe_big_lwe_words(const fhe_params* params);   /* k*N + 1 */
size_t fhe_small_lwe_words(const fhe_params* params); /* n + 1 */

/* ---- keys ----------------------------------------------------------------
 * Replaces Concrete keygen inside compile() (fhe_similarity.py:120) and the
 * key material FHEKeyManager.generate_keys means to persist
 * (key_management.py:112-191). Every key word is a ChaCha20 stream word
 *  under a 256-bit key. fhe_keygen_key is the production entry:
 * pass 32 bytes from the OS CSPRNG. fhe_keygen expands a 64-bit seed by
 * splitmix64 — 64 bits of entropy, NOT for production keys: reproducible
 * tests, fixtures and benches only. */
int fhe_keygen_key(fhe_ctx* ctx, const uint32_t h_key[8], void* stream);
int fhe_keygen(fhe_ctx* ctx, uint64_t seed, void* stream);
/* Host copies of the canonical key material; any pointer may be NULL.
 * s_small: n words (0/1); s_big: k*N words (0/1); bsk: fhe_bsk_words
 * (coefficient domain, [i][row][component][coef]); ksk: fhe_ksk_words
 * ([i][level][n+1]). Synchronous. */
int fhe_export_keys(fhe_ctx* ctx, uint64_t* h_s_small, uint64_t* h_s_big, uint64_t* h_bsk, uint64_t* h_ksk);
int fhe_import_keys(fhe_ctx* ctx, const uint64_t* h_s_small, const uint64_t* h_s_big, const uint64_t* h_bsk,
                    const uint64_t* h_ksk);
/* a fast gadget's bootstrapping key, which = 1 (pbs_fast_*, stream tags
 * 9/10, or 13/14 for a multi-bit key), 2 (pbs_fast2_*, tags 11/12 or
 * 15/16), 3 (pbs_mid_*, tags 17/18), 4 (pbs_mid2_*, tags 19/20) or 5
 * (pbs_mid0_*, tags 25/26; 21/22, 23/24 and 27/28 multi-bit): the
 * layout of bsk with one GGSW per LWE coefficient, or three per
 * pair of coefficients ([pair][subset {1}, {2}, {1,2}][row][component][coef])
 * when that gadget's group is 2; fhe_fast_bsk_words words (0: no such
 * gadget). FHE_E_STATE without that gadget. Synchronous. */
size_t fhe_fast_bsk_words(const fhe_params* params, int32_t which);
int fhe_export_fast_bsk(fhe_ctx* ctx, int32_t which, uint64_t* h_bsk);

/* ---- client side: encrypt / decrypt --------------------------------------
 * Replaces the per-sample encrypt/decrypt of predict(fhe="execute")
 * (fhe_similarity.py:151). Ciphertext c uses stream id (id0 + c).
 * Encryption randomness. Every encrypting entry point comes in two forms:
 * `*_key` takes the 256-bit ChaCha20 stream key (h_key / h_enc_key, 8 words),
 * the production form — one fresh CSPRNG key per session, independent of the
 * secret key's, with a random 64-bit id0 start, and stream ids (id0 + ...)
 * never reused under one key; the plain form takes a 64-bit `seed`
 * expanded by splitmix64 (fhe_key_from_seed): tests and benches only. */
int fhe_encrypt_batch_key(fhe_ctx* ctx, const int64_t* d_msg, int64_t count, const uint32_t h_key[8], uint64_t id0,
                          uint64_t* d_ct, void* stream);
int fhe_encrypt_batch(fhe_ctx* ctx, const int64_t* d_msg, int64_t count, uint64_t seed, uint64_t id0,
                      uint64_t* d_ct, void* stream);
/* round(phase / Delta) as signed msg_bits-bit integers */
int fhe_decrypt_batch(fhe_ctx* ctx, const uint64_t* d_ct, int64_t count, int64_t* d_out, void* stream);
/* 1 iff phase is nearer 2^63 than 0 (decrypts a sign/bit ciphertext) */
int fhe_decrypt_bits_batch(fhe_ctx* ctx, const uint64_t* d_ct, int64_t count, int64_t* d_out, void* stream);
/* raw phases (tests / noise measurement) */
int fhe_phase_batch(fhe_ctx* ctx, const uint64_t* d_ct, int64_t count, uint64_t* d_out, void* stream);

/* ---- server side -----------------------------------------------------------
 * The leveled circuit of Concrete-ML LinearRegression._inference:
 *   out[b] = sum_j d_w[j] * ct[b, j] + trivial(cst * Delta),
 * ct: B x D big ciphertexts (row-major), d_w: D int64 (device). */
int fhe_linear_batch(fhe_ctx* ctx, const uint64_t* d_ct, int64_t B, int32_t D, const int64_t* d_w, int64_t cst,
                     uint64_t* d_out, void* stream);
/* Packed feature encryption, the client side of the
 * reference's predict(fhe="execute") (fhe_similarity.py:151): the D features
 * of row b (d_qx, B x D, encoded at Delta) are the first coefficients of
 * G = ceil(D / N) GLWE messages; GLWE (b, g) uses stream id id0 + b*G + g.
 * d_glwe: B x G x (k+1)N words [A_1 .. A_k, B] per GLWE. */
int fhe_encrypt_packed_batch_key(fhe_ctx* ctx, const int64_t* d_qx, int64_t B, int32_t D, const uint32_t h_key[8],
                                 uint64_t id0, uint64_t* d_glwe, void* stream);
int fhe_encrypt_packed_batch(fhe_ctx* ctx, const int64_t* d_qx, int64_t B, int32_t D, uint64_t seed, uint64_t id0,
                             uint64_t* d_glwe, void* stream);
/* The leveled dot product on packed inputs (Concrete-ML
 * LinearRegression._inference's q_x @ q_w + constant): out[b] = sum_g
 * SampleExtract_0(GLWE(b, g) * sum_t d_w[gN + t] X^-t) + trivial(cst * Delta),
 * a big LWE (B x (kN+1)) of sum_j d_w[j] x[b, j] + cst. Needs no secret key. */
int fhe_linear_packed_batch(fhe_ctx* ctx, const uint64_t* d_glwe, int64_t B, int32_t D, const int64_t* d_w,
                            int64_t cst, uint64_t* d_out, void* stream);
/* fhe_encrypt_packed_batch followed by fhe_linear_packed_batch, fused: the
 * GLWEs are never written (bit-identical to the two calls). The single-party
 * form of predict(fhe="execute"): client encryption and the server's leveled
 * dot product in one pass; d_out: B x (kN+1). */
int fhe_encrypt_linear_batch_key(fhe_ctx* ctx, const int64_t* d_qx, int64_t B, int32_t D, const uint32_t h_key[8],
                                 uint64_t id0, const int64_t* d_w, int64_t cst, uint64_t* d_out, void* stream);
int fhe_encrypt_linear_batch(fhe_ctx* ctx, const int64_t* d_qx, int64_t B, int32_t D, uint64_t seed, uint64_t id0,
                             const int64_t* d_w, int64_t cst, uint64_t* d_out, void* stream);
/* big -> small key switch of (ct << shift) + add_body (shift/add used by the
 * bit extraction; pass 0, 0 for a plain key switch) */
int fhe_keyswitch_batch(fhe_ctx* ctx, const uint64_t* d_big, int64_t count, int32_t shift, uint64_t add_body,
                        uint64_t* d_small, void* stream);
/* Programmable bootstrap with the constant test vector `tv` (output phase
 * ~ +tv if the input phase is in [0, 2^63), ~ -tv otherwise), sample-
 * extracted under the big key. d_small: count x (n+1); d_out: count x (kN+1). */
int fhe_pbs_batch(fhe_ctx* ctx, const uint64_t* d_small, int64_t count, uint64_t tv, uint64_t* d_out,
                  void* stream);
/* fhe_pbs_batch on one of the parameter set's gadgets: 0 = the main one
 * (pbs_base_log, pbs_level), 1 = pbs_fast_*, 2 = pbs_fast2_*, 3 = pbs_mid_*,
 * 4 = pbs_mid2_*, 5 = pbs_mid0_* (with their own
 * bootstrapping keys and kernels, e.g. the multi-bit rotation of
 * pbs_fast_group = 2). FHE_E_STATE if that gadget is
 * absent. */
int fhe_pbs_gadget_batch(fhe_ctx* ctx, const uint64_t* d_small, int64_t count, int32_t gadget, uint64_t tv,
                         uint64_t* d_out, void* stream);
/* Exact LSB-first bit extraction of the msg_bits-bit value v encrypted in
 * d_ct_v (consumed). d_refreshed receives a fresh encryption of v (sum of
 * the bit ciphertexts), d_sign the ciphertext of the top bit ([v < 0] at
 * 2^63). msg_bits key-switches and bootstraps per ciphertext. */
int fhe_bit_extract_batch(fhe_ctx* ctx, uint64_t* d_ct_v, int64_t count, uint64_t* d_refreshed, uint64_t* d_sign,
                          void* stream);

/* Sign of the msg_bits-bit value v in d_ct_v (consumed): d_sign receives the
 * encryption of [v < 0] at 2^63 (decrypt with fhe_decrypt_bits_batch). Uses
 * fhe_sign_pbs_count(params) key switches + bootstraps per ciphertext: d-bit
 * digits (d = fhe_sign_digit_bits), two bootstraps each, then the sign of the
 * top d bits; 7 at msg_bits = 16 (d = 4). */
int fhe_sign_batch(fhe_ctx* ctx, uint64_t* d_ct_v, int64_t count, uint64_t* d_sign, void* stream);
/* Resolved digit width (params->sign_digit_bits, or the noise-model choice
 * when it is 0); 0 for msg_bits < 4 (single-bit rounds); -1 on bad params. */
int fhe_sign_digit_bits(const fhe_params* params);
int fhe_sign_pbs_count(const fhe_params* params);
/* how many of them (the first ones) run on the main gadget; all of them
 * without a fast gadget */
int fhe_sign_precise_rounds(const fhe_params* params);
/* the whole plan: digit width, bootstraps [0, main_rounds) on the main
 * gadget, [main_rounds, fast_end) on the mid0, mid, mid2 and fast ones (in
 * that order, fhe_sign_schedule), the rest on fast2
 * (DESIGN.md §3.6). Any pointer may be NULL. */
int fhe_sign_plan(const fhe_params* params, int32_t* digit_bits, int32_t* main_rounds, int32_t* fast_end);
/* the gadget (0..5, as fhe_pbs_gadget_batch) of every bootstrap of
 * fhe_sign_batch in order, into gadgets[0 .. min(R, cap)); returns R (the
 * bootstraps per sign extraction) or FHE_E_ARG on bad params. */
int fhe_sign_schedule(const fhe_params* params, int32_t* gadgets, int32_t cap);
/* MEASUREMENT ONLY (reads the secret key; no reference counterpart): the
 * decision noise behind the exactness of fhe_sign_batch (the decision of
 * batch_operations.py:278). Runs fhe_sign_batch's rounds on one stream, with
 *  - h_sched (host, R entries, NULL = fhe_sign_schedule's plan): the gadget
 *    of every round, e.g. a deliberately noisier one to narrow a margin;
 *  - rounds: stop after the first `rounds` bootstraps (0 = all R); d_sign is
 *    written (and required) only when the last round runs;
 *  - d_phase (device, NULL = none): round r's rotation exponent for
 *    ciphertext c at d_phase[r * count + c], the bootstrap input's phase
 *    modulus-switched to 2N exactly as that round's rotation (classic or
 *    multi-bit) rounds it, i.e. the test-vector index the rotation selects.
 * tests/test_gpu_decision_noise.py compares these with the exact rounds. */
int fhe_sign_trace_batch(fhe_ctx* ctx, uint64_t* d_ct_v, int64_t count, const int32_t* h_sched, int32_t rounds,
                         uint64_t* d_sign, uint32_t* d_phase, void* stream);
/* Bootstrap with a staircase test vector over 2^log_slots slots of the half
 * torus: output phase ~ base + floor(phase * 2^log_slots / 2^63) * step for an
 * input phase in [0, 2^63) (negacyclic beyond). log_slots = 0, step = 0 is
 * fhe_pbs_batch with tv = base. */
int fhe_pbs_lut_batch(fhe_ctx* ctx, const uint64_t* d_small, int64_t count, uint64_t base, uint64_t step,
                      int32_t log_slots, uint64_t* d_out, void* stream);

/* Programmable bootstrap with an arbitrary table (SURVEY.md §8b
 * fhe_pbs_batch(ctx, ct_in, B, const int64* lut, ct_out)): the input small
 * LWE encrypts a message m in [0, 2^lut_bits) at 2^(63 - lut_bits) (one
 * padding bit); the output big LWE encrypts d_lut[m] (a signed msg_bits-bit
 * value) at Delta = 2^(64 - msg_bits). The test vector is built on the device
 * from d_lut (2^lut_bits int64, device memory): box m covers the input phases
 * within half a box of m * 2^(63 - lut_bits). 0 <= lut_bits <= log2(N) - 1;
 * the caller keeps the input noise (after key and modulus switching) inside
 * half a box. */
int fhe_pbs_table_batch(fhe_ctx* ctx, const uint64_t* d_small, int64_t count, const int64_t* d_lut, int32_t lut_bits,
                        uint64_t* d_out, void* stream);
/* fhe_pbs_table_batch on an explicit gadget (0..5, as fhe_pbs_gadget_batch):
 * a multi-bit gadget runs the sign extraction's multi-bit rotation
 * (k_blind_rotate_mb / _mb64) with the table test vector and that gadget's
 * key; 0 the classic main gadget. fhe_pbs_table_batch takes
 * fhe_pbs_table_gadget(params): the most precise multi-bit gadget of the set
 * (smallest bootstrap noise), 0 when it has none; FHE_E_ARG on bad params. */
int fhe_pbs_table_gadget_batch(fhe_ctx* ctx, const uint64_t* d_small, int64_t count, int32_t gadget,
                               const int64_t* d_lut, int32_t lut_bits, uint64_t* d_out, void* stream);
int fhe_pbs_table_gadget(const fhe_params* params);
/* The encrypted decision of batch_operations.py:278 (score >= min_similarity
 * <=> acc >= T, SURVEY.md §8b fhe_threshold_batch): d_ct_acc holds big LWEs of
 * msg_bits-bit accumulators (not modified); d_bit receives the encryption of
 * [acc >= T] at 2^63 (fhe_decrypt_bits_batch). acc - T must fit msg_bits
 * bits. fhe_sign_pbs_count(params) key switches + bootstraps per ciphertext. */
int fhe_threshold_batch(fhe_ctx* ctx, const uint64_t* d_ct_acc, int64_t count, int64_t T, uint64_t* d_bit,
                        void* stream);

/* ---- fused compare / search ------------------------------------------------
 * One call per batch of B (query, document) pairs — the batched replacement
 * of the per-document loop at batch_operations.py:268-279 and of
 * compare_encrypted (batch_operations.py:206-238):
 *   encrypt q_x (B x D) -> linear with d_w and cst - T -> decrypt the
 *   leveled accumulator -> sign extraction (fhe_sign_pbs_count(params)
 *   KS + PBS) -> decrypt the sign bit. d_acc[b] = the decrypted accumulator (exact int64, = Concrete's
 *   q_x @ q_w - zp*sum(q_w) + q_b; read from the leveled ciphertext like the
 *   reference's leveled circuit), d_below[b] = 1 iff acc < T (the decrypted
 *   bootstrapped threshold bit; acc >= T <=> score >= min_similarity).
 * Uses context-owned workspace of ~8 * B * (2(kN+1) + n + 2) bytes (grown on
 * demand; not graph-capturable): the encryption is fused into the linear step
 * (fhe_encrypt_linear_batch), so D does not enter the footprint. The `_key`
 * form takes the session's 256-bit encryption key (see "Encryption
 * randomness"); the enc_seed form is for tests and benches. */
int fhe_compare_batch_key(fhe_ctx* ctx, const int64_t* d_qx, int64_t B, int32_t D, const int64_t* d_w, int64_t cst,
                          int64_t T, const uint32_t h_enc_key[8], uint64_t id0, int64_t* d_acc, int64_t* d_below,
                          void* stream);
int fhe_compare_batch(fhe_ctx* ctx, const int64_t* d_qx, int64_t B, int32_t D, const int64_t* d_w, int64_t cst,
                      int64_t T, uint64_t enc_seed, uint64_t id0, int64_t* d_acc, int64_t* d_below, void* stream);
/* The reference's predict(fhe="execute") as it is (fhe_similarity.py:142-160,
 * one row per call at :149-158): a leveled circuit with no PBS. encrypt q_x
 * -> linear with d_w and cst - T -> decrypt; d_acc[b] = the accumulator
 * (exact int64). No key switch or bootstrap runs; T only centres the value in
 * the msg_bits-bit encoding (acc - T must fit it; the estimator passes the
 * middle of the accumulator range). Workspace ~8 * B * (kN + 2) bytes.
 * `_key` form: the session's 256-bit encryption key, as fhe_compare_batch_key. */
int fhe_score_batch_key(fhe_ctx* ctx, const int64_t* d_qx, int64_t B, int32_t D, const int64_t* d_w, int64_t cst,
                        int64_t T, const uint32_t h_enc_key[8], uint64_t id0, int64_t* d_acc, void* stream);
int fhe_score_batch(fhe_ctx* ctx, const int64_t* d_qx, int64_t B, int32_t D, const int64_t* d_w, int64_t cst,
                    int64_t T, uint64_t enc_seed, uint64_t id0, int64_t* d_acc, void* stream);

/* ---- seeded (compressed) ciphertexts: the encrypted document corpus -------
 * Persisted documents (EncryptedDocument at
 * encrypted_storage.py:19-51, whose `encrypted_embedding` is a plaintext
 * vector in the reference, batch_operations.py:175-178) are stored as
 * seeded LWEs: only the body word per feature. The mask of feature j of
 * document b is ChaCha20 stream (TAG_ENC_MASK, id0[b] + j) under the PUBLIC
 * 256-bit mask key; the noise comes from the SECRET noise key. A corpus in
 * HBM is then B x D body words plus B ids instead of B x D x (kN + 1) words;
 * the masks are regenerated inside the kernels that consume them.
 * d_msg / d_body: B x D (row-major), d_id0: B u64 (stream ids must not repeat
 * under one mask key). */
int fhe_encrypt_seeded_batch(fhe_ctx* ctx, const int64_t* d_msg, int64_t B, int32_t D, const uint32_t h_mask_key[8],
                             const uint32_t h_noise_key[8], const uint64_t* d_id0, uint64_t* d_body, void* stream);
/* full ciphertexts (B*D x (kN+1)) of a seeded corpus; needs no secret key */
int fhe_expand_seeded_batch(fhe_ctx* ctx, const uint64_t* d_body, const uint64_t* d_id0, int64_t B, int32_t D,
                            const uint32_t h_mask_key[8], uint64_t* d_ct, void* stream);
/* fhe_linear_batch on a seeded corpus (masks regenerated in registers):
 * out[b] = sum_j d_w[j] * ct(b, j) + trivial(cst * Delta); B x (kN+1). */
int fhe_linear_seeded_batch(fhe_ctx* ctx, const uint64_t* d_body, const uint64_t* d_id0, int64_t B, int32_t D,
                            const uint32_t h_mask_key[8], const int64_t* d_w, int64_t cst, uint64_t* d_out,
                            void* stream);
/* fhe_compare_batch over a stored encrypted corpus: linear (seeded) with d_w
 * and cst - T -> decrypt the leveled accumulator -> sign extraction ->
 * decrypt the threshold bit. The documents were encrypted at some P0 >= the
 * context's msg_bits P; the caller folds 2^(P0 - P) into d_w. */
int fhe_compare_seeded_batch(fhe_ctx* ctx, const uint64_t* d_body, const uint64_t* d_id0, int64_t B, int32_t D,
                             const uint32_t h_mask_key[8], const int64_t* d_w, int64_t cst, int64_t T,
                             int64_t* d_acc, int64_t* d_below, void* stream);
/* The 64-bit-seed -> 256-bit ChaCha key expansion used by the seed forms
 * (fhe_keygen, fhe_encrypt_batch, ...; splitmix64): tests and
 * benches only. Host only. */
void fhe_key_from_seed(uint64_t seed, uint32_t h_key_out[8]);

/* ---- clear pre/post-processing on the device ----------------------------
 * Pair features and Concrete-ML's input quantizer in one pass:
 * X[b, j] = query[j] * docs[b, j] in numpy's promoted dtype (the query may be
 * f64, batch_operations.py:260; stored docs are f32, :178), or X = docs when
 * d_query is NULL; then q = clip(rint(X / scale + zero_point), qmin, qmax)
 * in float64 (concrete-ml UniformQuantizer.quant). Bit-identical to numpy. */
int fhe_quantize_pairs(fhe_ctx* ctx, const void* d_query, int32_t query_is_f64, const void* d_docs,
                       int32_t docs_is_f64, int64_t B, int32_t D, double scale, int64_t zero_point, int64_t qmin,
                       int64_t qmax, int64_t* d_qx, void* stream);
/* The embedding stage's PCA (dimension_reduction.py:67-72: sklearn
 * PCA.transform, no whitening), SURVEY.md §8f-4: d_out[b][d] = sum_k
 * (d_x[b][k] - d_mean[k]) * d_components[d][k] for B rows of K <= 1024
 * float32 features and D components (row-major, as PCA.components_),
 * accumulated in f64 and stored as float32 (the reference stores float32
 * embeddings, batch_operations.py:175-178). Needs no keys. */
int fhe_pca_transform(fhe_ctx* ctx, const float* d_x, int64_t B, int32_t K, const float* d_mean,
                      const float* d_components, int32_t D, float* d_out, void* stream);
/* score[b] = out_scale * (double)acc[b] (UniformQuantizer.dequant, zp 0) */
int fhe_dequantize(fhe_ctx* ctx, const int64_t* d_acc, int64_t B, double out_scale, double* d_score, void* stream);

/* Top-k of d_acc over entries with d_below == 0 (or all if d_below is
 * NULL), ordered by (acc desc, index asc) — Python's stable sort of
 * batch_operations.py:282 on a monotone dequantisation. Indices are
 * base_idx + position. Missing slots get acc = INT64_MIN, idx = -1. */
int fhe_topk(fhe_ctx* ctx, const int64_t* d_acc, const int64_t* d_below, int64_t B, int64_t base_idx, int32_t k,
             int64_t* d_out_acc, int64_t* d_out_idx, void* stream);

/* ---- device memory -------------------------------------------------------
 * For callers without a device allocator of their own (a ctypes binding from
 * numpy); torch callers pass tensor pointers instead.
 * fhe_memcpy_d2h returns after the copy completed (it synchronises `stream`). */
int fhe_dev_alloc(fhe_ctx* ctx, size_t bytes, void** d_out);
int fhe_dev_free(fhe_ctx* ctx, void* d_ptr);
int fhe_memcpy_h2d(fhe_ctx* ctx, void* d_dst, const void* h_src, size_t bytes, void* stream);
int fhe_memcpy_d2h(fhe_ctx* ctx, void* h_dst, const void* d_src, size_t bytes, void* stream);
int fhe_stream_sync(fhe_ctx* ctx, void* stream);

/* ---- measurement ------------------------------------------------------------
 * When enabled, every blind-rotation (external-product) and key-switch
 * launch is bracketed by hipEvents on its own stream. fhe_profile_read
 * synchronises and returns total milliseconds, launch count and ciphertexts
 * processed for kernel "blind_rotate" (all gadgets), "blind_rotate_main",
 * "blind_rotate_fast" (fhe_params.pbs_fast_*), "blind_rotate_fast2",
 * "blind_rotate_mid", "blind_rotate_mid2", "blind_rotate_mid0", "keyswitch" or "encrypt_linear"
 * (the fused client encryption + leveled dot), then resets what it
 * read. */
int fhe_profile_enable(fhe_ctx* ctx, int enable);
int fhe_profile_read(fhe_ctx* ctx, const char* kernel, double* total_ms, int64_t* launches, int64_t* items);
/* The kernel last launched for that bucket, as rocprofv3 names it (e.g.
 * "k_blind_rotate_v4<2, true, 0, 4, false, 15>", "k_blind_rotate_mb<1, 0, 23>",
 * "k_keyswitch_mfma"); "" before any launch. Not reset by fhe_profile_read. */
int fhe_profile_kernel_name(fhe_ctx* ctx, const char* kernel, char* h_buf, size_t len);
/* "libfheicp gfx950 ab=0" for the shipped build; ab=1 for A/B builds
 * (tools/build_variant.sh -DFHEICP_AB: extra v4 shapes, v3, timing kernels). */
const char* fhe_build_info(void);
#ifdef __cplusplus
}
#endif
#endif /* FHE_ICP_H */
