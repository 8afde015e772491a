/*
 * ORACLE (test infrastructure only) — exact CPU restatement of the
 * FHEICP-TFHE v1 scheme that the MI355X kernels implement.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load this library, and only as the checker. It is plain C (gcc, optional
 * OpenMP) and shares NO code with the product (fhe-icp_amd/csrc): every
 * primitive is written again from the spec in DESIGN.md §3.
 *
 * Reference anchor. The reference's encrypted path is
 * FHESimilarityModel.predict_encrypted -> model.predict(X[i:i+1], fhe="execute")
 * (fhe_similarity.py:142-160, :151): quantize -> encrypt -> leveled dot
 * product with clear weights -> decrypt, run by concrete-python 2.10.0's CPU
 * runtime (pinned at requirements.txt:5-7). That runtime is not in
 * /root/reference and cannot be installed offline, so the TFHE parameters are
 * this build's own; parity with the reference is asserted on the DECRYPTED
 * integer accumulator, which tests compare with oracle/quant_ref.py (the
 * restated Concrete-ML clear inference). The PBS stage (LSB-first bit
 * extraction) has no reference counterpart; its parity
 * target is the exact accumulator and the threshold bit of
 * batch_operations.py:278.
 *
 * Arithmetic. Everything is exact integer arithmetic modulo 2^64 (unsigned
 * wrap-around). Negacyclic polynomial products use Karatsuba over Z_{2^64},
 * an exact ring algorithm, whereas the GPU uses an f64 FFT whose rounding is
 * extra noise; so GPU and oracle agree bit-for-bit on keys, encryptions,
 * linear combinations and key switching, agree on decrypted values after a
 * bootstrap, and differ there only by a small bounded phase error
 * (tests/test_gpu_parity.py checks both).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef struct {
  int32_t n;               /* small LWE dimension */
  int32_t k;               /* GLWE dimension */
  int32_t N;               /* polynomial size (power of two) */
  int32_t pbs_base_log;
  int32_t pbs_level;
  int32_t ks_base_log;
  int32_t ks_level;
  int32_t lwe_noise_bits;  /* TUniform bound: small LWE / KSK */
  int32_t glwe_noise_bits; /* TUniform bound: GLWE / BSK / big-key LWE */
  int32_t msg_bits;        /* P: message width */
  int32_t sign_digit_bits; /* sign-extraction digit width, 0 = noise-model choice */
  int32_t pbs_fast_base_log; /* second (fast) bootstrap gadget for the low-  */
  int32_t pbs_fast_level;    /* amplification sign rounds; 0, 0 = none      */
  int32_t pbs_fast2_base_log; /* third, cheapest gadget for the last rounds */
  int32_t pbs_fast2_level;    /* (needs the fast one); 0, 0 = none          */
  int32_t pbs_fast_group;     /* blind rotation of the fast / fast2 gadget: */
  int32_t pbs_fast2_group;    /* 0, 1 classic; 2 multi-bit pairs            */
  int32_t pbs_mid_base_log;   /* gadgets between the main and the fast one  */
  int32_t pbs_mid_level;      /* (classic rotation; 0, 0 = none; mid needs  */
  int32_t pbs_mid2_base_log;  /* the fast gadget, mid2 needs mid)           */
  int32_t pbs_mid2_level;
  int32_t pbs_mid_group;      /* blind rotation of the mid / mid2 gadget    */
  int32_t pbs_mid2_group;     /* (as pbs_fast_group)                        */
  int32_t pbs_mid0_base_log;  /* sixth gadget, between the main and the mid */
  int32_t pbs_mid0_level;     /* one (0, 0 = none; needs mid)               */
  int32_t pbs_mid0_group;
} ref_params;

/* --------------------------------------------------------------- chacha --- */
#define ROTL(a, b) (((a) << (b)) | ((a) >> (32 - (b))))
#define QR(a, b, c, d) \
  a += b; d ^= a; d = ROTL(d, 16); c += d; b ^= c; b = ROTL(b, 12); \
  a += b; d ^= a; d = ROTL(d, 8);  c += d; b ^= c; b = ROTL(b, 7);

typedef struct { uint32_t key[8]; } ref_key;

/* RFC 8439 ChaCha20 block: state = consts | key | counter | nonce[3] */
static void chacha20_block(const ref_key* K, uint32_t counter, uint32_t n0, uint32_t n1, uint32_t n2,
                           uint32_t out[16]) {
  uint32_t s[16] = {0x61707865u, 0x3320646eu, 0x79622d32u, 0x6b206574u,
                    K->key[0], K->key[1], K->key[2], K->key[3], K->key[4], K->key[5], K->key[6], K->key[7],
                    counter, n0, n1, n2};
  uint32_t x[16];
  memcpy(x, s, sizeof x);
  for (int i = 0; i < 10; ++i) {
    QR(x[0], x[4], x[8], x[12]); QR(x[1], x[5], x[9], x[13]);
    QR(x[2], x[6], x[10], x[14]); QR(x[3], x[7], x[11], x[15]);
    QR(x[0], x[5], x[10], x[15]); QR(x[1], x[6], x[11], x[12]);
    QR(x[2], x[7], x[8], x[13]); QR(x[3], x[4], x[9], x[14]);
  }
  for (int i = 0; i < 16; ++i) out[i] = x[i] + s[i];
}
/* exposed for tests (RFC 8439 §2.3.2 vector) */
void ref_chacha20_block(const uint32_t key[8], uint32_t counter, const uint32_t nonce[3], uint32_t out[16]) {
  ref_key K;
  memcpy(K.key, key, 32);
  chacha20_block(&K, counter, nonce[0], nonce[1], nonce[2], out);
}

/* Stream (tag, id): u64 word w = block w/8 (counter), words 2j, 2j+1 of it. */
typedef struct {
  const ref_key* K;
  uint32_t tag;
  uint64_t id;
  uint64_t cur_block;
  uint32_t buf[16];
} ref_stream;

static void stream_init(ref_stream* st, const ref_key* K, uint32_t tag, uint64_t id) {
  st->K = K; st->tag = tag; st->id = id; st->cur_block = (uint64_t)-1;
}
static uint64_t stream_word(ref_stream* st, uint64_t w) {
  uint64_t blk = w >> 3;
  if (blk != st->cur_block) {
    chacha20_block(st->K, (uint32_t)blk, st->tag, (uint32_t)st->id, (uint32_t)(st->id >> 32), st->buf);
    st->cur_block = blk;
  }
  unsigned j = (unsigned)(w & 7);
  return (uint64_t)st->buf[2 * j] | ((uint64_t)st->buf[2 * j + 1] << 32);
}

static uint64_t splitmix64(uint64_t* x) {
  uint64_t z = (*x += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
static void key_from_seed(uint64_t seed, ref_key* K) {
  uint64_t x = seed;
  for (int i = 0; i < 4; ++i) {
    uint64_t v = splitmix64(&x);
    K->key[2 * i] = (uint32_t)v;
    K->key[2 * i + 1] = (uint32_t)(v >> 32);
  }
}

/* TUniform(b) from one u64 word: b+2 low bits -> (bits>>1)+(bits&1) - 2^b */
static int64_t tuniform(uint64_t w, int b) {
  uint64_t bits = w & ((2ull << (b + 1)) - 1);
  return (int64_t)((bits >> 1) + (bits & 1)) - ((int64_t)1 << b);
}
int64_t ref_tuniform(uint64_t w, int b) { return tuniform(w, b); }

enum { TAG_SK_SMALL = 1, TAG_SK_GLWE = 2, TAG_BSK_MASK = 3, TAG_BSK_NOISE = 4, TAG_KSK_MASK = 5,
       TAG_KSK_NOISE = 6, TAG_ENC_MASK = 7, TAG_ENC_NOISE = 8, TAG_BSK2_MASK = 9, TAG_BSK2_NOISE = 10,
       TAG_BSK3_MASK = 11, TAG_BSK3_NOISE = 12, TAG_MB2_MASK = 13, TAG_MB2_NOISE = 14, TAG_MB3_MASK = 15,
       TAG_MB3_NOISE = 16, TAG_BSK4_MASK = 17, TAG_BSK4_NOISE = 18, TAG_BSK5_MASK = 19, TAG_BSK5_NOISE = 20,
       TAG_MB4_MASK = 21, TAG_MB4_NOISE = 22, TAG_MB5_MASK = 23, TAG_MB5_NOISE = 24, TAG_BSK6_MASK = 25,
       TAG_BSK6_NOISE = 26, TAG_MB6_MASK = 27, TAG_MB6_NOISE = 28 };

/* --------------------------------------------------- negacyclic product --- */
/* c[0..2n-2] = a * b (plain product over Z_{2^64}); scratch >= 4n words */
static void kara(const uint64_t* a, const uint64_t* b, uint64_t* c, int n, uint64_t* scratch) {
  if (n <= 32) {
    for (int i = 0; i < 2 * n - 1; ++i) c[i] = 0;
    for (int i = 0; i < n; ++i) {
      const uint64_t ai = a[i];
      for (int j = 0; j < n; ++j) c[i + j] += ai * b[j];
    }
    return;
  }
  const int h = n / 2;
  uint64_t* as = scratch;        /* h */
  uint64_t* bs = scratch + h;    /* h */
  uint64_t* mid = scratch + 2 * h; /* 2h-1 */
  uint64_t* rest = scratch + 4 * h;
  /* low and high products straight into c */
  kara(a, b, c, h, rest);                 /* c[0..2h-2] */
  c[2 * h - 1] = 0;
  kara(a + h, b + h, c + 2 * h, h, rest); /* c[2h..4h-2] */
  for (int i = 0; i < h; ++i) { as[i] = a[i] + a[i + h]; bs[i] = b[i] + b[i + h]; }
  kara(as, bs, mid, h, rest);
  for (int i = 0; i < 2 * h - 1; ++i) mid[i] -= c[i] + c[2 * h + i];
  for (int i = 0; i < 2 * h - 1; ++i) c[h + i] += mid[i];
}
/* acc += a * b mod (X^N + 1), all mod 2^64. scratch >= 8N words */
static void negacyclic_mac(const uint64_t* a, const uint64_t* b, uint64_t* acc, int N, uint64_t* scratch) {
  uint64_t* full = scratch;          /* 2N */
  kara(a, b, full, N, scratch + 2 * N);
  full[2 * N - 1] = 0;
  for (int t = 0; t < N; ++t) acc[t] += full[t] - full[t + N];
}
/* exposed for tests */
void ref_negacyclic_mul(const uint64_t* a, const uint64_t* b, uint64_t* c, int N) {
  uint64_t* scratch = (uint64_t*)malloc(8 * (size_t)(16 * N));
  for (int t = 0; t < N; ++t) c[t] = 0;
  negacyclic_mac(a, b, c, N, scratch);
  free(scratch);
}

/* ---------------------------------------------------------------- sizes --- */
static int rows(const ref_params* P) { return (P->k + 1) * P->pbs_level; }
size_t ref_bsk_words(const ref_params* P) { return (size_t)P->n * rows(P) * (P->k + 1) * P->N; }
size_t ref_ksk_words(const ref_params* P) { return (size_t)P->k * P->N * P->ks_level * (P->n + 1); }

/* --------------------------------------------------------------- keygen --- */
/* GGSW i (i < count), row r: GLWE_S(0) + msg[i] * g_lvl on component c_in,
 * g_lvl = 2^(64 - lvl*beta); (beta, L) and the stream tags select the main or
 * a fast gadget's key. msg = s_small (one GGSW per LWE coefficient) or the
 * multi-bit messages of mb_msgs (three per pair). */
static void bsk_gen(const ref_params* P, const ref_key* Kp, int beta, int L, int tag_mask, int tag_noise,
                    const uint64_t* msg, int count, const uint64_t* s_big, uint64_t* bsk) {
  const ref_key K = *Kp;
  const int k = P->k, N = P->N, R = (k + 1) * L;
#pragma omp parallel for schedule(dynamic)
  for (int i = 0; i < count; ++i) {
    uint64_t* scratch = (uint64_t*)malloc(8 * (size_t)(16 * N));
    uint64_t* S = (uint64_t*)malloc(8 * (size_t)N);
    ref_stream sm, sn;
    for (int r = 0; r < R; ++r) {
      const int c_in = r / L, lvl = r % L + 1;
      uint64_t* row = bsk + ((size_t)i * R + r) * (k + 1) * N;
      uint64_t* body = row + (size_t)k * N;
      for (int t = 0; t < N; ++t) body[t] = 0;
      for (int j = 0; j < k; ++j) {
        uint64_t* A = row + (size_t)j * N;
        stream_init(&sm, &K, tag_mask, ((uint64_t)i * R + r) * k + j);
        for (int t = 0; t < N; ++t) A[t] = stream_word(&sm, (uint64_t)t);
        for (int t = 0; t < N; ++t) S[t] = s_big[j * N + t];
        negacyclic_mac(A, S, body, N, scratch);
      }
      stream_init(&sn, &K, tag_noise, (uint64_t)i * R + r);
      for (int t = 0; t < N; ++t) body[t] += (uint64_t)tuniform(stream_word(&sn, (uint64_t)t), P->glwe_noise_bits);
      if (msg[i]) row[(size_t)c_in * N] += ((uint64_t)1) << (64 - lvl * beta);
    }
    free(scratch);
    free(S);
  }
}

/* Multi-bit keys (group 2): the LWE coefficients go in
 * pairs (s1, s2) = (s[2j], s[2j+1]), s2 = 0 past n; pair j has three GGSWs,
 * of s1(1-s2), (1-s1)s2 and s1 s2 (the subsets {1}, {2}, {1,2}). */
static int gadget_group(const ref_params* P, int which) {
  const int g = which == 1 ? P->pbs_fast_group : which == 2 ? P->pbs_fast2_group
              : which == 3 ? P->pbs_mid_group : which == 4 ? P->pbs_mid2_group
              : which == 5 ? P->pbs_mid0_group : 1;
  return g == 2 ? 2 : 1;
}
/* gadget `which`: 0 main, 1 fast, 2 fast2, 3 mid, 4 mid2, 5 mid0 (level 0: absent) */
#define NGAD 6
static int gadget_level(const ref_params* P, int which) {
  switch (which) {
    case 0: return P->pbs_level;
    case 1: return P->pbs_fast_level;
    case 2: return P->pbs_fast2_level;
    case 3: return P->pbs_mid_level;
    case 4: return P->pbs_mid2_level;
    case 5: return P->pbs_mid0_level;
  }
  return 0;
}
static int gadget_base_log(const ref_params* P, int which) {
  switch (which) {
    case 0: return P->pbs_base_log;
    case 1: return P->pbs_fast_base_log;
    case 2: return P->pbs_fast2_base_log;
    case 3: return P->pbs_mid_base_log;
    case 4: return P->pbs_mid2_base_log;
    case 5: return P->pbs_mid0_base_log;
  }
  return 0;
}
static int npairs(const ref_params* P) { return (P->n + 1) / 2; }
static void mb_msgs(const ref_params* P, const uint64_t* s_small, uint64_t* msg) {
  for (int j = 0; j < npairs(P); ++j) {
    const uint64_t s1 = s_small[2 * j], s2 = 2 * j + 1 < P->n ? s_small[2 * j + 1] : 0;
    msg[3 * j] = s1 & (1 - s2);
    msg[3 * j + 1] = (1 - s1) & s2;
    msg[3 * j + 2] = s1 & s2;
  }
}
/* another gadget's bootstrapping key (fhe_keygen with pbs_fast_*,
 * pbs_fast2_*, pbs_mid_*, pbs_mid2_*): same secrets; which = 1: TAG_BSK2_*
 * streams (TAG_MB2_* multi-bit), 2: TAG_BSK3_* (TAG_MB3_*), 3: TAG_BSK4_*,
 * 4: TAG_BSK5_*; ref_bsk2_words words (the bsk layout of that gadget, with 3
 * GGSWs per pair for a multi-bit key) */
size_t ref_bsk2_words(const ref_params* P, int which) {
  const int L = which >= 1 && which < NGAD ? gadget_level(P, which) : 0;
  const size_t ggsws = gadget_group(P, which) == 2 ? 3 * (size_t)npairs(P) : (size_t)P->n;
  return ggsws * (P->k + 1) * L * (P->k + 1) * P->N;
}
int ref_keygen_fast_bsk(const ref_params* P, uint64_t seed, int which, const uint64_t* s_small,
                        const uint64_t* s_big, uint64_t* bsk2) {
  const int L = which >= 1 && which < NGAD ? gadget_level(P, which) : 0;
  if (!L) return -1;
  ref_key K;
  key_from_seed(seed, &K);
  const int bl = gadget_base_log(P, which);
  static const int tmask[NGAD] = {TAG_BSK_MASK, TAG_BSK2_MASK, TAG_BSK3_MASK, TAG_BSK4_MASK, TAG_BSK5_MASK,
                                  TAG_BSK6_MASK};
  static const int tnoise[NGAD] = {TAG_BSK_NOISE, TAG_BSK2_NOISE, TAG_BSK3_NOISE, TAG_BSK4_NOISE, TAG_BSK5_NOISE,
                                   TAG_BSK6_NOISE};
  if (gadget_group(P, which) == 2) {
    uint64_t* msg = (uint64_t*)malloc(8 * 3 * (size_t)npairs(P));
    mb_msgs(P, s_small, msg);
    static const int mmask[NGAD] = {0, TAG_MB2_MASK, TAG_MB3_MASK, TAG_MB4_MASK, TAG_MB5_MASK, TAG_MB6_MASK};
    static const int mnoise[NGAD] = {0, TAG_MB2_NOISE, TAG_MB3_NOISE, TAG_MB4_NOISE, TAG_MB5_NOISE, TAG_MB6_NOISE};
    bsk_gen(P, &K, bl, L, mmask[which], mnoise[which], msg, 3 * npairs(P), s_big, bsk2);
    free(msg);
  } else {
    bsk_gen(P, &K, bl, L, tmask[which], tnoise[which], s_small, P->n, s_big, bsk2);
  }
  return 0;
}

/* s_small[n] (0/1), s_big[kN] (0/1), bsk[ref_bsk_words], ksk[ref_ksk_words] */
int ref_keygen(const ref_params* P, uint64_t seed, uint64_t* s_small, uint64_t* s_big, uint64_t* bsk,
               uint64_t* ksk) {
  ref_key K;
  key_from_seed(seed, &K);
  const int n = P->n, k = P->k, N = P->N;
  ref_stream st;
  stream_init(&st, &K, TAG_SK_SMALL, 0);
  for (int i = 0; i < n; ++i) s_small[i] = stream_word(&st, (uint64_t)i) & 1;
  stream_init(&st, &K, TAG_SK_GLWE, 0);
  for (int i = 0; i < k * N; ++i) s_big[i] = stream_word(&st, (uint64_t)i) & 1;

  bsk_gen(P, &K, P->pbs_base_log, P->pbs_level, TAG_BSK_MASK, TAG_BSK_NOISE, s_small, n, s_big, bsk);

  /* key-switching key big -> small */
  const int KL = P->ks_level;
#pragma omp parallel for schedule(static)
  for (int i = 0; i < k * N; ++i) {
    ref_stream sm, sn;
    for (int l = 0; l < KL; ++l) {
      uint64_t* row = ksk + ((size_t)i * KL + l) * (n + 1);
      stream_init(&sm, &K, TAG_KSK_MASK, (uint64_t)i * KL + l);
      stream_init(&sn, &K, TAG_KSK_NOISE, (uint64_t)i * KL + l);
      uint64_t b = 0;
      for (int t = 0; t < n; ++t) {
        row[t] = stream_word(&sm, (uint64_t)t);
        if (s_small[t]) b += row[t];
      }
      b += (uint64_t)tuniform(stream_word(&sn, 0), P->lwe_noise_bits);
      if (s_big[i]) b += ((uint64_t)1) << (64 - (l + 1) * P->ks_base_log);
      row[n] = b;
    }
  }
  return 0;
}

/* -------------------------------------------------------------- encrypt --- */
/* Encrypt count torus messages msg[c] under s_big (dim kN); ciphertext ids
 * are id0 + c. ct: count x (kN+1) words, layout [a_0..a_{kN-1}, b]. */
void ref_encrypt_raw(const ref_params* P, const uint64_t* s_big, const uint64_t* msg, int64_t count,
                     uint64_t seed, uint64_t id0, uint64_t* ct) {
  ref_key K;
  key_from_seed(seed, &K);
  const int dim = P->k * P->N;
#pragma omp parallel for schedule(static)
  for (int64_t c = 0; c < count; ++c) {
    ref_stream sm, sn;
    stream_init(&sm, &K, TAG_ENC_MASK, id0 + (uint64_t)c);
    stream_init(&sn, &K, TAG_ENC_NOISE, id0 + (uint64_t)c);
    uint64_t* o = ct + (size_t)c * (dim + 1);
    uint64_t b = 0;
    for (int t = 0; t < dim; ++t) {
      o[t] = stream_word(&sm, (uint64_t)t);
      if (s_big[t]) b += o[t];
    }
    b += (uint64_t)tuniform(stream_word(&sn, 0), P->glwe_noise_bits);
    o[dim] = b + msg[c];
  }
}

/* Encode signed integers v at Delta = 2^(64-P) and encrypt. */
void ref_encrypt_ints(const ref_params* P, const uint64_t* s_big, const int64_t* v, int64_t count, uint64_t seed,
                      uint64_t id0, uint64_t* ct) {
  uint64_t* m = (uint64_t*)malloc(8 * (size_t)(count > 0 ? count : 1));
  for (int64_t i = 0; i < count; ++i) m[i] = ((uint64_t)v[i]) << (64 - P->msg_bits);
  ref_encrypt_raw(P, s_big, m, count, seed, id0, ct);
  free(m);
}

/* Packed features (GPU: k_encrypt_packed, k_linear_packed,
 * k_encrypt_linear). The D features of row b fill the first coefficients of
 * G = ceil(D / N) GLWE messages M_g = sum_t v[b][gN + t] Delta X^t; GLWE
 * (b, g) has stream id id0 + b*G + g: A_i[t] = word iN + t of the TAG_ENC_MASK
 * stream, E[t] = TUniform of word t of the TAG_ENC_NOISE stream, and the body
 * B = sum_i A_i S_i + M + E (S_i: the GLWE secret's polynomials, s_big =
 * S_1 .. S_k). Textbook: the body by full negacyclic products. glwe: B x G x
 * (k+1)N words. */
void ref_encrypt_packed(const ref_params* P, const uint64_t* s_big, const int64_t* v, int64_t B, int32_t D,
                        uint64_t seed, uint64_t id0, uint64_t* glwe) {
  ref_key K;
  key_from_seed(seed, &K);
  const int N = P->N, k = P->k, G = (D + N - 1) / N;
#pragma omp parallel for schedule(dynamic)
  for (int64_t bg = 0; bg < B * G; ++bg) {
    const int64_t b = bg / G;
    const int g = (int)(bg % G);
    uint64_t* scratch = (uint64_t*)malloc(8 * (size_t)(16 * N));
    ref_stream sm, sn;
    stream_init(&sm, &K, TAG_ENC_MASK, id0 + (uint64_t)bg);
    stream_init(&sn, &K, TAG_ENC_NOISE, id0 + (uint64_t)bg);
    uint64_t* o = glwe + (size_t)bg * (k + 1) * N;
    uint64_t* body = o + (size_t)k * N;
    for (int t = 0; t < N; ++t) body[t] = 0;
    for (int i = 0; i < k; ++i) {
      for (int t = 0; t < N; ++t) o[(size_t)i * N + t] = stream_word(&sm, (uint64_t)i * N + t);
      negacyclic_mac(o + (size_t)i * N, s_big + (size_t)i * N, body, N, scratch);
    }
    for (int t = 0; t < N; ++t) {
      const int j = g * N + t;
      const uint64_t m = j < D ? ((uint64_t)v[b * D + j]) << (64 - P->msg_bits) : 0;
      body[t] += m + (uint64_t)tuniform(stream_word(&sn, (uint64_t)t), P->glwe_noise_bits);
    }
    free(scratch);
  }
}

/* The leveled dot product on packed GLWEs: for each chunk, the GLWE times
 * W_g = sum_t w[gN + t] X^-t (X^-t = -X^(N-t)), then the LWE of coefficient 0
 * (sample extraction: a_{i,0} = C_i[0], a_{i,u} = -C_i[N-u], b = C_B[0]),
 * summed over the chunks, plus trivial(cst * Delta). out: B x (kN+1). */
void ref_linear_packed(const ref_params* P, const uint64_t* glwe, int64_t B, int32_t D, const int64_t* w, int64_t cst,
                       uint64_t* out) {
  const int N = P->N, k = P->k, G = (D + N - 1) / N, W = k * N + 1;
#pragma omp parallel for schedule(dynamic)
  for (int64_t b = 0; b < B; ++b) {
    uint64_t* scratch = (uint64_t*)malloc(8 * (size_t)(16 * N));
    uint64_t* wp = (uint64_t*)malloc(8 * (size_t)N);
    uint64_t* c = (uint64_t*)malloc(8 * (size_t)N);
    uint64_t* o = out + (size_t)b * W;
    for (int t = 0; t < W; ++t) o[t] = 0;
    for (int g = 0; g < G; ++g) {
      const uint64_t* in = glwe + ((size_t)b * G + g) * (k + 1) * N;
      for (int t = 0; t < N; ++t) wp[t] = 0;
      for (int t = 0; t < N && g * N + t < D; ++t) {
        const uint64_t wt = (uint64_t)w[g * N + t];
        if (t == 0) wp[0] += wt;
        else wp[N - t] -= wt;
      }
      for (int i = 0; i <= k; ++i) {
        for (int t = 0; t < N; ++t) c[t] = 0;
        negacyclic_mac(in + (size_t)i * N, wp, c, N, scratch);
        if (i == k) {
          o[k * N] += c[0];
        } else {
          o[(size_t)i * N] += c[0];
          for (int u = 1; u < N; ++u) o[(size_t)i * N + u] -= c[N - u];
        }
      }
    }
    o[W - 1] += ((uint64_t)cst) << (64 - P->msg_bits);
    free(scratch);
    free(wp);
    free(c);
  }
}

/* Seeded encryption of a document corpus: feature j of
 * document b has stream id id0[b] + j; its mask is the TAG_ENC_MASK stream
 * of the public key `mkey`, its noise the TAG_ENC_NOISE stream of the
 * secret key `nkey`. Only the bodies are produced (B x D). */
void ref_encrypt_seeded(const ref_params* P, const uint64_t* s_big, const int64_t* v, int64_t B, int32_t D,
                        const uint32_t mkey[8], const uint32_t nkey[8], const uint64_t* id0, uint64_t* body) {
  ref_key Km, Kn;
  memcpy(Km.key, mkey, 32);
  memcpy(Kn.key, nkey, 32);
  const int dim = P->k * P->N;
#pragma omp parallel for schedule(static)
  for (int64_t c = 0; c < B * D; ++c) {
    const uint64_t id = id0[c / D] + (uint64_t)(c % D);
    ref_stream sm, sn;
    stream_init(&sm, &Km, TAG_ENC_MASK, id);
    stream_init(&sn, &Kn, TAG_ENC_NOISE, id);
    uint64_t b = 0;
    for (int t = 0; t < dim; ++t)
      if (s_big[t]) b += stream_word(&sm, (uint64_t)t);
    b += (uint64_t)tuniform(stream_word(&sn, 0), P->glwe_noise_bits);
    body[c] = b + (((uint64_t)v[c]) << (64 - P->msg_bits));
  }
}
/* full ciphertexts (B*D x (kN+1)) of a seeded corpus */
void ref_expand_seeded(const ref_params* P, const uint64_t* body, const uint64_t* id0, int64_t B, int32_t D,
                       const uint32_t mkey[8], uint64_t* ct) {
  ref_key Km;
  memcpy(Km.key, mkey, 32);
  const int dim = P->k * P->N;
  for (int64_t c = 0; c < B * D; ++c) {
    ref_stream sm;
    stream_init(&sm, &Km, TAG_ENC_MASK, id0[c / D] + (uint64_t)(c % D));
    uint64_t* o = ct + (size_t)c * (dim + 1);
    for (int t = 0; t < dim; ++t) o[t] = stream_word(&sm, (uint64_t)t);
    o[dim] = body[c];
  }
}
void ref_key_from_seed(uint64_t seed, uint32_t out[8]) {
  ref_key K;
  key_from_seed(seed, &K);
  memcpy(out, K.key, 32);
}

static uint64_t lwe_phase(const uint64_t* ct, const uint64_t* s, int dim) {
  uint64_t acc = ct[dim];
  for (int t = 0; t < dim; ++t)
    if (s[t]) acc -= ct[t];
  return acc;
}
void ref_phase(const uint64_t* ct, const uint64_t* s, int dim, int64_t count, uint64_t* out) {
  for (int64_t c = 0; c < count; ++c) out[c] = lwe_phase(ct + (size_t)c * (dim + 1), s, dim);
}
/* round(phase / 2^(64-P)) as a signed P-bit integer */
static int64_t decode(uint64_t ph, int Pb) {
  uint64_t r = ((ph >> (63 - Pb)) + 1) >> 1;
  r &= (Pb >= 64) ? ~0ull : ((1ull << Pb) - 1);
  if (r >> (Pb - 1)) return (int64_t)r - ((int64_t)1 << Pb);
  return (int64_t)r;
}
void ref_decrypt_ints(const ref_params* P, const uint64_t* s_big, const uint64_t* ct, int64_t count, int64_t* out) {
  const int dim = P->k * P->N;
  for (int64_t c = 0; c < count; ++c) out[c] = decode(lwe_phase(ct + (size_t)c * (dim + 1), s_big, dim), P->msg_bits);
}

/* --------------------------------------------------------------- linear --- */
/* out[b] = sum_j w[j] * ct[b, j] + trivial(cst * Delta); cts of dim kN. */
void ref_linear(const ref_params* P, const uint64_t* ct, int64_t B, int32_t D, const int64_t* w, int64_t cst,
                uint64_t* out) {
  const int W = P->k * P->N + 1;
#pragma omp parallel for schedule(static)
  for (int64_t b = 0; b < B; ++b) {
    uint64_t* o = out + (size_t)b * W;
    for (int t = 0; t < W; ++t) o[t] = 0;
    for (int j = 0; j < D; ++j) {
      const uint64_t* x = ct + ((size_t)b * D + j) * W;
      const uint64_t wj = (uint64_t)w[j];
      for (int t = 0; t < W; ++t) o[t] += wj * x[t];
    }
    o[W - 1] += ((uint64_t)cst) << (64 - P->msg_bits);
  }
}

/* ------------------------------------------------------------ keyswitch --- */
/* closest multiple of 2^(64 - L*bl), as L balanced digits d[0..L-1] (level 1 first) */
static void decompose(uint64_t x, int bl, int L, int64_t* d) {
  const int prec = L * bl;
  uint64_t r = ((x >> (63 - prec)) + 1) >> 1;
  r &= (prec >= 64) ? ~0ull : ((1ull << prec) - 1);
  int64_t v = (int64_t)r;
  const int64_t B = (int64_t)1 << bl;
  for (int l = L; l >= 1; --l) {
    int64_t dd = v & (B - 1);
    v >>= bl;
    if (dd >= B / 2) { dd -= B; v += 1; }
    d[l - 1] = dd;
  }
}
void ref_decompose(uint64_t x, int bl, int L, int64_t* d) { decompose(x, bl, L, d); }
/* The key switch's digits: the same closest multiple, as L
 * digits in [-B/2, B/2], a tie at B/2 taking the sign of a coin: the digit
 * of LSB-first index j (level L - j) is -B/2 (with a carry) when bit
 * 62 - prec - j of x is 1. Those bits lie below the rounding bit, so for
 * uniform x they are fair and independent of the rounded value: every
 * digit is then zero-mean with E[d^2] = (B^2 + 2) / 12, the noise model's
 * factor, where digits in [-B/2, B/2) have mean -1/2 and put a
 * key-dependent bias 0.5 * sum(KSK noise) on every key switch. (The lowest
 * coin, bit 63 - prec - L, must lie at or above any shift of the input:
 * shift <= 63 - prec - L. fhe_ctx_create checks prec + L + msg_bits <= 64,
 * the sign extraction shifting by at most msg_bits - 1, and
 * fhe_keyswitch_batch refuses larger shifts.) */
static void decompose_ks(uint64_t x, int bl, int L, int64_t* d) {
  const int prec = L * bl;
  uint64_t v = ((x >> (63 - prec)) + 1) >> 1;
  const uint64_t B = (uint64_t)1 << bl, half = B >> 1;
  for (int l = L; l >= 1; --l) {
    const uint64_t low = v & (B - 1);
    v >>= bl;
    const uint64_t coin = (x >> (62 - prec - (L - l))) & 1;
    if (low > half || (low == half && coin)) {
      d[l - 1] = (int64_t)low - (int64_t)B;
      v += 1;
    } else {
      d[l - 1] = (int64_t)low;
    }
  }
}
void ref_decompose_ks(uint64_t x, int bl, int L, int64_t* d) { decompose_ks(x, bl, L, d); }

/* The key switch uses each KSK word rounded to the nearest multiple of 2^R,
 * R = 8 floor((lwe_noise_bits - 6) / 8) (at most 40, 0 below 14 bits): the
 * rounding error is below 2^-7 of the KSK's TUniform noise, and the GPU's i8
 * matrix-core key switch needs 8 - R / 8 byte planes of it (libfheicp
 * ks_round_bits / k_server.h ks_round). */
static int ks_round_bits(const ref_params* P) {
  if (P->lwe_noise_bits < 14) return 0;
  const int r = (P->lwe_noise_bits - 6) / 8;
  return 8 * (r < 5 ? r : 5);
}
static uint64_t ks_round(uint64_t x, int R) { return R ? (x + (1ull << (R - 1))) & ~((1ull << R) - 1) : x; }

static void keyswitch1(const ref_params* P, const uint64_t* ksk, const uint64_t* in, uint64_t* out) {
  const int n = P->n, dimb = P->k * P->N, KL = P->ks_level, R = ks_round_bits(P);
  int64_t d[64];
  for (int t = 0; t < n; ++t) out[t] = 0;
  out[n] = in[dimb];
  for (int i = 0; i < dimb; ++i) {
    decompose_ks(in[i], P->ks_base_log, KL, d);
    for (int l = 0; l < KL; ++l) {
      if (!d[l]) continue;
      const uint64_t* row = ksk + ((size_t)i * KL + l) * (n + 1);
      const uint64_t dd = (uint64_t)d[l];
      for (int t = 0; t <= n; ++t) out[t] -= dd * ks_round(row[t], R);
    }
  }
}
void ref_keyswitch(const ref_params* P, const uint64_t* ksk, const uint64_t* in, int64_t count, uint64_t* out) {
#pragma omp parallel for schedule(static)
  for (int64_t c = 0; c < count; ++c)
    keyswitch1(P, ksk, in + (size_t)c * (P->k * P->N + 1), out + (size_t)c * (P->n + 1));
}

/* ------------------------------------------------------- blind rotation --- */
static int ilog2(int x) { int r = 0; while ((1 << r) < x) r++; return r; }
/* round(a * 2N / 2^64) mod 2N */
static uint32_t modswitch(uint64_t a, int log2N2) {
  return (uint32_t)((((a >> (63 - log2N2)) + 1) >> 1) & ((1ull << log2N2) - 1));
}

/* Test vector TV_j, j in [0, N), extended negacyclically: a staircase
 * base + (j >> shift) * step (step 0 = constant), or, with a table (lut !=
 * NULL, fhe_pbs_table_batch), box m = (j + half box) >> log_box holding
 * lut[m] * delta, and the top half box holding -lut[0] * delta (its
 * negacyclic image is the half box just below phase 0). */
typedef struct {
  uint64_t base, step;
  int shift;
  const int64_t* lut;
  int lut_count, log_box;
  uint64_t delta;
} tv_desc;
static uint64_t tv_at(const tv_desc* tv, uint32_t idx, int N) {
  const uint32_t j = idx & (uint32_t)(N - 1);
  uint64_t v;
  if (tv->lut) {
    const uint32_t m = (j + (1u << (tv->log_box - 1))) >> tv->log_box;
    v = m < (uint32_t)tv->lut_count ? (uint64_t)tv->lut[m] * tv->delta : (uint64_t)0 - (uint64_t)tv->lut[0] * tv->delta;
  } else {
    v = tv->base + (uint64_t)(j >> tv->shift) * tv->step;
  }
  return idx < (uint32_t)N ? v : (uint64_t)0 - v;
}

/* acc += X^a * p - p (negacyclic, a in [0, 2N)) */
static void add_rot_minus(const uint64_t* p, uint32_t a, int N, uint64_t* acc) {
  for (int t = 0; t < N; ++t) {
    const uint32_t idx = (uint32_t)(t - (int)a) & (uint32_t)(2 * N - 1);
    const uint64_t rot = idx < (uint32_t)N ? p[idx] : (uint64_t)0 - p[idx - N];
    acc[t] += rot - p[t];
  }
}

/* Multi-bit blind rotation (group 2), exact: per pair j with
 * a1, a2 (a2 = 0 past n) switched to 2N and a12 the switch of the exact sum
 * of the two mask words (not a1 + a2: one rounding, not two, when both key
 * bits are set),
 *   G_r = sum_S (X^{a_S} - 1) GGSW_S[r]   (exact, mod 2^64),
 *   ACC += sum_r digits_r(ACC) * G_r,
 * the algebra of k_blind_rotate_mb (the GPU forms the same products in the
 * FFT domain). */
static void pbs1_mb(const ref_params* P, const uint64_t* bsk, const uint64_t* small, uint64_t* acc, uint64_t* dig,
                    uint64_t* scratch, uint64_t* G) {
  const int n = P->n, k = P->k, N = P->N, L = P->pbs_level, R = rows(P), bl = P->pbs_base_log;
  const int lg = ilog2(2 * N);
  const size_t ggsw = (size_t)R * (k + 1) * N;
  int64_t d[64];
  for (int j = 0; j < npairs(P); ++j) {
    const uint32_t a1 = modswitch(small[2 * j], lg);
    const uint32_t a2 = 2 * j + 1 < n ? modswitch(small[2 * j + 1], lg) : 0;
    const uint32_t a12 = 2 * j + 1 < n ? modswitch(small[2 * j] + small[2 * j + 1], lg) : a1;
    const uint32_t aS[3] = {a1, a2, a12};
    if (!a1 && !a2 && !a12) continue;  /* a12 can be +-1 with a1 = a2 = 0 */
    for (size_t x = 0; x < ggsw; ++x) G[x] = 0;
    for (int S = 0; S < 3; ++S) {
      if (!aS[S]) continue;
      const uint64_t* B = bsk + ((size_t)j * 3 + S) * ggsw;
      for (size_t q = 0; q < (size_t)R * (k + 1); ++q) add_rot_minus(B + q * N, aS[S], N, G + q * N);
    }
    for (int c = 0; c <= k; ++c)
      for (int t = 0; t < N; ++t) {
        decompose(acc[(size_t)c * N + t], bl, L, d);
        for (int l = 0; l < L; ++l) dig[((size_t)c * L + l) * N + t] = (uint64_t)d[l];
      }
    for (int r = 0; r < R; ++r)
      for (int o = 0; o <= k; ++o)
        negacyclic_mac(dig + (size_t)r * N, G + ((size_t)r * (k + 1) + o) * N, acc + (size_t)o * N, N, scratch);
  }
}

/* Bootstrap one small LWE (dim n) with test vector tv; sample extract
 * coefficient 0. out: kN + 1 words under s_big. group 2: the multi-bit
 * rotation with a multi-bit key. */
static void pbs1g(const ref_params* P, int group, const uint64_t* bsk, const uint64_t* small, const tv_desc* tv,
                  uint64_t* out, uint64_t* work);
static void pbs1(const ref_params* P, const uint64_t* bsk, const uint64_t* small, const tv_desc* tv, uint64_t* out,
                 uint64_t* work) {
  pbs1g(P, 1, bsk, small, tv, out, work);
}
static void pbs1g(const ref_params* P, int group, const uint64_t* bsk, const uint64_t* small, const tv_desc* tv,
                  uint64_t* out, uint64_t* work) {
  const int n = P->n, k = P->k, N = P->N, L = P->pbs_level, R = rows(P), bl = P->pbs_base_log;
  const int lg = ilog2(2 * N);
  uint64_t* acc = work;                           /* (k+1)N */
  uint64_t* dig = acc + (size_t)(k + 1) * N;      /* R*N */
  uint64_t* scratch = dig + (size_t)R * N;        /* 16N */
  int64_t d[64];
  const uint32_t bt = modswitch(small[n], lg);
  for (int t = 0; t < k * N; ++t) acc[t] = 0;
  for (int t = 0; t < N; ++t) {
    const uint32_t idx = (uint32_t)(t + bt) & (2 * N - 1);
    acc[(size_t)k * N + t] = tv_at(tv, idx, N);
  }
  if (group == 2) pbs1_mb(P, bsk, small, acc, dig, scratch, scratch + 16 * (size_t)N);
  for (int i = 0; group != 2 && i < n; ++i) {
    const uint32_t ai = modswitch(small[i], lg);
    if (ai == 0) continue;
    /* digits of X^{a_i} ACC - ACC */
    for (int c = 0; c <= k; ++c) {
      const uint64_t* f = acc + (size_t)c * N;
      for (int t = 0; t < N; ++t) {
        const uint32_t idx = (uint32_t)(t - (int)ai) & (2 * N - 1);
        const uint64_t rot = idx < (uint32_t)N ? f[idx] : (uint64_t)0 - f[idx - N];
        decompose(rot - f[t], bl, L, d);
        for (int l = 0; l < L; ++l) dig[((size_t)c * L + l) * N + t] = (uint64_t)d[l];
      }
    }
    /* ACC += sum_r dig_r * BSK_i[r] */
    const uint64_t* G = bsk + (size_t)i * R * (k + 1) * N;
    for (int r = 0; r < R; ++r)
      for (int o = 0; o <= k; ++o)
        negacyclic_mac(dig + (size_t)r * N, G + ((size_t)r * (k + 1) + o) * N, acc + (size_t)o * N, N, scratch);
  }
  for (int j = 0; j < k; ++j) {
    const uint64_t* A = acc + (size_t)j * N;
    out[(size_t)j * N] = A[0];
    for (int t = 1; t < N; ++t) out[(size_t)j * N + t] = (uint64_t)0 - A[N - t];
  }
  out[(size_t)k * N] = acc[(size_t)k * N];
}
static size_t pbs_work_words(const ref_params* P) {
  /* acc | digits | scratch (16N) | the multi-bit combined GGSW (R (k+1) N) */
  return (size_t)(P->k + 1) * P->N + (size_t)rows(P) * P->N + 16 * (size_t)P->N +
         (size_t)rows(P) * (P->k + 1) * P->N;
}

/* Bootstrap count small LWEs with a constant test vector (amplitude tv). */
void ref_pbs_const(const ref_params* P, const uint64_t* bsk, const uint64_t* small, int64_t count, uint64_t tv,
                   uint64_t* out) {
#pragma omp parallel
  {
    uint64_t* work = (uint64_t*)malloc(8 * pbs_work_words(P));
    const tv_desc d = {tv, 0, 0, NULL, 0, 0, 0};
#pragma omp for schedule(dynamic)
    for (int64_t c = 0; c < count; ++c)
      pbs1(P, bsk, small + (size_t)c * (P->n + 1), &d, out + (size_t)c * (P->k * P->N + 1), work);
    free(work);
  }
}

/* ref_pbs_const on gadget g (fhe_pbs_gadget_batch): 0 = main with bsk, 1..4
 * = the fast / fast2 / mid / mid2 gadget with its key from
 * ref_keygen_fast_bsk, on the classic or the multi-bit rotation by that
 * gadget's group. */
void ref_pbs_gadget(const ref_params* P0, const uint64_t* bsk, const uint64_t* small, int64_t count, int gadget,
                    uint64_t tv, uint64_t* out) {
  ref_params P = *P0;
  int group = 1;
  if (gadget >= 1 && gadget < NGAD && gadget_level(P0, gadget)) {
    P.pbs_base_log = gadget_base_log(P0, gadget); P.pbs_level = gadget_level(P0, gadget);
    group = gadget_group(P0, gadget);
  }
#pragma omp parallel
  {
    uint64_t* work = (uint64_t*)malloc(8 * pbs_work_words(&P));
    const tv_desc d = {tv, 0, 0, NULL, 0, 0, 0};
#pragma omp for schedule(dynamic)
    for (int64_t c = 0; c < count; ++c)
      pbs1g(&P, group, bsk, small + (size_t)c * (P.n + 1), &d, out + (size_t)c * (P.k * P.N + 1), work);
    free(work);
  }
}

/* Bootstrap with a staircase test vector over 2^log_slots slots of the half
 * torus (fhe_pbs_lut_batch semantics). */
void ref_pbs_lut(const ref_params* P, const uint64_t* bsk, const uint64_t* small, int64_t count, uint64_t base,
                 uint64_t step, int log_slots, uint64_t* out) {
#pragma omp parallel
  {
    uint64_t* work = (uint64_t*)malloc(8 * pbs_work_words(P));
    const tv_desc d = {base, step, ilog2(P->N) - log_slots, NULL, 0, 0, 0};
#pragma omp for schedule(dynamic)
    for (int64_t c = 0; c < count; ++c)
      pbs1(P, bsk, small + (size_t)c * (P->n + 1), &d, out + (size_t)c * (P->k * P->N + 1), work);
    free(work);
  }
}

/* Bootstrap with a table test vector (fhe_pbs_table_batch semantics): the
 * input encrypts m in [0, 2^lut_bits) at 2^(63 - lut_bits), the output lut[m]
 * at 2^(64 - msg_bits). */
void ref_pbs_table(const ref_params* P, const uint64_t* bsk, const uint64_t* small, int64_t count, const int64_t* lut,
                   int lut_bits, uint64_t* out) {
#pragma omp parallel
  {
    uint64_t* work = (uint64_t*)malloc(8 * pbs_work_words(P));
    tv_desc d = {0, 0, 0, lut, 1 << lut_bits, ilog2(P->N) - lut_bits, 0};
    d.delta = 1ull << (64 - P->msg_bits);
#pragma omp for schedule(dynamic)
    for (int64_t c = 0; c < count; ++c)
      pbs1(P, bsk, small + (size_t)c * (P->n + 1), &d, out + (size_t)c * (P->k * P->N + 1), work);
    free(work);
  }
}

/* ref_pbs_table on gadget g (fhe_pbs_table_gadget_batch): 0 = the classic
 * main gadget with bsk, 1..5 a gadget of ref_keygen_fast_bsk on the rotation
 * of its group (the multi-bit one for the shipped table gadgets). */
void ref_pbs_table_gadget(const ref_params* P0, const uint64_t* bsk, const uint64_t* small, int64_t count, int gadget,
                          const int64_t* lut, int lut_bits, uint64_t* out) {
  ref_params P = *P0;
  int group = 1;
  if (gadget >= 1 && gadget < NGAD && gadget_level(P0, gadget)) {
    P.pbs_base_log = gadget_base_log(P0, gadget); P.pbs_level = gadget_level(P0, gadget);
    group = gadget_group(P0, gadget);
  }
#pragma omp parallel
  {
    uint64_t* work = (uint64_t*)malloc(8 * pbs_work_words(&P));
    tv_desc d = {0, 0, 0, lut, 1 << lut_bits, ilog2(P.N) - lut_bits, 0};
    d.delta = 1ull << (64 - P.msg_bits);
#pragma omp for schedule(dynamic)
    for (int64_t c = 0; c < count; ++c)
      pbs1g(&P, group, bsk, small + (size_t)c * (P.n + 1), &d, out + (size_t)c * (P.k * P.N + 1), work);
    free(work);
  }
}

/* modswitched (a~, b~) of small LWEs, for tests */
void ref_modswitch(const ref_params* P, const uint64_t* small, int64_t count, uint32_t* out) {
  const int lg = ilog2(2 * P->N);
  for (int64_t c = 0; c < count * (P->n + 1); ++c) out[c] = modswitch(small[c], lg);
}

/* ------------------------------------------------------- bit extraction --- */
/* LSB-first extraction of the P bits of v from ct_v (encrypting v * 2^(64-P)),
 * DESIGN.md §3.4. Iteration i: sh = ct_v * 2^(P-1-i) (+2^62 on the body),
 * KS, PBS with constant tv = 2^(63-P+i), bit_i = trivial(tv) - PBS (encrypts
 * bit_i * 2^(64-P+i)), ct_v -= bit_i, refreshed += bit_i.
 * refreshed[count x (kN+1)] encrypts v; sign[count x (kN+1)] is bit P-1.
 * ct_v is consumed (overwritten). */
void ref_bit_extract(const ref_params* P, const uint64_t* bsk, const uint64_t* ksk, uint64_t* ct_v, int64_t count,
                     uint64_t* refreshed, uint64_t* sign) {
  const int Wb = P->k * P->N + 1, Pb = P->msg_bits;
#pragma omp parallel
  {
    uint64_t* work = (uint64_t*)malloc(8 * pbs_work_words(P));
    uint64_t* sh = (uint64_t*)malloc(8 * (size_t)Wb);
    uint64_t* sm = (uint64_t*)malloc(8 * (size_t)(P->n + 1));
    uint64_t* ob = (uint64_t*)malloc(8 * (size_t)Wb);
#pragma omp for schedule(dynamic)
    for (int64_t c = 0; c < count; ++c) {
      uint64_t* cv = ct_v + (size_t)c * Wb;
      uint64_t* acc = refreshed + (size_t)c * Wb;
      for (int t = 0; t < Wb; ++t) acc[t] = 0;
      for (int i = 0; i < Pb; ++i) {
        const int s = Pb - 1 - i;
        for (int t = 0; t < Wb; ++t) sh[t] = cv[t] << s;
        sh[Wb - 1] += 1ull << 62;
        keyswitch1(P, ksk, sh, sm);
        const uint64_t tv = 1ull << (63 - Pb + i);
        const tv_desc d = {tv, 0, 0, NULL, 0, 0, 0};
        pbs1(P, bsk, sm, &d, ob, work);
        for (int t = 0; t < Wb - 1; ++t) ob[t] = (uint64_t)0 - ob[t];
        ob[Wb - 1] = tv - ob[Wb - 1];
        for (int t = 0; t < Wb; ++t) { cv[t] -= ob[t]; acc[t] += ob[t]; }
        if (i == Pb - 1) memcpy(sign + (size_t)c * Wb, ob, 8 * (size_t)Wb);
      }
    }
    free(work); free(sh); free(sm); free(ob);
  }
}

/* ------------------------------------------------------------ sign ----- */
/* One round on ct_v: sh = (ct_v << shift) + add on the body, KS, PBS with tv;
 * mode 1: d = trivial(tv.base) - PBS; mode 2: d = PBS; then ct_v -= d. */
static void sign_round_g(const ref_params* P, int group, const uint64_t* bsk, const uint64_t* ksk, uint64_t* cv,
                         int shift, uint64_t add, const tv_desc* tv, int mode, uint64_t* sh, uint64_t* sm,
                         uint64_t* ob, uint64_t* work) {
  const int Wb = P->k * P->N + 1;
  for (int t = 0; t < Wb; ++t) sh[t] = cv[t] << shift;
  sh[Wb - 1] += add;
  keyswitch1(P, ksk, sh, sm);
  pbs1g(P, group, bsk, sm, tv, ob, work);
  if (mode == 1) {
    for (int t = 0; t < Wb - 1; ++t) ob[t] = (uint64_t)0 - ob[t];
    ob[Wb - 1] = tv->base - ob[Wb - 1];
  }
  for (int t = 0; t < Wb; ++t) cv[t] -= ob[t];
}
static void sign_round(const ref_params* P, const uint64_t* bsk, const uint64_t* ksk, uint64_t* cv, int shift,
                       uint64_t add, const tv_desc* tv, int mode, uint64_t* sh, uint64_t* sm, uint64_t* ob,
                       uint64_t* work) {
  sign_round_g(P, 1, bsk, ksk, cv, shift, add, tv, mode, sh, sm, ob, work);
}

/* Plan of the sign extraction: digit width d and the number
 * j of leading bootstraps on the main gadget (the rest on the fast one).
 * Round r decides on v << shift_r with margin 2^mlog_r; every earlier
 * bootstrap's output variance is amplified by 4^shift_r, the key-switch and
 * modulus-switch variances are not. Without a fast gadget: the explicit
 * sign_digit_bits, else d = 4 if its worst round keeps >= 9.2 sigma, else 3;
 * j = all rounds. With one: the widest d (or the explicit one) and the fewest
 * main rounds keeping every round at 9.2 sigma. */
static double tu_var(int b) { return (ldexp(1.0, 2 * b + 1) + 1.0) / 6.0; }

/* Bootstrap output variance: GGSW key noise + gadget rounding (counted over
 * all n steps) + the f64 FFT's arithmetic error per step and output
 * coefficient, C_FFT * rows * N * B^2 / 144 * 2^-106 (the product's variance
 * times the f64 unit roundoff squared; C_FFT = 16 bounds the 11.6-13.8
 * measured on every MI355X kernel instance, tests/test_gpu_noise.py), plus
 * the 2^32 output rounding of the 32-bit-accumulator kernels (L*beta <= 31);
 * both key-weighted like the gadget rounding. */
#define C_FFT 16.0
/* group 2 (multi-bit): three GGSWs per pair, each times
 * X^a - 1 (3x the key noise), one rounding per pair times X^e - 1 (the same
 * total), three subsets' products (3x the FFT error), half the 2^32 output
 * roundings */
static double pbs_variance(const ref_params* P, int base_log, int L, int group) {
  const double beta = ldexp(1.0, base_log);
  const double rows = (double)L * (P->k + 1) * P->N;
  double key = (double)P->n * rows * (beta * beta + 2) / 12.0 * tu_var(P->glwe_noise_bits) / ldexp(1.0, 128);
  const double steps = (double)P->n * (1 + P->k * P->N / 2.0);
  const double fft = C_FFT * rows * beta * beta / 144.0 * ldexp(1.0, -106);
  const double out32 = base_log * L <= 31 ? ldexp(1.0, -64) / 12.0 : 0.0;
  double arith = fft + out32;
  if (group == 2) {
    key *= 3.0;
    arith = 3.0 * fft + 0.5 * out32;
  }
  return key + steps / (12.0 * pow(beta, 2.0 * L)) + steps * arith;
}
/* key switch + modulus switch of a bootstrap on a rotation of `group`: the
 * classic one rounds every set key bit's exponent and the body's (1/12
 * each); the multi-bit one (pbs1_mb) rounds the active subset's exponent
 * from the exact sum, one rounding per pair with a set bit (3/4 of the full
 * pairs, 1/2 of a lone last coefficient) */
static double fixed_variance_g(const ref_params* P, int group) {
  const double bk = ldexp(1.0, P->ks_base_log);
  const double ks = (double)P->k * P->N * P->ks_level * (bk * bk + 2) / 12.0 * tu_var(P->lwe_noise_bits) /
                        ldexp(1.0, 128) +
                    P->k * P->N / 2.0 * ldexp(1.0, -2 * P->ks_level * P->ks_base_log) / 12.0;
  const double per = group == 2 ? (P->n / 2) * 0.75 / 12.0 + (P->n % 2) * 0.5 / 12.0 + 1.0 / 12.0
                                : (P->n / 2.0 + 1) / 12.0;
  return ks + per / ((2.0 * P->N) * (2.0 * P->N));
}
static double fixed_variance(const ref_params* P) { return fixed_variance_g(P, 1); }
/* rounds of the extraction in order: (shift, log2 margin); returns the count */
static int plan_rounds(int Pb, int d, int* shift, int* mlog) {
  int R = 0, b = 0;
  const int m = Pb - d;
  for (; b + d <= m; b += d)
    for (int t = 0; t < 2; ++t) { shift[R] = Pb - b - d; mlog[R++] = -(d + 1); }
  if (m - b >= 3) {
    const int c = m - b;
    for (int t = 0; t < 2; ++t) { shift[R] = Pb - b - c; mlog[R++] = -(c + 1); }
    b = m;
  }
  for (; b < m; ++b) { shift[R] = Pb - b - 1; mlog[R++] = -2; }
  shift[R] = 0; mlog[R++] = -(d + 1);
  return R;
}
/* worst margin (sigmas) when round r runs on gadget sched[r] */
static double plan_margin(const ref_params* P, int d, const int* sched) {
  int sh[64], ml[64];
  const int R = plan_rounds(P->msg_bits, d, sh, ml);
  double var[NGAD];
  for (int g = 0; g < NGAD; ++g)
    var[g] = gadget_level(P, g) ? pbs_variance(P, gadget_base_log(P, g), gadget_level(P, g), gadget_group(P, g)) : 0.0;
  double fx[NGAD];
  for (int g = 0; g < NGAD; ++g) fx[g] = fixed_variance_g(P, gadget_group(P, g));
  double acc = 0, worst = INFINITY;
  for (int r = 0; r < R; ++r) {
    const double m = ldexp(1.0, ml[r]) / sqrt(acc * ldexp(1.0, 2 * sh[r]) + fx[sched[r]]);
    if (m < worst) worst = m;
    acc += var[sched[r]];
  }
  /* the last bootstrap's output is the sign ciphertext: decryptable at 1/4 */
  const double ml_last = 0.25 / sqrt(var[sched[R - 1]]);
  return ml_last < worst ? ml_last : worst;
}
/* The plan: digit width d and the gadget of every bootstrap (sched, returns
 * R). With fast gadgets, along the ladder main, mid, mid2, fast, fast2 (those
 * present) each gadget takes the fewest leading rounds for which the next one
 * on all remaining rounds keeps every decision at 9.2 sigma; the last takes
 * the rest. */
static int sign_schedule(const ref_params* P, int* d_out, int* sched) {
  int sh[64], ml[64];
  const int Pb = P->msg_bits, d4 = Pb < 4 ? Pb : 4;
  if (Pb < 4) {
    *d_out = 0;
    for (int r = 0; r < Pb; ++r) sched[r] = 0;
    return Pb;
  }
  int dd = 3;
  if (P->pbs_fast_level) {
    int lad[NGAD], m = 0;
    const int order[5] = {5, 3, 4, 1, 2};
    lad[m++] = 0;
    for (int i = 0; i < 5; ++i)
      if (gadget_level(P, order[i])) lad[m++] = order[i];
    const int first = P->sign_digit_bits ? (P->sign_digit_bits < Pb ? P->sign_digit_bits : Pb) : d4;
    const int last = P->sign_digit_bits ? first : 3;
    for (int d = first; d >= last; --d) {
      const int R = plan_rounds(Pb, d, sh, ml);
      int start = 0, ok = 1;
      for (int i = 0; i + 1 < m; ++i) {
        int c = start;
        for (; c <= R; ++c) {
          for (int r = start; r < R; ++r) sched[r] = r < c ? lad[i] : lad[i + 1];
          if (plan_margin(P, d, sched) >= 9.2) break;
        }
        if (c > R) { ok = 0; break; } /* the main gadget alone cannot: narrower d */
        start = c;
      }
      if (ok) { *d_out = d; return R; }
    }
    dd = last;
  } else if (P->sign_digit_bits) {
    dd = P->sign_digit_bits < Pb ? P->sign_digit_bits : Pb;
  } else {
    /* the worst round of a single-gadget plan: the staircase round of the
     * lowest digit, the preceding bootstrap amplified by 4^(P-d) */
    const double v = pbs_variance(P, P->pbs_base_log, P->pbs_level, 1) * ldexp(1.0, 2 * (Pb - d4)) + fixed_variance(P);
    if (ldexp(1.0, -(d4 + 1)) / sqrt(v) >= 9.2) dd = d4;
  }
  *d_out = dd;
  const int R = plan_rounds(Pb, dd, sh, ml);
  for (int r = 0; r < R; ++r) sched[r] = 0;
  return R;
}
/* (d, j1, j2): the leading main-gadget bootstraps j1 and the first fast2
 * one j2 (R without one) of sign_schedule */
static void sign_plan(const ref_params* P, int* d_out, int* j1_out, int* j2_out) {
  int sched[64];
  const int R = sign_schedule(P, d_out, sched);
  int j1 = 0, j2 = R;
  while (j1 < R && sched[j1] == 0) ++j1;
  while (j2 > 0 && sched[j2 - 1] == 2) --j2;
  *j1_out = j1; *j2_out = j2;
}
static int digit_bits(const ref_params* P) {
  int d, j1, j2;
  sign_plan(P, &d, &j1, &j2);
  return d;
}

/* the bootstrap gadget and key of the next round (sign_schedule) */
typedef struct {
  const ref_params* P;
  ref_params Pf[NGAD - 1]; /* P seen through gadget 1..5 */
  const uint64_t* bsk[NGAD];
  int sched[64];
  int r;
} gadget_sched;
static int sched_next(gadget_sched* g, const ref_params** Pr, const uint64_t** bk) {
  const int gi = g->sched[g->r++];
  *Pr = gi ? &g->Pf[gi - 1] : g->P;
  *bk = g->bsk[gi];
  return gi ? gadget_group(g->P, gi) : 1;
}

/* One c-bit digit [b, b+c) of the value in cv: a sign bootstrap of its top bit
 * (v << (P-b-c), centred by 2^(63-c), tv 2^(62-P+b+c)), then a
 * 2^(c-1)-slot staircase of its c-1 low bits (step 2^(64-P+b)). */
static void digit_rounds(gadget_sched* g, const uint64_t* ksk, uint64_t* cv, int b, int c, uint64_t* sh, uint64_t* sm,
                         uint64_t* ob, uint64_t* work) {
  const ref_params* Pr;
  const uint64_t* bk;
  const int Pb = g->P->msg_bits, lgN = ilog2(g->P->N);
  const tv_desc hi = {1ull << (62 - Pb + b + c), 0, 0, NULL, 0, 0, 0};
  int grp = sched_next(g, &Pr, &bk);
  sign_round_g(Pr, grp, bk, ksk, cv, Pb - b - c, 1ull << (63 - c), &hi, 1, sh, sm, ob, work);
  const tv_desc lo = {0, 1ull << (64 - Pb + b), lgN - (c - 1), NULL, 0, 0, 0};
  grp = sched_next(g, &Pr, &bk);
  sign_round_g(Pr, grp, bk, ksk, cv, Pb - b - c, 1ull << (63 - c), &lo, 2, sh, sm, ob, work);
}

/* Sign of the P-bit value in ct_v with d-bit digits (the
 * algorithm of fhe_sign_batch): clear the low m = P - d bits LSB-first, full
 * digits [b, b+d) by digit_rounds, a leftover of >= 3 bits as one shorter
 * digit, of 1-2 bits by single-bit rounds; then the sign of the top d bits
 * (centred by 2^(63-d), tv 2^62). sign[count x (kN+1)] encrypts [v < 0] at
 * 2^63; ct_v is consumed. keys[g - 1] is the key of gadget g = 1..5 (fast,
 * fast2, mid, mid2, mid0); round r runs on gadget sign_schedule[r]; a NULL key
 * plans as if that gadget were not set (with the ones that need it). */
void ref_sign_extract_keys(const ref_params* P0, const uint64_t* bsk, const uint64_t* const* keys,
                           const uint64_t* ksk, uint64_t* ct_v, int64_t count, uint64_t* sign) {
  ref_params Pm = *P0;
  if (!keys[0]) Pm.pbs_fast_base_log = Pm.pbs_fast_level = Pm.pbs_fast_group = 0;
  if (!keys[0] || !keys[1]) Pm.pbs_fast2_base_log = Pm.pbs_fast2_level = Pm.pbs_fast2_group = 0;
  if (!keys[0] || !keys[2]) Pm.pbs_mid_base_log = Pm.pbs_mid_level = Pm.pbs_mid_group = 0;
  if (!Pm.pbs_mid_level || !keys[3]) Pm.pbs_mid2_base_log = Pm.pbs_mid2_level = Pm.pbs_mid2_group = 0;
  if (!Pm.pbs_mid_level || !keys[4]) Pm.pbs_mid0_base_log = Pm.pbs_mid0_level = Pm.pbs_mid0_group = 0;
  const ref_params* P = &Pm;
  const int Wb = P->k * P->N + 1, Pb = P->msg_bits;
  gadget_sched g0;
  g0.P = P;
  g0.r = 0;
  g0.bsk[0] = bsk;
  int d;
  sign_schedule(P, &d, g0.sched);
  size_t ww = pbs_work_words(P);
  for (int g = 1; g < NGAD; ++g) {
    g0.Pf[g - 1] = *P;
    g0.bsk[g] = keys[g - 1];
    if (gadget_level(P, g)) {
      g0.Pf[g - 1].pbs_base_log = gadget_base_log(P, g);
      g0.Pf[g - 1].pbs_level = gadget_level(P, g);
    }
    if (pbs_work_words(&g0.Pf[g - 1]) > ww) ww = pbs_work_words(&g0.Pf[g - 1]);
  }
#pragma omp parallel
  {
    uint64_t* work = (uint64_t*)malloc(8 * ww);
    uint64_t* sh = (uint64_t*)malloc(8 * (size_t)Wb);
    uint64_t* sm = (uint64_t*)malloc(8 * (size_t)(P->n + 1));
    uint64_t* ob = (uint64_t*)malloc(8 * (size_t)Wb);
#pragma omp for schedule(dynamic)
    for (int64_t c = 0; c < count; ++c) {
      uint64_t* cv = ct_v + (size_t)c * Wb;
      gadget_sched g = g0;
      const ref_params* Pr;
      const uint64_t* bk;
      if (Pb < 4) {
        for (int i = 0; i < Pb; ++i) {
          const tv_desc t = {1ull << (63 - Pb + i), 0, 0, NULL, 0, 0, 0};
          sign_round(P, bsk, ksk, cv, Pb - 1 - i, 1ull << 62, &t, 1, sh, sm, ob, work);
        }
      } else {
        const int m = Pb - d;
        int b = 0;
        for (; b + d <= m; b += d) digit_rounds(&g, ksk, cv, b, d, sh, sm, ob, work);
        if (m - b >= 3) {
          digit_rounds(&g, ksk, cv, b, m - b, sh, sm, ob, work);
          b = m;
        }
        for (; b < m; ++b) {
          const tv_desc t = {1ull << (63 - Pb + b), 0, 0, NULL, 0, 0, 0};
          const int grp = sched_next(&g, &Pr, &bk);
          sign_round_g(Pr, grp, bk, ksk, cv, Pb - b - 1, 1ull << 62, &t, 1, sh, sm, ob, work);
        }
        const tv_desc top = {1ull << 62, 0, 0, NULL, 0, 0, 0};
        const int grp = sched_next(&g, &Pr, &bk);
        sign_round_g(Pr, grp, bk, ksk, cv, 0, 1ull << (63 - d), &top, 1, sh, sm, ob, work);
      }
      memcpy(sign + (size_t)c * Wb, ob, 8 * (size_t)Wb);
    }
    free(work); free(sh); free(sm); free(ob);
  }
}
void ref_sign_extract3(const ref_params* P, const uint64_t* bsk, const uint64_t* bsk2, const uint64_t* bsk3,
                       const uint64_t* ksk, uint64_t* ct_v, int64_t count, uint64_t* sign) {
  /* one slot per gadget 1 .. NGAD - 1 (ref_sign_extract_keys reads them all) */
  const uint64_t* keys[NGAD - 1] = {bsk2, bsk3, NULL, NULL, NULL};
  ref_sign_extract_keys(P, bsk, keys, ksk, ct_v, count, sign);
}
void ref_sign_extract(const ref_params* P, const uint64_t* bsk, const uint64_t* ksk, uint64_t* ct_v, int64_t count,
                      uint64_t* sign) {
  ref_sign_extract3(P, bsk, NULL, NULL, ksk, ct_v, count, sign);
}

int ref_sign_precise_rounds(const ref_params* P) {
  int d, j1, j2;
  sign_plan(P, &d, &j1, &j2);
  return j1;
}
int ref_sign_schedule(const ref_params* P, int32_t* out, int32_t cap) {
  int d, sched[64];
  const int R = sign_schedule(P, &d, sched);
  for (int r = 0; r < R && r < cap; ++r) out[r] = sched[r];
  return R;
}
void ref_sign_plan(const ref_params* P, int32_t* d, int32_t* j1, int32_t* j2) {
  int a, b, c;
  sign_plan(P, &a, &b, &c);
  *d = a; *j1 = b; *j2 = c;
}

int ref_sign_digit_bits(const ref_params* P) { return digit_bits(P); }

int ref_sign_pbs_count(const ref_params* P) {
  const int Pb = P->msg_bits, d = digit_bits(P);
  if (Pb < 1) return 0;
  if (Pb < 4) return Pb;
  const int m = Pb - d, r = m % d;
  return 2 * (m / d) + (r >= 3 ? 2 : r) + 1;
}

/* Decrypt the sign ciphertext: 1 iff phase in [2^62, 3*2^62) i.e. bit set. */
void ref_decrypt_bits(const ref_params* P, const uint64_t* s_big, const uint64_t* ct, int64_t count, int64_t* out) {
  const int dim = P->k * P->N;
  for (int64_t c = 0; c < count; ++c) {
    uint64_t ph = lwe_phase(ct + (size_t)c * (dim + 1), s_big, dim);
    out[c] = (int64_t)(((ph + (1ull << 62)) >> 63) & 1);
  }
}
