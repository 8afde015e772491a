// ChaCha20 (RFC 8439) counter-mode streams and TUniform noise — device side.
//
// Every random word of the scheme (secret keys, key masks, key noise,
// encryption masks and noise) is addressed as stream(tag, id)[w]: u64 word w
// is ChaCha20 block floor(w/8) (block counter) of (key, nonce = {tag,
// id_lo, id_hi}), 32-bit output words 2(w%8) and 2(w%8)+1. Addressing by
// (tag, id, w) makes generation embarrassingly parallel and reproducible
// across any launch geometry.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace fhei {

enum StreamTag : uint32_t {
  TAG_SK_SMALL = 1,
  TAG_SK_GLWE = 2,
  TAG_BSK_MASK = 3,
  TAG_BSK_NOISE = 4,
  TAG_KSK_MASK = 5,
  TAG_KSK_NOISE = 6,
  TAG_ENC_MASK = 7,
  TAG_ENC_NOISE = 8,
  TAG_BSK2_MASK = 9,   // the fast-gadget bootstrapping key (fhe_params.pbs_fast_*)
  TAG_BSK2_NOISE = 10,
  TAG_BSK3_MASK = 11,  // the fast2-gadget bootstrapping key (fhe_params.pbs_fast2_*)
  TAG_BSK3_NOISE = 12,
  TAG_MB2_MASK = 13,   // the fast gadget's multi-bit key (pairs of LWE coefficients; fhe_params.pbs_fast_group = 2)
  TAG_MB2_NOISE = 14,
  TAG_MB3_MASK = 15,   // the fast2 gadget's multi-bit key
  TAG_MB3_NOISE = 16,
  TAG_BSK4_MASK = 17,  // the mid gadget's bootstrapping key (fhe_params.pbs_mid_*)
  TAG_BSK4_NOISE = 18,
  TAG_BSK5_MASK = 19,  // the mid2 gadget's bootstrapping key (fhe_params.pbs_mid2_*)
  TAG_BSK5_NOISE = 20,
  TAG_MB4_MASK = 21,   // the mid gadget's multi-bit key (fhe_params.pbs_mid_group = 2)
  TAG_MB4_NOISE = 22,
  TAG_MB5_MASK = 23,   // the mid2 gadget's multi-bit key
  TAG_MB5_NOISE = 24,
  TAG_BSK6_MASK = 25,  // the mid0 gadget's bootstrapping key (fhe_params.pbs_mid0_*)
  TAG_BSK6_NOISE = 26,
  TAG_MB6_MASK = 27,   // the mid0 gadget's multi-bit key
  TAG_MB6_NOISE = 28,
};

struct ChaKey {
  uint32_t w[8];
};

__host__ __device__ __forceinline__ uint32_t rotl32(uint32_t a, int b) { return (a << b) | (a >> (32 - b)); }

#define FHEI_QR(a, b, c, d)                       \
  a += b; d ^= a; d = rotl32(d, 16);              \
  c += d; b ^= c; b = rotl32(b, 12);              \
  a += b; d ^= a; d = rotl32(d, 8);               \
  c += d; b ^= c; b = rotl32(b, 7);

// One ChaCha20 block; out[16] little-endian 32-bit words.
__host__ __device__ __forceinline__ void chacha20_block(const ChaKey& K, uint32_t counter, uint32_t tag,
                                                        uint64_t id, uint32_t out[16]) {
  uint32_t x0 = 0x61707865u, x1 = 0x3320646eu, x2 = 0x79622d32u, x3 = 0x6b206574u;
  uint32_t x4 = K.w[0], x5 = K.w[1], x6 = K.w[2], x7 = K.w[3];
  uint32_t x8 = K.w[4], x9 = K.w[5], x10 = K.w[6], x11 = K.w[7];
  uint32_t x12 = counter, x13 = tag, x14 = (uint32_t)id, x15 = (uint32_t)(id >> 32);
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    FHEI_QR(x0, x4, x8, x12) FHEI_QR(x1, x5, x9, x13) FHEI_QR(x2, x6, x10, x14) FHEI_QR(x3, x7, x11, x15)
    FHEI_QR(x0, x5, x10, x15) FHEI_QR(x1, x6, x11, x12) FHEI_QR(x2, x7, x8, x13) FHEI_QR(x3, x4, x9, x14)
  }
  out[0] = x0 + 0x61707865u; out[1] = x1 + 0x3320646eu; out[2] = x2 + 0x79622d32u; out[3] = x3 + 0x6b206574u;
  out[4] = x4 + K.w[0]; out[5] = x5 + K.w[1]; out[6] = x6 + K.w[2]; out[7] = x7 + K.w[3];
  out[8] = x8 + K.w[4]; out[9] = x9 + K.w[5]; out[10] = x10 + K.w[6]; out[11] = x11 + K.w[7];
  out[12] = x12 + counter; out[13] = x13 + tag; out[14] = x14 + (uint32_t)id; out[15] = x15 + (uint32_t)(id >> 32);
}
#undef FHEI_QR

// One ChaCha20 block computed by the four lanes of a quad (lane q = lane & 3
// holds column q: state words q, 4 + q, 8 + q, 12 + q): the column round is
// each lane's own quarter round, the diagonal round the same after rotating
// rows 1-3 of the state by 1, 2, 3 lanes (DPP quad_perm, and back). 10 x (24
// + 6) instructions per lane instead of 976 on one lane: for the few blocks a
// workgroup needs beside a full pass (k_encrypt_linear's noise words). All
// four lanes of the quad must be active. out[r] = output word q + 4 r.
template <int CTRL>
__device__ __forceinline__ uint32_t quad_mov(uint32_t x) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, CTRL, 0xf, 0xf, false);
}
constexpr int QP_ROT1 = 0x39, QP_ROT2 = 0x4e, QP_ROT3 = 0x93, QP_XOR1 = 0xb1;  // quad_perm [1230] [2301] [3012] [1032]
#define FHEI_QRL(a, b, c, d)                      \
  a += b; d ^= a; d = rotl32(d, 16);              \
  c += d; b ^= c; b = rotl32(b, 12);              \
  a += b; d ^= a; d = rotl32(d, 8);               \
  c += d; b ^= c; b = rotl32(b, 7);
// v_q of four values without an indexable array: a select chain on struct
// words (K.w[0..3]) folded into a per-lane dynamic index made hipcc keep the
// key in scratch (36 bytes per lane, 8.4 MB of writes per 1024-pair
// k_encrypt_linear launch, docs/AB_LOG_r06.md); the select is two masked
// blends, and sel4u first makes WAVE-UNIFORM words (the key, constants)
// plain values by readfirstlane (never for per-lane or per-quad values)
__device__ __forceinline__ uint32_t sel4(int q, uint32_t v0, uint32_t v1, uint32_t v2, uint32_t v3) {
  const uint32_t m1 = 0u - (uint32_t)(q & 1), m2 = 0u - (uint32_t)((q >> 1) & 1);
  const uint32_t lo = v0 ^ ((v0 ^ v1) & m1), hi = v2 ^ ((v2 ^ v3) & m1);
  return lo ^ ((lo ^ hi) & m2);
}
__device__ __forceinline__ uint32_t sel4u(int q, uint32_t v0, uint32_t v1, uint32_t v2, uint32_t v3) {
  return sel4(q, (uint32_t)__builtin_amdgcn_readfirstlane((int)v0), (uint32_t)__builtin_amdgcn_readfirstlane((int)v1),
              (uint32_t)__builtin_amdgcn_readfirstlane((int)v2), (uint32_t)__builtin_amdgcn_readfirstlane((int)v3));
}
struct QuadState {
  uint32_t a, b, c, d, a0, b0, c0, d0;
};
__device__ __forceinline__ QuadState quad_init(const ChaKey& K, uint32_t counter, uint32_t tag, uint64_t id, int q) {
  QuadState s;
  s.a0 = sel4(q, 0x61707865u, 0x3320646eu, 0x79622d32u, 0x6b206574u);
  s.b0 = sel4u(q, K.w[0], K.w[1], K.w[2], K.w[3]);
  s.c0 = sel4u(q, K.w[4], K.w[5], K.w[6], K.w[7]);
  s.d0 = sel4(q, counter, tag, (uint32_t)id, (uint32_t)(id >> 32));  // counter: per quad
  s.a = s.a0; s.b = s.b0; s.c = s.c0; s.d = s.d0;
  return s;
}
// one double round of the quad block: column round, rows rotated, diagonal
// round, rotated back
__device__ __forceinline__ void quad_double_round(QuadState& s) {
  FHEI_QRL(s.a, s.b, s.c, s.d)
  s.b = quad_mov<QP_ROT1>(s.b); s.c = quad_mov<QP_ROT2>(s.c); s.d = quad_mov<QP_ROT3>(s.d);
  FHEI_QRL(s.a, s.b, s.c, s.d)
  s.b = quad_mov<QP_ROT3>(s.b); s.c = quad_mov<QP_ROT2>(s.c); s.d = quad_mov<QP_ROT1>(s.d);
}
__device__ __forceinline__ void quad_out(const QuadState& s, uint32_t out[4]) {
  out[0] = s.a + s.a0; out[1] = s.b + s.b0; out[2] = s.c + s.c0; out[3] = s.d + s.d0;
}
__device__ __forceinline__ void chacha20_block_quad(const ChaKey& K, uint32_t counter, uint32_t tag, uint64_t id,
                                                    int q, uint32_t out[4]) {
  QuadState s = quad_init(K, counter, tag, id, q);
#pragma unroll
  for (int r = 0; r < 10; ++r) quad_double_round(s);
  quad_out(s, out);
}
#undef FHEI_QRL

// A lane's own ChaCha20 block (as chacha20_block) with a quad block
// (chacha20_block_quad) interleaved round by round: the quad's dependent
// chain (one quarter round per lane, DPP between rounds) issues in the
// shadow of the lane block's four independent quarter rounds instead of as a
// latency-bound pass of its own (k_encrypt_linear's noise blocks).
#define FHEI_QR2(a, b, c, d)                      \
  a += b; d ^= a; d = rotl32(d, 16);              \
  c += d; b ^= c; b = rotl32(b, 12);              \
  a += b; d ^= a; d = rotl32(d, 8);               \
  c += d; b ^= c; b = rotl32(b, 7);
__device__ __forceinline__ void chacha20_block_with_quad(const ChaKey& K, uint32_t counter, uint32_t tag, uint64_t id,
                                                         uint32_t out[16], uint32_t qcounter, uint32_t qtag,
                                                         uint64_t qid, int q, uint32_t qout[4]) {
  uint32_t x0 = 0x61707865u, x1 = 0x3320646eu, x2 = 0x79622d32u, x3 = 0x6b206574u;
  uint32_t x4 = K.w[0], x5 = K.w[1], x6 = K.w[2], x7 = K.w[3];
  uint32_t x8 = K.w[4], x9 = K.w[5], x10 = K.w[6], x11 = K.w[7];
  uint32_t x12 = counter, x13 = tag, x14 = (uint32_t)id, x15 = (uint32_t)(id >> 32);
  QuadState s = quad_init(K, qcounter, qtag, qid, q);
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    FHEI_QR2(x0, x4, x8, x12) FHEI_QR2(x1, x5, x9, x13) FHEI_QR2(x2, x6, x10, x14) FHEI_QR2(x3, x7, x11, x15)
    FHEI_QR2(x0, x5, x10, x15) FHEI_QR2(x1, x6, x11, x12) FHEI_QR2(x2, x7, x8, x13) FHEI_QR2(x3, x4, x9, x14)
    quad_double_round(s);
  }
  out[0] = x0 + 0x61707865u; out[1] = x1 + 0x3320646eu; out[2] = x2 + 0x79622d32u; out[3] = x3 + 0x6b206574u;
  out[4] = x4 + K.w[0]; out[5] = x5 + K.w[1]; out[6] = x6 + K.w[2]; out[7] = x7 + K.w[3];
  out[8] = x8 + K.w[4]; out[9] = x9 + K.w[5]; out[10] = x10 + K.w[6]; out[11] = x11 + K.w[7];
  out[12] = x12 + counter; out[13] = x13 + tag; out[14] = x14 + (uint32_t)id; out[15] = x15 + (uint32_t)(id >> 32);
  quad_out(s, qout);
}
#undef FHEI_QR2

// Eight consecutive u64 words [8*blk, 8*blk+8) of stream (tag, id).
__host__ __device__ __forceinline__ void stream_block(const ChaKey& K, uint32_t tag, uint64_t id, uint32_t blk,
                                                      uint64_t w[8]) {
  uint32_t o[16];
  chacha20_block(K, blk, tag, id, o);
#pragma unroll
  for (int j = 0; j < 8; ++j) w[j] = (uint64_t)o[2 * j] | ((uint64_t)o[2 * j + 1] << 32);
}

__host__ __device__ __forceinline__ uint64_t stream_word(const ChaKey& K, uint32_t tag, uint64_t id, uint64_t w) {
  uint32_t o[16];
  chacha20_block(K, (uint32_t)(w >> 3), tag, id, o);
  const int j = (int)(w & 7);
  return (uint64_t)o[2 * j] | ((uint64_t)o[2 * j + 1] << 32);
}

// TUniform(b): uniform on [-2^b, 2^b] with the two endpoints at half weight.
__host__ __device__ __forceinline__ int64_t tuniform(uint64_t w, int b) {
  const uint64_t bits = w & ((2ull << (b + 1)) - 1);  // b + 2 bits
  return (int64_t)((bits >> 1) + (bits & 1)) - ((int64_t)1 << b);
}

__host__ __device__ __forceinline__ uint64_t splitmix64(uint64_t& x) {
  uint64_t z = (x += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// 64-bit seed -> 256-bit ChaCha key (for reproducible tests and benches; a
// deployment passes 32 bytes from the OS CSPRNG via fhe_*_key entry points).
__host__ __device__ __forceinline__ ChaKey key_from_seed(uint64_t seed) {
  ChaKey K;
  uint64_t x = seed;
  for (int i = 0; i < 4; ++i) {
    const uint64_t v = splitmix64(x);
    K.w[2 * i] = (uint32_t)v;
    K.w[2 * i + 1] = (uint32_t)(v >> 32);
  }
  return K;
}

}  // namespace fhei
