// libfheicp: MI355X-native TFHE engine for the encrypted pairwise compare of
// shipstone-labs/fhe-icp. C ABI in include/fhe_icp.h; design in DESIGN.md.
//
// Kernels (one file so the whole engine is one code object):
//   keygen:   k_keygen_secrets, k_keygen_bsk, k_keygen_ksk, k_bsk_to_fft
//   client:   k_encrypt, k_decrypt
//   server:   k_linear          (Concrete-ML _inference, leveled)
//             k_keyswitch       (big -> small key, tiled GEMM-like)
//             k_blind_rotate    (external products, f64 wave FFT)  <- hot
//   search:   k_topk
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/fhe_icp.h"
#include "prng.h"
#include "wave_fft.h"
#include "br_m512.h"
#include "br_m512q.h"
#include "br_v4.h"

using namespace fhei;
typedef uint64_t u64;

// ============================================================ helpers ======
__device__ __forceinline__ uint32_t modswitch_2n(u64 a, int log2n2) {
  return (uint32_t)((((a >> (63 - log2n2)) + 1) >> 1) & ((1ull << log2n2) - 1));
}

// Closest multiple of 2^(64 - L*beta) of x, re-encoded as L balanced digits
// packed offset-binary: digit of level lvl (1 = most significant) is
// ((packed >> ((L - lvl) * beta)) & (B-1)) - B/2.  
__device__ __forceinline__ u64 decompose_packed(u64 x, int beta, int L) {
  const int prec = L * beta;
  u64 r = ((x >> (63 - prec)) + 1) >> 1;
  if (prec < 64) r &= ((1ull << prec) - 1);
  int64_t v = (int64_t)r;
  const int64_t B = (int64_t)1 << beta;
  u64 packed = 0;
  for (int l = L; l >= 1; --l) {
    int64_t d = v & (B - 1);
    v >>= beta;
    if (d >= B / 2) {
      d -= B;
      v += 1;
    }
    packed |= (u64)(d + B / 2) << ((L - l) * beta);
  }
  return packed;
}
__device__ __forceinline__ int digit_of(u64 packed, int lvl, int beta, int L) {
  const int64_t B = (int64_t)1 << beta;
  return (int)((int64_t)((packed >> ((L - lvl) * beta)) & (u64)(B - 1)) - B / 2);
}

template <int NT>
__device__ __forceinline__ u64 block_sum_u64(u64 v, u64* red) {
  // wave reduce
  for (int off = 32; off > 0; off >>= 1) v += __shfl_down(v, off, 64);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) red[w] = v;
  __syncthreads();
  u64 s = 0;
  if (threadIdx.x == 0)
    for (int i = 0; i < NT / 64; ++i) s += red[i];
  __syncthreads();
  return s;  // valid in thread 0
}

// ============================================================ keygen =======
__global__ void k_keygen_secrets(ChaKey K, int n, int big, u64* s_small, u64* s_big) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) s_small[i] = stream_word(K, TAG_SK_SMALL, 0, (u64)i) & 1;
  if (i < big) s_big[i] = stream_word(K, TAG_SK_GLWE, 0, (u64)i) & 1;
}

// One workgroup per GGSW row (i, r): GLWE_S(0) + s_small[i] * g_lvl on
// component c_in. body = sum_j A_j * S_j (negacyclic, binary S) + E.
__global__ void __launch_bounds__(256) k_keygen_bsk(ChaKey K, int N, int k, int L, int beta, int noise_bits,
                                                    const u64* __restrict__ s_small, const u64* __restrict__ s_big,
                                                    u64* __restrict__ bsk) {
  extern __shared__ u64 shm[];
  u64* A = shm;                                          // N
  unsigned char* S = (unsigned char*)(shm + N);          // N
  const int R = (k + 1) * L;
  const int row = blockIdx.x;  // i * R + r
  const int i = row / R, r = row % R;
  const int c_in = r / L, lvl = r % L + 1;
  u64* dst = bsk + (size_t)row * (k + 1) * N;
  constexpr int MAXC = 8;  // N <= 2048 -> 8 coefficients per thread
  u64 body[MAXC];
  const int per = N / 256;
  for (int q = 0; q < per; ++q) body[q] = 0;
  for (int j = 0; j < k; ++j) {
    const u64 sid = (u64)row * k + j;
    for (int blk = threadIdx.x; blk < N / 8; blk += 256) {
      u64 w[8];
      stream_block(K, TAG_BSK_MASK, sid, (uint32_t)blk, w);
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        A[8 * blk + q] = w[q];
        dst[(size_t)j * N + 8 * blk + q] = w[q];
      }
    }
    for (int t = threadIdx.x; t < N; t += 256) S[t] = (unsigned char)s_big[(size_t)j * N + t];
    __syncthreads();
    for (int v = 0; v < N; ++v) {
      if (!S[v]) continue;  // uniform across the block
      for (int q = 0; q < per; ++q) {
        const int t = threadIdx.x + 256 * q;
        body[q] += (t >= v) ? A[t - v] : (u64)0 - A[t - v + N];
      }
    }
    __syncthreads();
  }
  for (int q = 0; q < per; ++q) {
    const int t = threadIdx.x + 256 * q;
    u64 b = body[q] + (u64)tuniform(stream_word(K, TAG_BSK_NOISE, (u64)row, (u64)t), noise_bits);
    dst[(size_t)k * N + t] = b;
  }
  __syncthreads();
  if (threadIdx.x == 0 && s_small[i]) dst[(size_t)c_in * N] += 1ull << (64 - lvl * beta);
}

// One workgroup per KSK row (i, l): LWE_{s_small}(s_big[i] * 2^(64 - (l+1) beta)).
__global__ void __launch_bounds__(256) k_keygen_ksk(ChaKey K, int n, int KL, int kbeta, int noise_bits,
                                                    const u64* __restrict__ s_small, const u64* __restrict__ s_big,
                                                    u64* __restrict__ ksk) {
  __shared__ u64 red[4];
  const int row = blockIdx.x;  // i * KL + l
  const int i = row / KL, l = row % KL;
  u64* dst = ksk + (size_t)row * (n + 1);
  u64 part = 0;
  for (int blk = threadIdx.x; blk < (n + 7) / 8; blk += 256) {
    u64 w[8];
    stream_block(K, TAG_KSK_MASK, (u64)row, (uint32_t)blk, w);
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int t = 8 * blk + q;
      if (t < n) {
        dst[t] = w[q];
        if (s_small[t]) part += w[q];
      }
    }
  }
  const u64 s = block_sum_u64<256>(part, red);
  if (threadIdx.x == 0) {
    u64 b = s + (u64)tuniform(stream_word(K, TAG_KSK_NOISE, (u64)row, 0), noise_bits);
    if (s_big[i]) b += 1ull << (64 - (l + 1) * kbeta);
    dst[n] = b;
  }
}

// One wave per polynomial: fold/twist, forward FFT, scale 1/M, store in the
// [u][lane] order the blind rotation reads (coalesced 1 KiB per slot).
template <int LOGM>
__global__ void __launch_bounds__(64) k_bsk_to_fft(const u64* __restrict__ bsk, int npoly,
                                                   const c64* __restrict__ tw, const c64* __restrict__ twist,
                                                   c64* __restrict__ out) {
  using F = WaveFFT<LOGM>;
  constexpr int M = F::M, S = F::S;
  __shared__ c64 lds[F::LDS_ELEMS];
  const int poly = blockIdx.x, l = threadIdx.x;
  if (poly >= npoly) return;
  const u64* src = bsk + (size_t)poly * 2 * M;
  c64 v[S];
#pragma unroll
  for (int u = 0; u < S; ++u) {
    const int t = l + 64 * u;
    const c64 a = {(double)(int64_t)src[t], (double)(int64_t)src[t + M]};
    v[u] = cmul(a, twist[t]);
  }
  F::forward(v, tw, lds, l);
  const double inv = 1.0 / (double)M;
  c64* dst = out + (size_t)poly * M;
#pragma unroll
  for (int u = 0; u < S; ++u) dst[u * 64 + l] = {v[u].x * inv, v[u].y * inv};
}

// ============================================================ client =======
// One workgroup (256 threads) per ciphertext of dimension `dim` (multiple of 8).
__global__ void __launch_bounds__(256) k_encrypt(ChaKey K, int dim, int msg_bits, int noise_bits,
                                                 const u64* __restrict__ s_big, const int64_t* __restrict__ msg,
                                                 u64 id0, u64* __restrict__ ct) {
  __shared__ u64 red[4];
  const int64_t c = blockIdx.x;
  const u64 id = id0 + (u64)c;
  u64* o = ct + (size_t)c * (dim + 1);
  u64 part = 0;
  for (int blk = threadIdx.x; blk < dim / 8; blk += 256) {
    u64 w[8];
    stream_block(K, TAG_ENC_MASK, id, (uint32_t)blk, w);
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      o[8 * blk + q] = w[q];
      part += w[q] & (0 - s_big[8 * blk + q]);
    }
  }
  const u64 s = block_sum_u64<256>(part, red);
  if (threadIdx.x == 0) {
    const u64 e = (u64)tuniform(stream_word(K, TAG_ENC_NOISE, id, 0), noise_bits);
    o[dim] = s + e + ((u64)msg[c] << (64 - msg_bits));
  }
}

// ---- seeded (compressed) ciphertexts: the stored document corpus ----------
// A seeded LWE keeps only its body; the mask is stream(TAG_ENC_MASK, id) of
// a PUBLIC mask key Km, the noise stream(TAG_ENC_NOISE, id) of a SECRET
// noise key Kn. Document b of a corpus holds D bodies,
// feature j under stream id id0[b] + j. 2049 -> 1 word per feature in HBM:
// the masks are regenerated where they are consumed (k_linear_seeded).
__global__ void __launch_bounds__(256) k_encrypt_seeded(ChaKey Km, ChaKey Kn, int dim, int msg_bits, int noise_bits,
                                                        const u64* __restrict__ s_big,
                                                        const int64_t* __restrict__ msg,
                                                        const u64* __restrict__ id0, int D, u64* __restrict__ body) {
  __shared__ u64 red[4];
  const int64_t c = blockIdx.x;
  const int64_t b = c / D;
  const u64 id = id0[b] + (u64)(c - b * D);
  u64 part = 0;
  for (int blk = threadIdx.x; blk < dim / 8; blk += 256) {
    u64 w[8];
    stream_block(Km, TAG_ENC_MASK, id, (uint32_t)blk, w);
#pragma unroll
    for (int q = 0; q < 8; ++q) part += w[q] & (0 - s_big[8 * blk + q]);
  }
  const u64 s = block_sum_u64<256>(part, red);
  if (threadIdx.x == 0) {
    const u64 e = (u64)tuniform(stream_word(Kn, TAG_ENC_NOISE, id, 0), noise_bits);
    body[c] = s + e + ((u64)msg[c] << (64 - msg_bits));
  }
}

// full ciphertexts [B*D][dim+1] from the seeded corpus (interop / tests)
__global__ void __launch_bounds__(256) k_expand_seeded(ChaKey Km, int dim, const u64* __restrict__ body,
                                                       const u64* __restrict__ id0, int D, u64* __restrict__ ct) {
  const int64_t c = blockIdx.x;
  const int64_t b = c / D;
  const u64 id = id0[b] + (u64)(c - b * D);
  u64* o = ct + (size_t)c * (dim + 1);
  for (int blk = threadIdx.x; blk < dim / 8; blk += 256) {
    u64 w[8];
    stream_block(Km, TAG_ENC_MASK, id, (uint32_t)blk, w);
#pragma unroll
    for (int q = 0; q < 8; ++q) o[8 * blk + q] = w[q];
  }
  if (threadIdx.x == 0) o[dim] = body[c];
}

// out[b] = sum_j w[j] * ct(b, j) + cst * Delta on the seeded corpus: one
// workgroup per document, each thread owns one 8-word ChaCha block of the
// mask (dim / 8 threads), regenerated per feature in registers. Reads D + 1
// words per document from HBM instead of D (dim + 1).
__global__ void __launch_bounds__(256) k_linear_seeded(ChaKey Km, int dim, const u64* __restrict__ body,
                                                       const u64* __restrict__ id0, int D,
                                                       const int64_t* __restrict__ w, u64 cst_scaled,
                                                       u64* __restrict__ out) {
  const int64_t b = blockIdx.x;
  const u64 base = id0[b];
  u64* o = out + (size_t)b * (dim + 1);
  for (int blk = threadIdx.x; blk < dim / 8; blk += 256) {
    u64 acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int j = 0; j < D; ++j) {
      u64 m[8];
      stream_block(Km, TAG_ENC_MASK, base + (u64)j, (uint32_t)blk, m);
      const u64 wj = (u64)w[j];
#pragma unroll
      for (int q = 0; q < 8; ++q) acc[q] += wj * m[q];
    }
#pragma unroll
    for (int q = 0; q < 8; ++q) o[8 * blk + q] = acc[q];
  }
  if (threadIdx.x == 0) {
    u64 acc = cst_scaled;
    for (int j = 0; j < D; ++j) acc += (u64)w[j] * body[(size_t)b * D + j];
    o[dim] = acc;
  }
}

// mode 0: decode signed msg_bits integer; 1: bit (nearer 2^63); 2: raw phase
__global__ void __launch_bounds__(256) k_decrypt(int dim, int msg_bits, int mode, const u64* __restrict__ s,
                                                 const u64* __restrict__ ct, int64_t* __restrict__ out) {
  __shared__ u64 red[4];
  const int64_t c = blockIdx.x;
  const u64* x = ct + (size_t)c * (dim + 1);
  u64 part = 0;
  for (int t = threadIdx.x; t < dim; t += 256) part += x[t] & (0 - s[t]);
  const u64 sum = block_sum_u64<256>(part, red);
  if (threadIdx.x == 0) {
    const u64 ph = x[dim] - sum;
    int64_t r;
    if (mode == 0) {
      u64 q = ((ph >> (63 - msg_bits)) + 1) >> 1;
      if (msg_bits < 64) q &= (1ull << msg_bits) - 1;
      r = (q >> (msg_bits - 1)) ? (int64_t)q - ((int64_t)1 << msg_bits) : (int64_t)q;
    } else if (mode == 1) {
      r = (int64_t)(((ph + (1ull << 62)) >> 63) & 1);
    } else {
      r = (int64_t)ph;
    }
    out[c] = r;
  }
}

// ============================================================ server =======
// out[b][t] = sum_j w[j] ct[b][j][t] (+ cst * Delta on the body)
__global__ void __launch_bounds__(256) k_linear(const u64* __restrict__ ct, int D, int W,
                                                const int64_t* __restrict__ w, u64 cst_scaled,
                                                u64* __restrict__ out) {
  const int64_t b = blockIdx.y;
  const int t = blockIdx.x * 256 + threadIdx.x;
  if (t >= W) return;
  const u64* x = ct + (size_t)b * D * W + t;
  u64 acc = 0;
  for (int j = 0; j < D; ++j) acc += (u64)w[j] * x[(size_t)j * W];
  if (t == W - 1) acc += cst_scaled;
  out[(size_t)b * W + t] = acc;
}

// Key switch (big -> small key), as a split-K integer GEMM:
//   out[c][t] = body_c + (B/2) colsum[t] - sum_{i,l} d'[c][i][l] * KSK[i][l][t]
// with offset-binary digits d' = d + B/2 in [0, B) (so each term is two
// v_mad_u64_u32 on the 32-bit halves of the KSK word) and
// colsum[t] = sum over all rows of KSK[.][t] (precomputed at keygen).
// Workgroup = KS_TC ciphertexts x 256 output columns x one slice of the
// input rows; slices are combined with u64 atomics, which are exact and
// order-independent modulo 2^64 (bit-identical results every run).
constexpr int KS_TC = 16, KS_IC = 32, KS_SPLIT = 8;
__global__ void __launch_bounds__(256) k_keyswitch(const u64* __restrict__ in, int64_t count, int big, int n,
                                                   int KL, int kbeta, int shift, u64 add_body,
                                                   const u64* __restrict__ ksk, const u64* __restrict__ colsum,
                                                   u64* __restrict__ out) {
  __shared__ uint8_t dig[KS_IC][8][KS_TC];  // [input][level][ciphertext]
  const int col = blockIdx.x * 256 + threadIdx.x;
  const int64_t c0 = (int64_t)blockIdx.y * KS_TC;
  const int nct = (int)min((int64_t)KS_TC, count - c0);
  const int per = (big + KS_SPLIT - 1) / KS_SPLIT;
  const int ibeg = blockIdx.z * per, iend_all = min(big, ibeg + per);
  const u64 half = 1ull << (kbeta - 1);
  u64 lo[KS_TC], hi[KS_TC];
#pragma unroll
  for (int q = 0; q < KS_TC; ++q) lo[q] = hi[q] = 0;
  for (int i0 = ibeg; i0 < iend_all; i0 += KS_IC) {
    for (int e = threadIdx.x; e < KS_TC * KS_IC; e += 256) {
      const int q = e / KS_IC, ii = e % KS_IC;
      if (q < nct && i0 + ii < iend_all) {
        const u64 a = in[(size_t)(c0 + q) * (big + 1) + i0 + ii] << shift;
        const u64 packed = decompose_packed(a, kbeta, KL);  // offset-binary already
        for (int l = 1; l <= KL; ++l) dig[ii][l - 1][q] = (uint8_t)((packed >> ((KL - l) * kbeta)) & ((1u << kbeta) - 1));
      } else {
        for (int l = 0; l < KL; ++l) dig[ii][l][q] = (uint8_t)half;  // digit 0
      }
    }
    __syncthreads();
    if (col <= n) {
      const int cnt = min(KS_IC, iend_all - i0);
      for (int ii = 0; ii < cnt; ++ii) {
        for (int l = 0; l < KL; ++l) {
          const u64 kv = ksk[((size_t)(i0 + ii) * KL + l) * (n + 1) + col];
          const uint32_t kl = (uint32_t)kv, kh = (uint32_t)(kv >> 32);
          const uint32_t* d4 = (const uint32_t*)&dig[ii][l][0];
#pragma unroll
          for (int w = 0; w < KS_TC / 4; ++w) {
            const uint32_t pk = d4[w];
#pragma unroll
            for (int b = 0; b < 4; ++b) {
              const uint32_t d = (pk >> (8 * b)) & 0xFF;
              lo[4 * w + b] += (u64)d * kl;
              hi[4 * w + b] += (u64)d * kh;
            }
          }
        }
      }
    }
    __syncthreads();
  }
  if (col <= n) {
#pragma unroll
    for (int q = 0; q < KS_TC; ++q) {
      if (q < nct) {
        u64 v = (u64)0 - (lo[q] + (hi[q] << 32));
        if (blockIdx.z == 0) {
          v += half * colsum[col];
          if (col == n) v += (in[(size_t)(c0 + q) * (big + 1) + big] << shift) + add_body;
        }
        atomicAdd((unsigned long long*)&out[(size_t)(c0 + q) * (n + 1) + col], (unsigned long long)v);
      }
    }
  }
}

// colsum[t] = sum over all KSK rows of KSK[row][t] (mod 2^64)
__global__ void k_ksk_colsum(const u64* __restrict__ ksk, int rows, int n, u64* __restrict__ colsum) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t > n) return;
  u64 s = 0;
  for (int r = 0; r < rows; ++r) s += ksk[(size_t)r * (n + 1) + t];
  colsum[t] = s;
}

// Test vector of a bootstrap: TV_j = base + (j >> shift) * step for
// j in [0, N) (a staircase; step = 0 gives the constant TV of a sign
// bootstrap), extended negacyclically: coefficient t of X^{-b} TV is
// TV_{(t+b) mod 2N} with a minus sign when (t + b) mod 2N >= N.
struct BrTv {
  u64 base, step;
  int shift;
};
__device__ __forceinline__ u64 tv_rot(const BrTv& tv, uint32_t idx, int N) {
  const uint32_t j = idx & (uint32_t)(N - 1);
  const u64 v = tv.base + (u64)(j >> tv.shift) * tv.step;
  return idx < (uint32_t)N ? v : (u64)0 - v;
}
// Output of one extracted LWE word x (word `pos` of ciphertext c):
//   mode 0: out = x
//   mode 1: sign-bit round: bit = trivial(tv.base) - x; ct_v -= bit;
//           refreshed += bit (if given); sign = bit (if given)
//   mode 2: digit round: ct_v -= x; refreshed += x (if given)
__device__ __forceinline__ void br_emit(int mode, u64 x, bool body, const BrTv& tv, size_t pos, u64* out, u64* ct_v,
                                        u64* refreshed, u64* sign) {
  if (mode == 0) {
    out[pos] = x;
    return;
  }
  const u64 d = mode == 1 ? (body ? tv.base : (u64)0) - x : x;
  ct_v[pos] -= d;
  if (refreshed) refreshed[pos] += d;
  if (sign) sign[pos] = d;
}


// ---- key switch on the i8 matrix cores (v_mfma_i32_16x16x64_i8) ----------
// out[c] = (0, .., 0, b'[c]) - sum_r D[c][r] * KSK[r], r = i * ks_level + l,
// a GEMM [count x K] (digits in [-2^(b-1), 2^(b-1))) x [K x (n+1)] over
// Z_2^64. The key is split into 8 balanced radix-256 byte planes,
// KSK = sum_q s_q 2^(8q) with s_q in [-128, 127], each an i8 GEMM with i32
// accumulation (|sum| <= K * 2^(b-1) * 128 < 2^31); the epilogue recombines
// sum_q acc_q << 8q modulo 2^64 (exact: DESIGN.md §4.3).
// Fragment layouts (checked by tools/mfma_i8_probe.hip): lane l holds
// A[row l&15][k = 16 (l>>4) + j] and B[k = 16 (l>>4) + j][col l&15] in byte j;
// C/D: row 4 (l>>4) + reg, col l&15.
typedef int v4i __attribute__((ext_vector_type(4)));
constexpr int KSM_NB_COLS = 16;  // columns per block

// key planes: [kb][nb][q][lane][16 B]
__global__ void k_ksk_to_i8(const u64* __restrict__ ksk, int K, int n1, int NB, int8_t* __restrict__ out) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (int64_t)K * NB * 16) return;
  const int row = (int)(e / (NB * 16)), col = (int)(e % (NB * 16));
  u64 x = col < n1 ? ksk[(size_t)row * n1 + col] : 0;
  const int kb = row >> 6, g = (row >> 4) & 3, j = row & 15;
  const int nb = col >> 4, lane = (col & 15) + 16 * g;
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const int8_t sq = (int8_t)(x & 0xff);
    x = (x - (u64)(int64_t)sq) >> 8;
    out[((((size_t)kb * NB + nb) * 8 + q) * 64 + lane) * 16 + j] = sq;
  }
}

// digits in A-fragment order [cb][kb][lane][16 B] (ks_level = 4: a
// coefficient's 4 digits are 4 consecutive bytes) and b' = (b << shift) + add
__global__ void __launch_bounds__(256) k_ks_digits(const u64* __restrict__ in, int64_t count, int big, int beta,
                                                   int shift, u64 add_body, int KB, uint32_t* __restrict__ D,
                                                   u64* __restrict__ body) {
  const int t = threadIdx.x, cl = t >> 4, il = t & 15;
  const int64_t cb = blockIdx.y, c = cb * 16 + cl;
  const int kb = blockIdx.x, i = kb * 16 + il;
  if (c >= count) return;
  const u64* src = in + (size_t)c * (big + 1);
  if (kb == 0 && il == 0) body[c] = (src[big] << shift) + add_body;
  const int prec = 4 * beta;
  uint32_t r = (uint32_t)((((src[i] << shift) >> (63 - prec)) + 1) >> 1);
  uint32_t packed = 0;
#pragma unroll
  for (int s = 0; s < 4; ++s) {  // LSB-first; level l = 3 - s sits in byte l
    const int d = __builtin_amdgcn_sbfe((int)r, s * beta, beta);
    r -= (uint32_t)d << (s * beta);
    packed |= (uint32_t)(uint8_t)(int8_t)d << (8 * (3 - s));
  }
  const int lane = cl + 16 * (il >> 2);
  D[(((size_t)cb * KB + kb) * 64 + lane) * 4 + (il & 3)] = packed;
}

// workgroup = 4 waves = 64 ciphertexts x 16 columns x 8 byte planes; the key
// tile of each k-block (8 KB) is shared through double-buffered LDS
__global__ void __launch_bounds__(256) k_keyswitch_mfma(const v4i* __restrict__ D, const v4i* __restrict__ K8,
                                                        const u64* __restrict__ body, int64_t count, int n1, int NB,
                                                        int KB, u64* __restrict__ out) {
  __shared__ v4i bt[2][8 * 64];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int nb = blockIdx.y;
  const int64_t cb = (int64_t)blockIdx.x * 4 + w;
  const bool act = cb * 16 < count;
  const v4i zero = {0, 0, 0, 0};
  const v4i* Dv = D + (size_t)cb * KB * 64 + lane;
  const v4i* Kv = K8 + (size_t)nb * 8 * 64;
  v4i acc[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) acc[q] = zero;
  bt[0][tid] = Kv[tid];
  bt[0][tid + 256] = Kv[tid + 256];
  v4i a = act ? Dv[0] : zero;
  __syncthreads();
  for (int kb = 0; kb < KB; ++kb) {
    const int cur = kb & 1;
    v4i n0 = zero, n1v = zero, an = zero;
    const bool more = kb + 1 < KB;
    if (more) {
      const v4i* srcp = Kv + (size_t)(kb + 1) * NB * 8 * 64;
      n0 = srcp[tid];
      n1v = srcp[tid + 256];
      if (act) an = Dv[(size_t)(kb + 1) * 64];
    }
#pragma unroll
    for (int q = 0; q < 8; ++q) acc[q] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, bt[cur][q * 64 + lane], acc[q], 0, 0, 0);
    if (more) {
      bt[cur ^ 1][tid] = n0;
      bt[cur ^ 1][tid + 256] = n1v;
      a = an;
    }
    __syncthreads();
  }
  if (!act) return;
  const int col = nb * KSM_NB_COLS + (lane & 15);
  if (col >= n1) return;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int64_t c = cb * 16 + 4 * (lane >> 4) + r;
    if (c >= count) continue;
    u64 v = 0;
#pragma unroll
    for (int q = 0; q < 8; ++q) v += (u64)(int64_t)acc[q][r] << (8 * q);
    out[(size_t)c * n1 + col] = (col == n1 - 1 ? body[c] : (u64)0) - v;
  }
}

// Blind rotation + sample extraction. One 64-lane wavefront (= workgroup)
// per ciphertext; the GLWE accumulator ((K+1) x N u64) lives in LDS, the
// external-product partial sums in registers.
// Test vector and epilogue modes: BrTv / br_emit above.
template <int LOGM, int K>
__global__ void __launch_bounds__(64) k_blind_rotate(const u64* __restrict__ small, int n, int L, int beta,
                                                     const c64* __restrict__ bsk, const c64* __restrict__ tw,
                                                     const c64* __restrict__ twist, BrTv tv, int mode,
                                                     u64* __restrict__ out, u64* __restrict__ ct_v,
                                                     u64* __restrict__ refreshed, u64* __restrict__ sign) {
  using F = WaveFFT<LOGM>;
  constexpr int M = F::M, S = F::S, N = 2 * M;
  constexpr int LOG2N2 = LOGM + 2;
  __shared__ u64 acc[(K + 1) * N];
  __shared__ c64 lds[F::LDS_ELEMS];
  const int l = threadIdx.x;
  const int64_t c = blockIdx.x;
  const u64* sm = small + (size_t)c * (n + 1);
  const int R = (K + 1) * L;

  // ACC = X^{-b~} * (0, .., 0, TV)
  const uint32_t bt = modswitch_2n(sm[n], LOG2N2);
  for (int t = l; t < N; t += 64) {
#pragma unroll
    for (int j = 0; j < K; ++j) acc[j * N + t] = 0;
    const uint32_t idx = (uint32_t)(t + bt) & (2 * N - 1);
    acc[K * N + t] = tv_rot(tv, idx, N);
  }
  __syncthreads();

  for (int i = 0; i < n; ++i) {
    const uint32_t ai = modswitch_2n(sm[i], LOG2N2);
    if (ai == 0) continue;
    c64 outv[K + 1][S];
#pragma unroll
    for (int o = 0; o <= K; ++o)
#pragma unroll
      for (int u = 0; u < S; ++u) outv[o][u] = {0.0, 0.0};
    const c64* G = bsk + (size_t)i * R * (K + 1) * M;
#pragma unroll
    for (int cc = 0; cc <= K; ++cc) {
      const u64* f = acc + cc * N;
      u64 p0[S], p1[S];
#pragma unroll
      for (int u = 0; u < S; ++u) {
        const int t0 = l + 64 * u, t1 = t0 + M;
        uint32_t i0 = (uint32_t)(t0 - (int)ai) & (2 * N - 1);
        uint32_t i1 = (uint32_t)(t1 - (int)ai) & (2 * N - 1);
        const u64 r0 = i0 < (uint32_t)N ? f[i0] : (u64)0 - f[i0 - N];
        const u64 r1 = i1 < (uint32_t)N ? f[i1] : (u64)0 - f[i1 - N];
        p0[u] = decompose_packed(r0 - f[t0], beta, L);
        p1[u] = decompose_packed(r1 - f[t1], beta, L);
      }
      for (int lvl = 1; lvl <= L; ++lvl) {
        c64 v[S];
#pragma unroll
        for (int u = 0; u < S; ++u) {
          const c64 d = {(double)digit_of(p0[u], lvl, beta, L), (double)digit_of(p1[u], lvl, beta, L)};
          v[u] = cmul(d, twist[l + 64 * u]);
        }
        F::forward(v, tw, lds, l);
        const c64* g = G + (size_t)((cc * L + lvl - 1) * (K + 1)) * M;
#pragma unroll
        for (int o = 0; o <= K; ++o)
#pragma unroll
          for (int u = 0; u < S; ++u) cmac(outv[o][u], v[u], g[o * M + u * 64 + l]);
      }
    }
#pragma unroll
    for (int o = 0; o <= K; ++o) {
      F::inverse(outv[o], tw, lds, l);
#pragma unroll
      for (int u = 0; u < S; ++u) {
        const int t0 = l + 64 * u;
        const c64 z = cmulc(outv[o][u], twist[t0]);
        acc[o * N + t0] += f64_to_torus(z.x);
        acc[o * N + t0 + M] += f64_to_torus(z.y);
      }
    }
    __syncthreads();
  }

  // sample extract coefficient 0 -> LWE under s_big (dim K*N)
  const int W = K * N + 1;
  for (int j = 0; j < K; ++j) {
    for (int t = l; t < N; t += 64) {
      const u64 a = (t == 0) ? acc[j * N] : (u64)0 - acc[j * N + N - t];
      br_emit(mode, a, false, tv, (size_t)c * W + j * N + t, out, ct_v, refreshed, sign);
    }
  }
  if (l == 0) br_emit(mode, acc[K * N], true, tv, (size_t)c * W + K * N, out, ct_v, refreshed, sign);
}

// Client-side input path of batch_operations.py:226/:273 + Concrete-ML's
// input quantizer, fused: X = query (.) doc in the operands' dtype (numpy
// promotion), then q = clip(rint(X / s + zp), qmin, qmax) in float64.
// IEEE division and rint make this bit-identical to numpy.
template <typename QT, typename DT>
__global__ void k_pair_quantize(const QT* __restrict__ query, const DT* __restrict__ docs, int64_t B, int D,
                                double scale, double zp, double qmin, double qmax, int64_t* __restrict__ qx) {
  using RT = decltype(QT() * DT());  // numpy promotion of the element-wise product
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= B * D) return;
  const RT x = query ? (RT)query[e % D] * (RT)docs[e] : (RT)docs[e];
  double q = rint((double)x / scale + zp);
  q = fmin(fmax(q, qmin), qmax);
  qx[e] = (int64_t)q;
}

// score[b] = out_scale * double(acc[b])  (UniformQuantizer.dequant, zp 0)
__global__ void k_dequantize(const int64_t* __restrict__ acc, int64_t B, double out_scale, double* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < B) out[i] = out_scale * (double)acc[i];
}

// ---- blind rotation for N = 1024, several waves per ciphertext -------------
// V = V2 (br_m512.h: 2 waves, 4 complex/lane) or V3 (br_m512q.h: 4 waves,
// 2 complex/lane); both share this kernel body.
// BSK conversion for v2: one 128-thread workgroup per polynomial, same FFT
// as the blind rotation, stored at [u][tid] (LCs layout) and scaled by 1/M.
template <class V>
__global__ void __launch_bounds__(V::NT) k_bsk_to_fft_mw(const u64* __restrict__ bsk, int npoly,
                                                         const c64* __restrict__ tw, const c64* __restrict__ twist,
                                                         c64* __restrict__ out) {
  constexpr int M = V::M, N = V::N, S = V::S;
  using Tw = typename V::Tw;
  __shared__ c64 lds[V::SCRATCH];
  const int poly = blockIdx.x, tid = threadIdx.x;
  if (poly >= npoly) return;
  Tw T;
  V::load_twiddles(T, tw, tid);
  const u64* src = bsk + (size_t)poly * N;
  c64 v[1][S];
#pragma unroll
  for (int u = 0; u < S; ++u) {
    const int t = V::tcoef(tid, u);
    v[0][u] = cmul({(double)(int64_t)src[t], (double)(int64_t)src[t + M]}, twist[t]);
  }
  if constexpr (V::MULTI) V::template forward<1>(v, T, lds, tid);
  else V::forward(v[0], T, lds, tid);
  const double inv = 1.0 / (double)M;
  c64* dst = out + (size_t)poly * M;
#pragma unroll
  for (int u = 0; u < S; ++u) dst[V::fslot(tid, u)] = {v[0][u].x * inv, v[0][u].y * inv};
}

template <class V, int K, int MINW>
__global__ void __launch_bounds__(V::NT, MINW) k_blind_rotate_mw(const u64* __restrict__ small, int n, int L, int beta,
                                                              const c64* __restrict__ bsk, const c64* __restrict__ tw,
                                                              const c64* __restrict__ twist, BrTv tv, int mode,
                                                              u64* __restrict__ out, u64* __restrict__ ct_v,
                                                              u64* __restrict__ refreshed, u64* __restrict__ sign) {
  constexpr int M = V::M, N = V::N, S = V::S, NT = V::NT;
  using Tw = typename V::Tw;
  constexpr int LOG2N2 = 11;
  __shared__ u64 acc[(K + 1) * N];
  __shared__ c64 lds[V::SCRATCH];
  const int tid = threadIdx.x;
  const int64_t c = blockIdx.x;
  const u64* sm = small + (size_t)c * (n + 1);
  const int R = (K + 1) * L;

  Tw T;
  V::load_twiddles(T, tw, tid);
  c64 twv[S];
  int tc[S];
#pragma unroll
  for (int u = 0; u < S; ++u) {
    tc[u] = V::tcoef(tid, u);
    twv[u] = twist[tc[u]];
  }

  const uint32_t bt = modswitch_2n(sm[n], LOG2N2);
  for (int t = tid; t < N; t += NT) {
#pragma unroll
    for (int j = 0; j < K; ++j) acc[j * N + t] = 0;
    const uint32_t idx = (uint32_t)(t + bt) & (2 * N - 1);
    acc[K * N + t] = tv_rot(tv, idx, N);
  }
  __syncthreads();

  for (int i = 0; i < n; ++i) {
    const uint32_t ai = modswitch_2n(sm[i], LOG2N2);
    if (ai == 0) continue;
    c64 outv[K + 1][S];
#pragma unroll
    for (int o = 0; o <= K; ++o)
#pragma unroll
      for (int u = 0; u < S; ++u) outv[o][u] = {0.0, 0.0};
    const c64* G = bsk + (size_t)i * R * (K + 1) * M;
#pragma unroll
    for (int cc = 0; cc <= K; ++cc) {
      const u64* f = acc + cc * N;
      u64 p0[S], p1[S];
#pragma unroll
      for (int u = 0; u < S; ++u) {
        const int t0 = tc[u], t1 = t0 + M;
        const uint32_t i0 = (uint32_t)(t0 - (int)ai) & (2 * N - 1);
        const uint32_t i1 = (uint32_t)(t1 - (int)ai) & (2 * N - 1);
        const u64 r0 = i0 < (uint32_t)N ? f[i0] : (u64)0 - f[i0 - N];
        const u64 r1 = i1 < (uint32_t)N ? f[i1] : (u64)0 - f[i1 - N];
        p0[u] = decompose_packed(r0 - f[t0], beta, L);
        p1[u] = decompose_packed(r1 - f[t1], beta, L);
      }
      if constexpr (V::MULTI) {
        // levels in pairs: both forward FFTs share every relayout
        for (int lvl = 1; lvl <= L; lvl += 2) {
          if (lvl + 1 <= L) {
            c64 v[2][S];
#pragma unroll
            for (int f = 0; f < 2; ++f)
#pragma unroll
              for (int u = 0; u < S; ++u)
                v[f][u] = cmul({(double)digit_of(p0[u], lvl + f, beta, L), (double)digit_of(p1[u], lvl + f, beta, L)},
                               twv[u]);
            V::template forward<2>(v, T, lds, tid);
#pragma unroll
            for (int f = 0; f < 2; ++f) {
              const c64* g = G + (size_t)((cc * L + lvl + f - 1) * (K + 1)) * M;
#pragma unroll
              for (int o = 0; o <= K; ++o)
#pragma unroll
                for (int u = 0; u < S; ++u) cmac(outv[o][u], v[f][u], g[o * M + V::fslot(tid, u)]);
            }
          } else {
            c64 v[1][S];
#pragma unroll
            for (int u = 0; u < S; ++u)
              v[0][u] = cmul({(double)digit_of(p0[u], lvl, beta, L), (double)digit_of(p1[u], lvl, beta, L)}, twv[u]);
            V::template forward<1>(v, T, lds, tid);
            const c64* g = G + (size_t)((cc * L + lvl - 1) * (K + 1)) * M;
#pragma unroll
            for (int o = 0; o <= K; ++o)
#pragma unroll
              for (int u = 0; u < S; ++u) cmac(outv[o][u], v[0][u], g[o * M + V::fslot(tid, u)]);
          }
        }
      } else {
        for (int lvl = 1; lvl <= L; ++lvl) {
          // issue this row's BSK loads first so they fly during the FFT
          const c64* g = G + (size_t)((cc * L + lvl - 1) * (K + 1)) * M;
          c64 kb[K + 1][S];
#pragma unroll
          for (int o = 0; o <= K; ++o)
#pragma unroll
            for (int u = 0; u < S; ++u) kb[o][u] = g[o * M + V::fslot(tid, u)];
          c64 v[S];
#pragma unroll
          for (int u = 0; u < S; ++u)
            v[u] = cmul({(double)digit_of(p0[u], lvl, beta, L), (double)digit_of(p1[u], lvl, beta, L)}, twv[u]);
          V::forward(v, T, lds, tid);
#pragma unroll
          for (int o = 0; o <= K; ++o)
#pragma unroll
            for (int u = 0; u < S; ++u) cmac(outv[o][u], v[u], kb[o][u]);
        }
      }
    }
    __syncthreads();  // every wave has read acc for this step
    if constexpr (V::MULTI) {
      // outputs in pairs (the scratch holds two polynomials)
#pragma unroll
      for (int o = 0; o <= K; o += 2) {
        if (o + 1 <= K) {
          V::template inverse<2>(*reinterpret_cast<c64(*)[2][S]>(&outv[o]), T, lds, tid);
        } else {
          V::template inverse<1>(*reinterpret_cast<c64(*)[1][S]>(&outv[o]), T, lds, tid);
        }
      }
    } else {
#pragma unroll
      for (int o = 0; o <= K; ++o) V::inverse(outv[o], T, lds, tid);
    }
#pragma unroll
    for (int o = 0; o <= K; ++o) {
#pragma unroll
      for (int u = 0; u < S; ++u) {
        const c64 z = cmulc(outv[o][u], twv[u]);
        acc[o * N + tc[u]] += f64_to_torus(z.x);
        acc[o * N + tc[u] + M] += f64_to_torus(z.y);
      }
    }
    __syncthreads();
  }

  const int W = K * N + 1;
  for (int j = 0; j < K; ++j) {
    for (int t = tid; t < N; t += NT) {
      const u64 a = (t == 0) ? acc[j * N] : (u64)0 - acc[j * N + N - t];
      br_emit(mode, a, false, tv, (size_t)c * W + j * N + t, out, ct_v, refreshed, sign);
    }
  }
  if (tid == 0) br_emit(mode, acc[K * N], true, tv, (size_t)c * W + K * N, out, ct_v, refreshed, sign);
}

// ---- blind rotation v4 (br_v4.h): a wave per GLWE component ---------------
// BSK conversion: one wave per polynomial, stored [poly][u][lane] (layout LC
// of the forward transform) and scaled by 1/M.
__global__ void __launch_bounds__(64) k_bsk_to_fft_v4(const u64* __restrict__ bsk, int npoly,
                                                      const c64* __restrict__ tw4, c64* __restrict__ out) {
  using namespace v4;
  __shared__ c64 twl[NTW];
  __shared__ c64 scr[SCR];
  const int lane = threadIdx.x;
  fill_tables(twl, tw4, lane, 64);
  __syncthreads();
  const double inv = 1.0 / (double)M;
  for (int poly = blockIdx.x; poly < npoly; poly += gridDim.x) {
    const u64* src = bsk + (size_t)poly * N;
    c64 v[S];
#pragma unroll
    for (int u = 0; u < S; ++u) {
      const int t = u * 64 + lane;
      v[u] = {(double)(int64_t)src[t], (double)(int64_t)src[t + M]};
    }
    forward(v, twl, scr, lane);
    c64* dst = out + (size_t)poly * M;
#pragma unroll
    for (int u = 0; u < S; ++u) dst[u * 64 + lane] = {v[u].x * inv, v[u].y * inv};
  }
}

// Balanced gadget digits of x (level 0 = most significant) into d[0..L):
// round to the top L*beta bits, then LSB-first each digit is the sign
// extension of its beta bits (>= B/2 becomes negative), subtracted before
// the next digit is read (that is the carry).
template <int L, bool A32>
__device__ __forceinline__ void decompose_v4(typename v4::Acc<A32>::T x, int beta, int (&d)[L]) {
  const int prec = L * beta;
  if constexpr (A32) {
    uint32_t r = ((x >> (31 - prec)) + 1) >> 1;
#pragma unroll
    for (int i = 0; i < L; ++i) {
      const int di = __builtin_amdgcn_sbfe((int)r, i * beta, beta);
      d[L - 1 - i] = di;
      if (i + 1 < L) r -= (uint32_t)di << (i * beta);
    }
  } else {
    u64 r = ((x >> (63 - prec)) + 1) >> 1;
#pragma unroll
    for (int i = 0; i < L; ++i) {
      const int64_t di = (int64_t)(r << (64 - (i + 1) * beta)) >> (64 - beta);
      d[L - 1 - i] = (int)di;
      if (i + 1 < L) r -= (u64)di << (i * beta);
    }
  }
}

// Phase timestamps (DBG bit 7): wave 0 of workgroup 0 records s_memtime at
// the phase boundaries of steps 100..103 (tools/prof_br.py --stamps).
__device__ unsigned long long g_v4_stamps[4][16];
// ... and every workgroup's {s_memrealtime at start, at end, HW_ID} (first 2048)
__device__ unsigned long long g_v4_span[2048][3];
#define V4_STAMP(k)                                                                        \
  do {                                                                                     \
    if constexpr ((DBG & 128) != 0) stamp_[k] = __builtin_amdgcn_s_memtime();              \
  } while (0)

// DBG != 0 only for timing experiments (tools/prof_br.py, FHEICP_V4_DBG):
// 1 twiddles from a register, 2 no BSK loads, 4 no barriers, 8 no FFT
// relayout, 16 no LDS rotation, 32 no LDS reads of the other components,
// 128 phase timestamps (results correct).
constexpr int FL_SYNC = 1;
template <int L, bool A32, int DBG = 0, int G = 2, bool FL = false>
__global__ void __launch_bounds__(v4::nthreads(G), A32 ? 3 : 2) k_blind_rotate_v4(const u64* __restrict__ small, int64_t count, int n,
                                                              int beta, const c64* __restrict__ bsk,
                                                              const c64* __restrict__ tw4, BrTv tv, int mode,
                                                              u64* __restrict__ out, u64* __restrict__ ct_v,
                                                              u64* __restrict__ refreshed, u64* __restrict__ sign) {
  using namespace v4;
  using AT = Acc<A32>;
  using T = typename AT::T;
  constexpr int NT = nthreads(G);
  __shared__ c64 xbuf[G * WPC * SCR];  // one 8.5 KB slot per wave
  __shared__ c64 twl[NTW];
  __shared__ uint16_t atab[G][NMAX + 1];
  __shared__ uint32_t ctflag[G][2];  // FL: per-ciphertext W / R hand-off counts
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = w / WPC, comp = w - g * WPC;
  const int64_t c = (int64_t)blockIdx.x * G + g;
  c64* slot = xbuf + (g * WPC + comp) * SCR;
  const c64* ctslots = xbuf + g * WPC * SCR;
  T* sa = reinterpret_cast<T*>(slot);

  if constexpr ((DBG & 128) != 0)
    if (tid == 0 && blockIdx.x < 2048) {
      g_v4_span[blockIdx.x][0] = __builtin_amdgcn_s_memrealtime();
      g_v4_span[blockIdx.x][2] = (unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 4);
    }
  fill_tables(twl, tw4, tid, NT);
  for (int x = tid; x < G * (n + 1); x += NT) {
    const int gg = x / (n + 1), ii = x - gg * (n + 1);
    const int64_t cc = (int64_t)blockIdx.x * G + gg;
    atab[gg][ii] = cc < count ? (uint16_t)modswitch_2n(small[(size_t)cc * (n + 1) + ii], 11) : (uint16_t)0;
  }
  if (tid < 2 * G) ctflag[tid >> 1][tid & 1] = 0;
  __syncthreads();
  uint32_t* fW = &ctflag[g][0];
  uint32_t* fR = &ctflag[g][1];
  uint32_t phase = 0;  // FL: hand-offs completed by this ciphertext

  T acc[2 * S];
  {
    const uint32_t bt = atab[g][n];
#pragma unroll
    for (int s = 0; s < 2 * S; ++s) {
      const uint32_t idx = (uint32_t)(s * 64 + lane + bt) & (2 * N - 1);
      acc[s] = comp == K ? AT::from64(tv_rot(tv, idx, N)) : (T)0;
    }
  }

  constexpr int R = WPC * L;
  const c64 wf = {0.5 + (double)beta * 1e-3, (double)L * 1e-3};  // DBG stand-in value
  for (int i = 0; i < n; ++i) {
    // FL: per-ciphertext hand-offs within a step, but one workgroup barrier
    // every FL_SYNC steps bounds how far the oldest ciphertext (highest issue
    // priority) runs ahead of the others
    if constexpr (FL && (DBG & 4) == 0)
      if ((i & (FL_SYNC - 1)) == 0) lds_barrier();
    const uint32_t a = __builtin_amdgcn_readfirstlane((uint32_t)atab[g][i]);
    [[maybe_unused]] unsigned long long stamp_[16];
    V4_STAMP(0);
    if constexpr ((DBG & 128) != 0) stamp_[14] = __builtin_amdgcn_s_memrealtime();
    // X^a ACC - ACC through the wave's slot, then the gadget digits
    if constexpr ((DBG & 16) == 0) {
#pragma unroll
      for (int s = 0; s < 2 * S; ++s) sa[s * 64 + lane] = acc[s];  // own slot: in-order DS, no wait
    }
    c64 v[S];
    uint32_t dg[L > 1 ? L - 1 : 1][S];  // levels >= 1, two int16 digits per word
    T rot[2 * S];  // all 16 rotated words as one batch of LDS reads
#pragma unroll
    for (int s = 0; s < 2 * S; ++s) {
      const uint32_t src = (uint32_t)(s * 64 + lane - (int)a) & (2 * N - 1);
      rot[s] = (DBG & 16) ? acc[(s + 1) & 15] + (T)src : sa[src & (N - 1)];
    }
    // coefficient pairs (t, t + N/2) fold into one complex point
#pragma unroll
    for (int s = 0; s < S; ++s) {
      int d[2][L];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const uint32_t src = (uint32_t)((s + h * S) * 64 + lane - (int)a) & (2 * N - 1);
        const T r = src >= (uint32_t)N ? (T)0 - rot[s + h * S] : rot[s + h * S];
        decompose_v4<L, A32>((T)(r - acc[s + h * S]), beta, d[h]);
      }
      v[s] = {(double)d[0][0], (double)d[1][0]};
#pragma unroll
      for (int l = 1; l < L; ++l) dg[l - 1][s] = (uint32_t)(d[0][l] & 0xffff) | ((uint32_t)d[1][l] << 16);
    }

    V4_STAMP(1);
    c64 mac[S];
#pragma unroll
    for (int u = 0; u < S; ++u) mac[u] = {0.0, 0.0};
    const c64* Gi = bsk + (size_t)i * R * WPC * M;
#pragma unroll
    for (int lv = 0; lv < L; ++lv) {
      if (lv > 0) {
#pragma unroll
        for (int u = 0; u < S; ++u)
          v[u] = {(double)(int16_t)(dg[lv - 1][u] & 0xffff), (double)((int32_t)dg[lv - 1][u] >> 16)};
      }
      // own-component BSK row: loads fly during the transform (which folds
      // the twist in); the u64 kernels load it after the transform (VGPRs)
      constexpr bool PF = A32 || G <= 2;  // u64 kernels at 4 per workgroup: load late (VGPRs)
      const c64* gpo = Gi + ((size_t)(comp * L + lv) * WPC + comp) * M;
      c64 kb[PF ? S : 1];
      if constexpr (PF) {
#pragma unroll
        for (int u = 0; u < S; ++u) kb[u] = (DBG & 2) ? c64{wf.x + u, wf.y} : gpo[u * 64 + lane];
      }
      // FL: the others must have read this slot's previous F before the
      // transform's relayouts overwrite it
      if constexpr (FL && (DBG & 4) == 0)
        if (lv > 0) ct_wait(fR, 3 * phase);
      forward<DBG>(v, twl, slot, lane, wf);
      V4_STAMP(2 + 5 * lv);
#pragma unroll
      for (int u = 0; u < S; ++u) slot[u * 64 + lane] = v[u];
      // own component first (no other wave needed), then the two other rows'
      // BSK loads fly across the barrier
#pragma unroll
      for (int u = 0; u < S; ++u) {
        if constexpr (PF) cmac(mac[u], v[u], kb[u]);
        else cmac(mac[u], v[u], (DBG & 2) ? c64{wf.x + u, wf.y} : gpo[u * 64 + lane]);
      }
      // the other two rows' BSK: A32 kernels issue the loads before the
      // barrier (they fly across it); the u64-accumulator kernels load them
      // after it, half a row at a time, to stay within 168 VGPRs (3 waves
      // per SIMD, 4 ciphertexts per workgroup)
      c64 kx[PF ? K : 1][PF ? S : 1];
      if constexpr (PF) {
#pragma unroll
        for (int ci = 0; ci < K; ++ci) {
          const int cin = comp + 1 + ci >= WPC ? comp + 1 + ci - WPC : comp + 1 + ci;
          const c64* gp = Gi + ((size_t)(cin * L + lv) * WPC + comp) * M;
#pragma unroll
          for (int u = 0; u < S; ++u) kx[ci][u] = (DBG & 2) ? c64{wf.x + ci, wf.y + u} : gp[u * 64 + lane];
        }
      }
      V4_STAMP(3 + 5 * lv);
      if constexpr ((DBG & 4) == 0) {
        if constexpr (FL) {
          ct_signal(fW);
          ct_wait(fW, 3 * (phase + 1));
        } else {
          lds_barrier();
        }
      }
      V4_STAMP(4 + 5 * lv);
#pragma unroll
      for (int ci = 0; ci < K; ++ci) {
        const int cin = comp + 1 + ci >= WPC ? comp + 1 + ci - WPC : comp + 1 + ci;
        const c64* fs = ctslots + cin * SCR;
        const c64* gp = Gi + ((size_t)(cin * L + lv) * WPC + comp) * M;
#pragma unroll
        for (int hh = 0; hh < 2; ++hh) {  // F in halves: bounds register use at the peak
          c64 fv[S / 2], kv[S / 2];
#pragma unroll
          for (int u = 0; u < S / 2; ++u) {
            fv[u] = (DBG & 32) ? v[hh * 4 + u] : fs[(hh * 4 + u) * 64 + lane];
            if constexpr (PF) kv[u] = kx[ci][hh * 4 + u];
            else kv[u] = (DBG & 2) ? c64{wf.x + ci, wf.y + u} : gp[(hh * 4 + u) * 64 + lane];
          }
#pragma unroll
          for (int u = 0; u < S / 2; ++u) cmac(mac[hh * 4 + u], fv[u], kv[u]);
        }
      }
      V4_STAMP(5 + 5 * lv);
      if constexpr ((DBG & 4) == 0) {
        if constexpr (FL) {
          ct_signal(fR);
          ++phase;
        } else {
          lds_barrier();
        }
      }
      V4_STAMP(6 + 5 * lv);
    }
    if constexpr (FL && (DBG & 4) == 0) ct_wait(fR, 3 * phase);
    inverse<DBG>(mac, twl, slot, lane, wf);
    V4_STAMP(12);
#pragma unroll
    for (int u = 0; u < S; ++u) {
      acc[u] += AT::from_f64(mac[u].x);
      acc[u + S] += AT::from_f64(mac[u].y);
    }
    V4_STAMP(13);
    if constexpr ((DBG & 128) != 0) stamp_[15] = __builtin_amdgcn_s_memrealtime();
    if constexpr ((DBG & 128) != 0)
      if (blockIdx.x == 0 && w == 0 && i >= 100 && i < 104 && lane < 16) {
        unsigned long long t_ = 0;
#pragma unroll
        for (int k = 0; k < 16; ++k) t_ = lane == k ? stamp_[k] : t_;
        g_v4_stamps[i - 100][lane] = t_;
      }
  }

  if constexpr ((DBG & 128) != 0)
    if (tid == 0 && blockIdx.x < 2048) g_v4_span[blockIdx.x][1] = __builtin_amdgcn_s_memrealtime();
  // sample extraction of coefficient 0: mask word t of component comp < K
  // is -ACC[N - t] (t > 0), read reversed through the slot
#pragma unroll
  for (int s = 0; s < 2 * S; ++s) sa[s * 64 + lane] = acc[s];
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  if (c < count) {
    const int W = K * N + 1;
    if (comp < K) {
#pragma unroll
      for (int s = 0; s < 2 * S; ++s) {
        const int t = s * 64 + lane;
        const u64 x = t == 0 ? AT::to64(sa[0]) : (u64)0 - AT::to64(sa[N - t]);
        br_emit(mode, x, false, tv, (size_t)c * W + comp * N + t, out, ct_v, refreshed, sign);
      }
    } else if (lane == 0) {
      br_emit(mode, AT::to64(acc[0]), true, tv, (size_t)c * W + K * N, out, ct_v, refreshed, sign);
    }
  }
}

// acc_out[b] = v[b] + T
__global__ void k_add_scalar(const int64_t* __restrict__ v, int64_t B, int64_t T, int64_t* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < B) out[i] = v[i] + T;
}

// Single-workgroup top-k by (acc desc, idx asc) over entries not below the
// threshold. k passes; pass p selects the largest key strictly smaller than
// the key chosen in pass p-1 (keys are unique because indices are).
__global__ void __launch_bounds__(1024) k_topk(const int64_t* __restrict__ accv, const int64_t* __restrict__ below,
                                               int64_t B, int64_t base_idx, int kk, int64_t* __restrict__ oa,
                                               int64_t* __restrict__ oi) {
  __shared__ int64_t sa[16], si[16];
  __shared__ int64_t last_a, last_i;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  if (tid == 0) {
    last_a = INT64_MAX;
    last_i = -1;
  }
  __syncthreads();
  for (int p = 0; p < kk; ++p) {
    const int64_t la = last_a, li = last_i;
    int64_t ba = INT64_MIN, bi = -1;
    for (int64_t x = tid; x < B; x += 1024) {
      if (below && below[x]) continue;
      const int64_t a = accv[x];
      // strictly after (la, li) in (acc desc, idx asc) order
      const bool after = (a < la) || (a == la && x > li);
      if (!after) continue;
      if (bi < 0 || a > ba || (a == ba && x < bi)) {
        ba = a;
        bi = x;
      }
    }
    for (int off = 32; off > 0; off >>= 1) {
      const int64_t oa2 = __shfl_down(ba, off, 64), oi2 = __shfl_down(bi, off, 64);
      if (oi2 >= 0 && (bi < 0 || oa2 > ba || (oa2 == ba && oi2 < bi))) {
        ba = oa2;
        bi = oi2;
      }
    }
    if (lane == 0) {
      sa[w] = ba;
      si[w] = bi;
    }
    __syncthreads();
    if (tid == 0) {
      int64_t fa = INT64_MIN, fi = -1;
      for (int q = 0; q < 16; ++q) {
        if (si[q] >= 0 && (fi < 0 || sa[q] > fa || (sa[q] == fa && si[q] < fi))) {
          fa = sa[q];
          fi = si[q];
        }
      }
      oa[p] = fi >= 0 ? fa : INT64_MIN;
      oi[p] = fi >= 0 ? fi + base_idx : -1;
      if (fi >= 0) {
        last_a = fa;
        last_i = fi;
      } else {
        last_a = INT64_MIN;  // nothing left: every later pass finds nothing
        last_i = INT64_MAX;
      }
    }
    __syncthreads();
  }
}

// ============================================================ host =========
struct ProfAcc {
  std::vector<std::pair<hipEvent_t, hipEvent_t>> ev;
  double ms = 0;
  int64_t launches = 0, items = 0;
};

struct fhe_ctx {
  fhe_params p{};
  int device = -1;
  std::string err;
  bool keys = false;
  u64 *s_small = nullptr, *s_big = nullptr, *bsk = nullptr, *ksk = nullptr, *ksk_colsum = nullptr;
  c64 *bsk_fft = nullptr, *tw = nullptr, *twist = nullptr, *tw4 = nullptr;
  // workspace
  void* ws = nullptr;
  size_t ws_bytes = 0;
  bool prof = false;
  ProfAcc prof_br, prof_ks;
  int v4_g = 4;        // v4 ciphertexts per workgroup (FHEICP_V4_G = 1, 2 or 4)
  int v4_fl = 0;       // v4 per-ciphertext LDS hand-offs instead of s_barrier (FHEICP_V4_FL=1)
  int br_variant = 4;  // N=1024 blind rotation: 4 = a wave per GLWE component (k = 2, default), 2, 3
  int v4_dbg = 0;      // timing experiments only (FHEICP_V4_DBG), wrong results
  // i8-MFMA key switch: key byte planes and a digit/body workspace
  int8_t* ksk8 = nullptr;
  void* ks_ws = nullptr;
  size_t ks_ws_bytes = 0;
  int ks_variant = 2;  // 2 = MFMA (default when ks_level == 4), 1 = VALU split-K
};

static std::mutex g_err_mu;
static std::string g_err;

static int fail(fhe_ctx* ctx, int code, const std::string& msg) {
  if (ctx) ctx->err = msg;
  std::lock_guard<std::mutex> lk(g_err_mu);
  g_err = msg;
  return code;
}
#define HIPCHK(ctx, x)                                                                          \
  do {                                                                                          \
    hipError_t e_ = (x);                                                                        \
    if (e_ != hipSuccess) return fail(ctx, FHE_E_DEVICE, std::string(#x ": ") + hipGetErrorString(e_)); \
  } while (0)

static int ilog2i(int x) {
  int r = 0;
  while ((1 << r) < x) ++r;
  return r;
}

static int validate(const fhe_params* p, std::string& why) {
  if (!p) { why = "null params"; return -1; }
  if (!(p->N == 256 || p->N == 512 || p->N == 1024 || p->N == 2048)) { why = "N must be 256/512/1024/2048"; return -1; }
  if (p->k < 1 || p->k > 2) { why = "k must be 1 or 2"; return -1; }
  if (p->N == 2048 && p->k != 1) { why = "N=2048 requires k=1"; return -1; }
  if (p->n < 1 || p->n > 4096) { why = "n out of range"; return -1; }
  if (p->pbs_level < 1 || p->pbs_level > 8 || p->pbs_base_log < 1 || p->pbs_level * p->pbs_base_log > 62) {
    why = "pbs decomposition out of range"; return -1;
  }
  if (p->ks_level < 1 || p->ks_level > 8 || p->ks_base_log < 1 || p->ks_base_log > 7 ||
      p->ks_level * p->ks_base_log > 62) {
    why = "ks decomposition out of range (base_log <= 7 for int8 digits)"; return -1;
  }
  if (p->msg_bits < 2 || p->msg_bits > 40) { why = "msg_bits must be in [2, 40]"; return -1; }
  if (p->lwe_noise_bits < 0 || p->lwe_noise_bits > 60 || p->glwe_noise_bits < 0 || p->glwe_noise_bits > 60) {
    why = "noise bits out of range"; return -1;
  }
  if (p->sign_digit_bits != 0 && (p->sign_digit_bits < 3 || p->sign_digit_bits > 4)) {
    why = "sign_digit_bits must be 0 (auto), 3 or 4"; return -1;
  }
  return 0;
}

static double tuniform_var(int b) { return (std::ldexp(1.0, 2 * b + 1) + 1.0) / 6.0; }

// Decision margin in sigmas of the worst round of a d-bit digit sign
// extraction: the staircase round of the lowest digit, margin 2^-(d+1) of the
// torus, the preceding bootstrap's noise amplified by 2^(P-d), plus key
// switch and modulus switch noise. Same model as fheicp/params.py
// noise_report.
static double digit_margin_sigmas(const fhe_params& p, int d) {
  const double q2 = std::ldexp(1.0, 128);
  const double s2_bsk = tuniform_var(p.glwe_noise_bits) / q2, s2_ksk = tuniform_var(p.lwe_noise_bits) / q2;
  const double B = std::ldexp(1.0, p.pbs_base_log), Bk = std::ldexp(1.0, p.ks_base_log);
  const double rows = (double)p.pbs_level * (p.k + 1) * p.N;
  const double v_pbs = p.n * rows * (B * B + 2) / 12.0 * s2_bsk +
                       p.n * (1 + p.k * p.N / 2.0) / (12.0 * std::pow(B, 2.0 * p.pbs_level));
  const double v_ks = (double)p.k * p.N * p.ks_level * (Bk * Bk + 2) / 12.0 * s2_ksk +
                      p.k * p.N / 2.0 * std::ldexp(1.0, -2 * p.ks_level * p.ks_base_log) / 12.0;
  const double v_ms = (p.n / 2.0 + 1) / 12.0 / ((2.0 * p.N) * (2.0 * p.N));
  const double v = v_pbs * std::ldexp(1.0, 2 * (p.msg_bits - d)) + v_ks + v_ms;
  return std::ldexp(1.0, -(d + 1)) / std::sqrt(v);
}

static int sign_digits(const fhe_params& p) {
  if (p.msg_bits < 4) return 0;
  if (p.sign_digit_bits) return std::min(p.sign_digit_bits, (int)p.msg_bits);
  for (int d = std::min(4, (int)p.msg_bits); d > 3; --d)
    if (digit_margin_sigmas(p, d) >= 9.2) return d;
  return 3;
}

extern "C" {

size_t fhe_bsk_words(const fhe_params* p) {
  return (size_t)p->n * (p->k + 1) * p->pbs_level * (p->k + 1) * p->N;
}
size_t fhe_ksk_words(const fhe_params* p) { return (size_t)p->k * p->N * p->ks_level * (p->n + 1); }
size_t fhe_big_lwe_words(const fhe_params* p) { return (size_t)p->k * p->N + 1; }
size_t fhe_small_lwe_words(const fhe_params* p) { return (size_t)p->n + 1; }

const char* fhe_last_error(const fhe_ctx* ctx) {
  if (ctx) return ctx->err.c_str();
  std::lock_guard<std::mutex> lk(g_err_mu);
  return g_err.c_str();
}

int fhe_get_params(const fhe_ctx* ctx, fhe_params* out) {
  if (!ctx || !out) return FHE_E_ARG;
  *out = ctx->p;
  return FHE_OK;
}

int fhe_ctx_create(const fhe_params* params, int device, fhe_ctx** out) {
  std::string why;
  if (!out) return fail(nullptr, FHE_E_ARG, "out is null");
  *out = nullptr;
  if (validate(params, why)) return fail(nullptr, FHE_E_ARG, why);
  fhe_ctx* ctx = new fhe_ctx();
  ctx->p = *params;
  ctx->device = device;
  if (const char* e = getenv("FHEICP_BR_VARIANT")) {
    const int v = atoi(e);
    ctx->br_variant = (v == 2 || v == 3 || v == 4) ? v : 4;
  }
  if (const char* e = getenv("FHEICP_V4_DBG")) ctx->v4_dbg = atoi(e);
  if (const char* e = getenv("FHEICP_V4_G")) {
    const int g = atoi(e);
    ctx->v4_g = (g == 1 || g == 2 || g == 4) ? g : 4;
  }
  if (const char* e = getenv("FHEICP_V4_FL")) ctx->v4_fl = atoi(e) != 0;
  if (const char* e = getenv("FHEICP_KS_VARIANT")) ctx->ks_variant = atoi(e) == 1 ? 1 : 2;
  if (params->ks_level != 4 || (params->k * params->N * 4) % 64 != 0) ctx->ks_variant = 1;
  // v4 covers k = 2, n <= 1023 at N = 1024; otherwise the two-wave kernel
  // (measured: v4 wins at gadget levels <= 3, e.g. 21.6 vs 23.6 ms at P=21; from
  // level 4 its 64-bit accumulator spills and v2 is faster, 40.6 vs 53.0 ms at P=26)
  if (ctx->br_variant == 4 && !(params->k == 2 && params->n <= v4::NMAX && params->pbs_level <= 3 &&
                                 (params->pbs_level == 1 || params->pbs_base_log <= 16)))
    ctx->br_variant = 2;
  if (device >= 0) {
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device >= ndev) {
      delete ctx;
      return fail(nullptr, FHE_E_DEVICE, "no HIP device " + std::to_string(device));
    }
    if (hipSetDevice(device) != hipSuccess) {
      delete ctx;
      return fail(nullptr, FHE_E_DEVICE, "hipSetDevice failed");
    }
    const int N = params->N, M = N / 2;
    std::vector<c64> tw(M / 2), twist(M);
    for (int x = 0; x < M / 2; ++x) {
      const long double ang = 2.0L * 3.14159265358979323846264338327950288L * (long double)x / (long double)M;
      tw[x] = {(double)cosl(ang), (double)sinl(ang)};
    }
    for (int t = 0; t < M; ++t) {
      const long double ang = 3.14159265358979323846264338327950288L * (long double)t / (long double)N;
      twist[t] = {(double)cosl(ang), (double)sinl(ang)};
    }
    if (N == 1024) {  // v4 per-lane twiddles (br_v4.h), long double
      const long double PI = 3.14159265358979323846264338327950288L;
      std::vector<c64> t4(v4::NTW);
      for (int m = 0; m < 8; ++m)
        for (int lane = 0; lane < 64; ++lane) {
          const long double ang = PI * (long double)lane * (long double)(1 + 4 * m) / 1024.0L;
          t4[m * 64 + lane] = {(double)cosl(ang), (double)sinl(ang)};
        }
      for (int m = 1; m < 8; ++m)
        for (int L = 0; L < 8; ++L) {
          const long double ang = 2.0L * PI * (long double)(L * m) / 64.0L;
          t4[v4::NTA + (m - 1) * 8 + L] = {(double)cosl(ang), (double)sinl(ang)};
        }
      if (hipMalloc(&ctx->tw4, sizeof(c64) * t4.size()) != hipSuccess ||
          hipMemcpy(ctx->tw4, t4.data(), sizeof(c64) * t4.size(), hipMemcpyHostToDevice) != hipSuccess) {
        fhe_ctx_destroy(ctx);
        return fail(nullptr, FHE_E_DEVICE, "twiddle upload failed");
      }
    }
    if (hipMalloc(&ctx->tw, sizeof(c64) * tw.size()) != hipSuccess ||
        hipMalloc(&ctx->twist, sizeof(c64) * twist.size()) != hipSuccess ||
        hipMemcpy(ctx->tw, tw.data(), sizeof(c64) * tw.size(), hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(ctx->twist, twist.data(), sizeof(c64) * twist.size(), hipMemcpyHostToDevice) != hipSuccess) {
      fhe_ctx_destroy(ctx);
      return fail(nullptr, FHE_E_DEVICE, "table upload failed");
    }
  }
  *out = ctx;
  return FHE_OK;
}

static void free_ev(ProfAcc& a) {
  for (auto& e : a.ev) {
    hipEventDestroy(e.first);
    hipEventDestroy(e.second);
  }
  a.ev.clear();
}

void fhe_ctx_destroy(fhe_ctx* ctx) {
  if (!ctx) return;
  if (ctx->device >= 0) {
    hipSetDevice(ctx->device);
    hipFree(ctx->s_small); hipFree(ctx->s_big); hipFree(ctx->bsk); hipFree(ctx->ksk); hipFree(ctx->ksk_colsum);
    hipFree(ctx->bsk_fft); hipFree(ctx->tw); hipFree(ctx->twist); hipFree(ctx->ws);
    hipFree(ctx->ksk8); hipFree(ctx->ks_ws); hipFree(ctx->tw4);
    free_ev(ctx->prof_br);
    free_ev(ctx->prof_ks);
  }
  delete ctx;
}

int fhe_set_msg_bits(fhe_ctx* ctx, int32_t msg_bits) {
  if (!ctx) return fail(nullptr, FHE_E_ARG, "null ctx");
  fhe_params q = ctx->p;
  q.msg_bits = msg_bits;
  std::string why;
  if (validate(&q, why)) return fail(ctx, FHE_E_ARG, why);
  ctx->p = q;
  return FHE_OK;
}

static int need_device(fhe_ctx* ctx) {
  if (!ctx) return fail(nullptr, FHE_E_ARG, "null ctx");
  if (ctx->device < 0) return fail(ctx, FHE_E_DEVICE, "host-only context");
  if (hipSetDevice(ctx->device) != hipSuccess) return fail(ctx, FHE_E_DEVICE, "hipSetDevice failed");
  return FHE_OK;
}
static int need_keys(fhe_ctx* ctx) {
  int rc = need_device(ctx);
  if (rc) return rc;
  if (!ctx->keys) return fail(ctx, FHE_E_STATE, "no keys: call fhe_keygen or fhe_import_keys");
  return FHE_OK;
}

static int alloc_keys(fhe_ctx* ctx) {
  const fhe_params& p = ctx->p;
  if (ctx->s_small) return FHE_OK;
  HIPCHK(ctx, hipMalloc(&ctx->s_small, 8 * (size_t)p.n));
  HIPCHK(ctx, hipMalloc(&ctx->s_big, 8 * (size_t)p.k * p.N));
  HIPCHK(ctx, hipMalloc(&ctx->bsk, 8 * fhe_bsk_words(&p)));
  HIPCHK(ctx, hipMalloc(&ctx->ksk, 8 * fhe_ksk_words(&p)));
  HIPCHK(ctx, hipMalloc(&ctx->ksk_colsum, 8 * (size_t)(p.n + 1)));
  HIPCHK(ctx, hipMalloc(&ctx->bsk_fft, sizeof(c64) * fhe_bsk_words(&p) / 2));
  return FHE_OK;
}

static int convert_bsk(fhe_ctx* ctx, hipStream_t st) {
  const fhe_params& p = ctx->p;
  hipLaunchKernelGGL(k_ksk_colsum, dim3((p.n + 1 + 255) / 256), dim3(256), 0, st, ctx->ksk, p.k * p.N * p.ks_level,
                     p.n, ctx->ksk_colsum);
  if (ctx->ks_variant == 2) {
    const int K = p.k * p.N * p.ks_level, n1 = p.n + 1, NB = (n1 + KSM_NB_COLS - 1) / KSM_NB_COLS;
    if (!ctx->ksk8) HIPCHK(ctx, hipMalloc(&ctx->ksk8, (size_t)K * NB * 16 * 8));
    const int64_t tot = (int64_t)K * NB * 16;
    hipLaunchKernelGGL(k_ksk_to_i8, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, st, ctx->ksk, K, n1, NB,
                       ctx->ksk8);
  }
  const int npoly = (int)(fhe_bsk_words(&p) / p.N);
  switch (p.N) {
    case 256: hipLaunchKernelGGL(k_bsk_to_fft<7>, dim3(npoly), dim3(64), 0, st, ctx->bsk, npoly, ctx->tw, ctx->twist, ctx->bsk_fft); break;
    case 512: hipLaunchKernelGGL(k_bsk_to_fft<8>, dim3(npoly), dim3(64), 0, st, ctx->bsk, npoly, ctx->tw, ctx->twist, ctx->bsk_fft); break;
    case 1024:
      if (ctx->br_variant == 4)
        hipLaunchKernelGGL(k_bsk_to_fft_v4, dim3(std::min(npoly, 4096)), dim3(64), 0, st, ctx->bsk, npoly, ctx->tw4,
                           ctx->bsk_fft);
      else if (ctx->br_variant == 3)
        hipLaunchKernelGGL(k_bsk_to_fft_mw<V3>, dim3(npoly), dim3(V3::NT), 0, st, ctx->bsk, npoly, ctx->tw, ctx->twist, ctx->bsk_fft);
      else
        hipLaunchKernelGGL(k_bsk_to_fft_mw<V2>, dim3(npoly), dim3(V2::NT), 0, st, ctx->bsk, npoly, ctx->tw, ctx->twist, ctx->bsk_fft);
      break;
    case 2048: hipLaunchKernelGGL(k_bsk_to_fft<10>, dim3(npoly), dim3(64), 0, st, ctx->bsk, npoly, ctx->tw, ctx->twist, ctx->bsk_fft); break;
  }
  HIPCHK(ctx, hipGetLastError());
  return FHE_OK;
}

int fhe_keygen_key(fhe_ctx* ctx, const uint32_t h_key[8], void* stream) {
  int rc = need_device(ctx);
  if (rc) return rc;
  if (!h_key) return fail(ctx, FHE_E_ARG, "null key");
  rc = alloc_keys(ctx);
  if (rc) return rc;
  const fhe_params& p = ctx->p;
  hipStream_t st = (hipStream_t)stream;
  ChaKey K;
  memcpy(K.w, h_key, 32);
  const int big = p.k * p.N;
  const int mx = std::max(p.n, big);
  hipLaunchKernelGGL(k_keygen_secrets, dim3((mx + 255) / 256), dim3(256), 0, st, K, p.n, big, ctx->s_small, ctx->s_big);
  const int rows_bsk = p.n * (p.k + 1) * p.pbs_level;
  const size_t shm = 8 * (size_t)p.N + p.N;
  hipLaunchKernelGGL(k_keygen_bsk, dim3(rows_bsk), dim3(256), shm, st, K, p.N, p.k, p.pbs_level, p.pbs_base_log,
                     p.glwe_noise_bits, ctx->s_small, ctx->s_big, ctx->bsk);
  hipLaunchKernelGGL(k_keygen_ksk, dim3(big * p.ks_level), dim3(256), 0, st, K, p.n, p.ks_level, p.ks_base_log,
                     p.lwe_noise_bits, ctx->s_small, ctx->s_big, ctx->ksk);
  HIPCHK(ctx, hipGetLastError());
  rc = convert_bsk(ctx, st);
  if (rc) return rc;
  HIPCHK(ctx, hipStreamSynchronize(st));
  ctx->keys = true;
  return FHE_OK;
}

int fhe_keygen(fhe_ctx* ctx, uint64_t seed, void* stream) {
  ChaKey K = key_from_seed(seed);
  return fhe_keygen_key(ctx, K.w, stream);
}

int fhe_export_keys(fhe_ctx* ctx, uint64_t* h_s_small, uint64_t* h_s_big, uint64_t* h_bsk, uint64_t* h_ksk) {
  int rc = need_keys(ctx);
  if (rc) return rc;
  const fhe_params& p = ctx->p;
  HIPCHK(ctx, hipDeviceSynchronize());
  if (h_s_small) HIPCHK(ctx, hipMemcpy(h_s_small, ctx->s_small, 8 * (size_t)p.n, hipMemcpyDeviceToHost));
  if (h_s_big) HIPCHK(ctx, hipMemcpy(h_s_big, ctx->s_big, 8 * (size_t)p.k * p.N, hipMemcpyDeviceToHost));
  if (h_bsk) HIPCHK(ctx, hipMemcpy(h_bsk, ctx->bsk, 8 * fhe_bsk_words(&p), hipMemcpyDeviceToHost));
  if (h_ksk) HIPCHK(ctx, hipMemcpy(h_ksk, ctx->ksk, 8 * fhe_ksk_words(&p), hipMemcpyDeviceToHost));
  return FHE_OK;
}

int fhe_import_keys(fhe_ctx* ctx, const uint64_t* h_s_small, const uint64_t* h_s_big, const uint64_t* h_bsk,
                    const uint64_t* h_ksk) {
  int rc = need_device(ctx);
  if (rc) return rc;
  if (!h_s_small || !h_s_big || !h_bsk || !h_ksk) return fail(ctx, FHE_E_ARG, "all four key buffers are required");
  rc = alloc_keys(ctx);
  if (rc) return rc;
  const fhe_params& p = ctx->p;
  HIPCHK(ctx, hipMemcpy(ctx->s_small, h_s_small, 8 * (size_t)p.n, hipMemcpyHostToDevice));
  HIPCHK(ctx, hipMemcpy(ctx->s_big, h_s_big, 8 * (size_t)p.k * p.N, hipMemcpyHostToDevice));
  HIPCHK(ctx, hipMemcpy(ctx->bsk, h_bsk, 8 * fhe_bsk_words(&p), hipMemcpyHostToDevice));
  HIPCHK(ctx, hipMemcpy(ctx->ksk, h_ksk, 8 * fhe_ksk_words(&p), hipMemcpyHostToDevice));
  rc = convert_bsk(ctx, nullptr);
  if (rc) return rc;
  HIPCHK(ctx, hipDeviceSynchronize());
  ctx->keys = true;
  return FHE_OK;
}

int fhe_encrypt_batch(fhe_ctx* ctx, const int64_t* d_msg, int64_t count, uint64_t seed, uint64_t id0,
                      uint64_t* d_ct, void* stream) {
  int rc = need_keys(ctx);
  if (rc) return rc;
  if (count < 0 || (count > 0 && (!d_msg || !d_ct))) return fail(ctx, FHE_E_ARG, "bad encrypt arguments");
  if (count == 0) return FHE_OK;
  const fhe_params& p = ctx->p;
  ChaKey K = key_from_seed(seed);
  hipLaunchKernelGGL(k_encrypt, dim3((unsigned)count), dim3(256), 0, (hipStream_t)stream, K, p.k * p.N, p.msg_bits,
                     p.glwe_noise_bits, ctx->s_big, d_msg, id0, d_ct);
  HIPCHK(ctx, hipGetLastError());
  return FHE_OK;
}

static int seeded_args(fhe_ctx* ctx, int64_t B, int32_t D, const void* a, const void* b, const void* c) {
  if (B < 0 || D <= 0 || (B > 0 && (!a || !b || !c))) return fail(ctx, FHE_E_ARG, "bad seeded-corpus arguments");
  if (B * (int64_t)D > 0x7fffffffLL) return fail(ctx, FHE_E_ARG, "seeded corpus batch too large (B*D >= 2^31)");
  return FHE_OK;
}

int fhe_encrypt_seeded_batch(fhe_ctx* ctx, const int64_t* d_msg, int64_t B, int32_t D, const uint32_t h_mask_key[8],
                             const uint32_t h_noise_key[8], const uint64_t* d_id0, uint64_t* d_body, void* stream) {
  int rc = need_keys(ctx);
  if (rc) return rc;
  if ((rc = seeded_args(ctx, B, D, d_msg, d_id0, d_body))) return rc;
  if (!h_mask_key || !h_noise_key) return fail(ctx, FHE_E_ARG, "seeded encryption needs both keys");
  if (B == 0) return FHE_OK;
  const fhe_params& p = ctx->p;
  ChaKey Km, Kn;
  for (int i = 0; i < 8; ++i) Km.w[i] = h_mask_key[i], Kn.w[i] = h_noise_key[i];
  hipLaunchKernelGGL(k_encrypt_seeded, dim3((unsigned)(B * D)), dim3(256), 0, (hipStream_t)stream, Km, Kn, p.k * p.N,
                     p.msg_bits, p.glwe_noise_bits, ctx->s_big, d_msg, d_id0, (int)D, d_body);
  HIPCHK(ctx, hipGetLastError());
  return FHE_OK;
}

int fhe_expand_seeded_batch(fhe_ctx* ctx, const uint64_t* d_body, const uint64_t* d_id0, int64_t B, int32_t D,
                            const uint32_t h_mask_key[8], uint64_t* d_ct, void* stream) {
  int rc = need_device(ctx);
  if (rc) return rc;
  if ((rc = seeded_args(ctx, B, D, d_body, d_id0, d_ct))) return rc;
  if (!h_mask_key) return fail(ctx, FHE_E_ARG, "missing mask key");
  if (B == 0) return FHE_OK;
  const fhe_params& p = ctx->p;
  ChaKey Km;
  for (int i = 0; i < 8; ++i) Km.w[i] = h_mask_key[i];
  hipLaunchKernelGGL(k_expand_seeded, dim3((unsigned)(B * D)), dim3(256), 0, (hipStream_t)stream, Km, p.k * p.N,
                     d_body, d_id0, (int)D, d_ct);
  HIPCHK(ctx, hipGetLastError());
  return FHE_OK;
}

int fhe_linear_seeded_batch(fhe_ctx* ctx, const uint64_t* d_body, const uint64_t* d_id0, int64_t B, int32_t D,
                            const uint32_t h_mask_key[8], const int64_t* d_w, int64_t cst, uint64_t* d_out,
                            void* stream) {
  int rc = need_device(ctx);
  if (rc) return rc;
  if ((rc = seeded_args(ctx, B, D, d_body, d_id0, d_out))) return rc;
  if (!h_mask_key || (B > 0 && !d_w)) return fail(ctx, FHE_E_ARG, "missing mask key or weights");
  if (B == 0) return FHE_OK;
  const fhe_params& p = ctx->p;
  ChaKey Km;
  for (int i = 0; i < 8; ++i) Km.w[i] = h_mask_key[i];
  hipLaunchKernelGGL(k_linear_seeded, dim3((unsigned)B), dim3(256), 0, (hipStream_t)stream, Km, p.k * p.N, d_body,
                     d_id0, (int)D, d_w, (u64)cst << (64 - p.msg_bits), d_out);
  HIPCHK(ctx, hipGetLastError());
  return FHE_OK;
}

static int decrypt_mode(fhe_ctx* ctx, const uint64_t* d_ct, int64_t count, int64_t* d_out, int mode, void* stream) {
  int rc = need_keys(ctx);
  if (rc) return rc;
  if (count < 0 || (count > 0 && (!d_ct || !d_out))) return fail(ctx, FHE_E_ARG, "bad decrypt arguments");
  if (count == 0) return FHE_OK;
  const fhe_params& p = ctx->p;
  hipLaunchKernelGGL(k_decrypt, dim3((unsigned)count), dim3(256), 0, (hipStream_t)stream, p.k * p.N, p.msg_bits,
                     mode, ctx->s_big, d_ct, d_out);
  HIPCHK(ctx, hipGetLastError());
  return FHE_OK;
}
int fhe_decrypt_batch(fhe_ctx* ctx, const uint64_t* d_ct, int64_t count, int64_t* d_out, void* stream) {
  return decrypt_mode(ctx, d_ct, count, d_out, 0, stream);
}
int fhe_decrypt_bits_batch(fhe_ctx* ctx, const uint64_t* d_ct, int64_t count, int64_t* d_out, void* stream) {
  return decrypt_mode(ctx, d_ct, count, d_out, 1, stream);
}
int fhe_phase_batch(fhe_ctx* ctx, const uint64_t* d_ct, int64_t count, uint64_t* d_out, void* stream) {
  return decrypt_mode(ctx, d_ct, count, (int64_t*)d_out, 2, stream);
}

int fhe_linear_batch(fhe_ctx* ctx, const uint64_t* d_ct, int64_t B, int32_t D, const int64_t* d_w, int64_t cst,
                     uint64_t* d_out, void* stream) {
  int rc = need_device(ctx);
  if (rc) return rc;
  if (B < 0 || D <= 0 || (B > 0 && (!d_ct || !d_w || !d_out))) return fail(ctx, FHE_E_ARG, "bad linear arguments");
  if (B == 0) return FHE_OK;
  if (B > 65535) return fail(ctx, FHE_E_ARG, "linear batch > 65535: split the call");
  const fhe_params& p = ctx->p;
  const int W = p.k * p.N + 1;
  hipLaunchKernelGGL(k_linear, dim3((W + 255) / 256, (unsigned)B), dim3(256), 0, (hipStream_t)stream, d_ct, D, W, d_w,
                     ((u64)cst) << (64 - p.msg_bits), d_out);
  HIPCHK(ctx, hipGetLastError());
  return FHE_OK;
}

static void prof_begin(fhe_ctx* ctx, ProfAcc& a, hipStream_t st, hipEvent_t* e1) {
  *e1 = nullptr;
  if (!ctx->prof) return;
  hipEvent_t e0;
  hipEventCreate(&e0);
  hipEventCreate(e1);
  hipEventRecord(e0, st);
  a.ev.push_back({e0, *e1});
}
static void prof_end(fhe_ctx* ctx, ProfAcc& a, hipStream_t st, hipEvent_t e1, int64_t items) {
  if (!ctx->prof || !e1) return;
  hipEventRecord(e1, st);
  a.launches += 1;
  a.items += items;
}

int fhe_keyswitch_batch(fhe_ctx* ctx, const uint64_t* d_big, int64_t count, int32_t shift, uint64_t add_body,
                        uint64_t* d_small, void* stream) {
  int rc = need_keys(ctx);
  if (rc) return rc;
  if (count < 0 || shift < 0 || shift > 63 || (count > 0 && (!d_big || !d_small)))
    return fail(ctx, FHE_E_ARG, "bad keyswitch arguments");
  if (count == 0) return FHE_OK;
  const fhe_params& p = ctx->p;
  hipStream_t st = (hipStream_t)stream;
  const int64_t tiles = (count + KS_TC - 1) / KS_TC;
  if (tiles > 65535) return fail(ctx, FHE_E_ARG, "keyswitch batch too large: split the call");
  if (ctx->ks_variant == 2) {
    const int K = p.k * p.N * p.ks_level, KB = K / 64, n1 = p.n + 1, NB = (n1 + KSM_NB_COLS - 1) / KSM_NB_COLS;
    const int64_t ncb = (count + 15) / 16;
    const size_t dbytes = (size_t)ncb * 16 * K, need = dbytes + 8 * (size_t)count;
    if (need > ctx->ks_ws_bytes) {
      if (ctx->ks_ws) {
        HIPCHK(ctx, hipDeviceSynchronize());
        HIPCHK(ctx, hipFree(ctx->ks_ws));
        ctx->ks_ws = nullptr;
      }
      HIPCHK(ctx, hipMalloc(&ctx->ks_ws, need));
      ctx->ks_ws_bytes = need;
    }
    if (ncb > 65535) return fail(ctx, FHE_E_ARG, "keyswitch batch too large: split the call");
    uint32_t* D = (uint32_t*)ctx->ks_ws;
    u64* body = (u64*)((char*)ctx->ks_ws + dbytes);
    hipEvent_t e1;
    prof_begin(ctx, ctx->prof_ks, st, &e1);
    hipLaunchKernelGGL(k_ks_digits, dim3((unsigned)KB, (unsigned)ncb), dim3(256), 0, st, d_big, count, p.k * p.N,
                       p.ks_base_log, shift, add_body, KB, D, body);
    hipLaunchKernelGGL(k_keyswitch_mfma, dim3((unsigned)((count + 63) / 64), (unsigned)NB), dim3(256), 0, st,
                       (const v4i*)D, (const v4i*)ctx->ksk8, body, count, n1, NB, KB, d_small);
    prof_end(ctx, ctx->prof_ks, st, e1, count);
    HIPCHK(ctx, hipGetLastError());
    return FHE_OK;
  }
  HIPCHK(ctx, hipMemsetAsync(d_small, 0, 8 * (size_t)count * (p.n + 1), st));
  hipEvent_t e1;
  prof_begin(ctx, ctx->prof_ks, st, &e1);
  hipLaunchKernelGGL(k_keyswitch, dim3((p.n + 1 + 255) / 256, (unsigned)tiles, KS_SPLIT), dim3(256), 0, st, d_big,
                     count, p.k * p.N, p.n, p.ks_level, p.ks_base_log, shift, add_body, ctx->ksk, ctx->ksk_colsum,
                     d_small);
  prof_end(ctx, ctx->prof_ks, st, e1, count);
  HIPCHK(ctx, hipGetLastError());
  return FHE_OK;
}

static int launch_br(fhe_ctx* ctx, const uint64_t* d_small, int64_t count, BrTv tv, int mode, uint64_t* out,
                     uint64_t* ct_v, uint64_t* refreshed, uint64_t* sign, hipStream_t st) {
  const fhe_params& p = ctx->p;
  hipEvent_t e1;
  prof_begin(ctx, ctx->prof_br, st, &e1);
  const dim3 g((unsigned)count), b(64);
#define BR(LOGM, K)                                                                                           \
  hipLaunchKernelGGL((k_blind_rotate<LOGM, K>), g, b, 0, st, d_small, p.n, p.pbs_level, p.pbs_base_log,      \
                     ctx->bsk_fft, ctx->tw, ctx->twist, tv, mode, out, ct_v, refreshed, sign)
#define BRV(V, K, W)                                                                                          \
  hipLaunchKernelGGL((k_blind_rotate_mw<V, K, W>), g, dim3(V::NT), 0, st, d_small, p.n, p.pbs_level,          \
                     p.pbs_base_log, ctx->bsk_fft, ctx->tw, ctx->twist, tv, mode, out, ct_v, refreshed, sign)
#define BR2(K) do { if (ctx->br_variant == 3) BRV(V3, K, 4); else BRV(V2, K, 2); } while (0)
#define BR4G(L, A32, D, GG)                                                                                   \
  if (ctx->v4_fl && GG > 1) BR4F(L, A32, D, GG, true); else BR4F(L, A32, D, GG, false)
#define BR4F(L, A32, D, GG, FLAGS)                                                                             \
  hipLaunchKernelGGL((k_blind_rotate_v4<L, A32, D, GG, FLAGS>), dim3((unsigned)((count + GG - 1) / GG)),       \
                     dim3(v4::nthreads(GG)), 0, st, d_small, count, p.n, p.pbs_base_log, ctx->bsk_fft, ctx->tw4, tv, \
                     mode, out, ct_v, refreshed, sign)
// G = 4 needs 3 waves per SIMD (<= 168 VGPRs): only the 32-bit-accumulator
// kernels; the u64 ones (208 VGPRs, 2 waves per SIMD) run 2 per workgroup
// (at 4 per workgroup they spill: P=21, 22.2 vs 20.9 ms per 1024 PBS).
#define BR4(L, A32)                                  \
  do {                                               \
    if (ctx->v4_g == 1) BR4G(L, A32, 0, 1);          \
    else if (ctx->v4_g == 2 || !A32) BR4G(L, A32, 0, 2); \
    else BR4G(L, A32, 0, 4);                         \
  } while (0)
#define BR4D(D)                                      \
  do {                                               \
    if (ctx->v4_g == 1) BR4G(2, true, D, 1);         \
    else if (ctx->v4_g == 2) BR4G(2, true, D, 2);    \
    else BR4G(2, true, D, 4);                        \
  } while (0)
  if (p.N == 1024 && p.k == 2 && ctx->br_variant == 4 && ctx->v4_dbg && p.pbs_level == 2 &&
      p.pbs_level * p.pbs_base_log <= 31) {
    switch (ctx->v4_dbg) {
      case 1: BR4D(1); break;
      case 2: BR4D(2); break;
      case 4: BR4D(4); break;
      case 8: BR4D(8); break;
      case 16: BR4D(16); break;
      case 32: BR4D(32); break;
      case 6: BR4D(6); break;
      case 128: BR4D(128); break;
      default: BR4D(63); break;
    }
  } else if (p.N == 1024 && p.k == 2 && ctx->br_variant == 4) {
    const bool a32 = p.pbs_level * p.pbs_base_log <= 31;
    switch (p.pbs_level) {
      case 1: if (a32) BR4(1, true); else BR4(1, false); break;
      case 2: if (a32) BR4(2, true); else BR4(2, false); break;
      case 3: BR4(3, false); break;
      default: return fail(ctx, FHE_E_ARG, "v4 blind rotation: pbs_level > 3");
    }
  } else if (p.N == 256 && p.k == 1) BR(7, 1);
  else if (p.N == 256 && p.k == 2) BR(7, 2);
  else if (p.N == 512 && p.k == 1) BR(8, 1);
  else if (p.N == 512 && p.k == 2) BR(8, 2);
  else if (p.N == 1024 && p.k == 1) BR2(1);
  else if (p.N == 1024 && p.k == 2) BR2(2);
  else if (p.N == 2048 && p.k == 1) BR(10, 1);
  else return fail(ctx, FHE_E_ARG, "unsupported (N, k)");
#undef BR
#undef BR2
#undef BR4
#undef BR4D
#undef BR4G
#undef BR4F
#undef BRV
  prof_end(ctx, ctx->prof_br, st, e1, count);
  HIPCHK(ctx, hipGetLastError());
  return FHE_OK;
}

int fhe_pbs_batch(fhe_ctx* ctx, const uint64_t* d_small, int64_t count, uint64_t tv, uint64_t* d_out, void* stream) {
  int rc = need_keys(ctx);
  if (rc) return rc;
  if (count < 0 || (count > 0 && (!d_small || !d_out))) return fail(ctx, FHE_E_ARG, "bad pbs arguments");
  if (count == 0) return FHE_OK;
  return launch_br(ctx, d_small, count, BrTv{tv, 0, 0}, 0, d_out, nullptr, nullptr, nullptr, (hipStream_t)stream);
}

static int log2i(int x) {
  int l = 0;
  while ((1 << l) < x) ++l;
  return l;
}

int fhe_pbs_lut_batch(fhe_ctx* ctx, const uint64_t* d_small, int64_t count, uint64_t base, uint64_t step,
                      int32_t log_slots, uint64_t* d_out, void* stream) {
  int rc = need_keys(ctx);
  if (rc) return rc;
  const int logN = log2i(ctx->p.N);
  if (count < 0 || (count > 0 && (!d_small || !d_out)) || log_slots < 0 || log_slots > logN)
    return fail(ctx, FHE_E_ARG, "bad pbs-lut arguments");
  if (count == 0) return FHE_OK;
  return launch_br(ctx, d_small, count, BrTv{base, step, logN - log_slots}, 0, d_out, nullptr, nullptr, nullptr,
                   (hipStream_t)stream);
}

static int ensure_ws(fhe_ctx* ctx, size_t bytes) {
  if (bytes <= ctx->ws_bytes) return FHE_OK;
  if (ctx->ws) {
    HIPCHK(ctx, hipDeviceSynchronize());
    HIPCHK(ctx, hipFree(ctx->ws));
    ctx->ws = nullptr;
    ctx->ws_bytes = 0;
  }
  HIPCHK(ctx, hipMalloc(&ctx->ws, bytes));
  ctx->ws_bytes = bytes;
  return FHE_OK;
}

// bit extraction driver; `small` is caller-provided scratch (count x (n+1))
static int bit_extract(fhe_ctx* ctx, uint64_t* d_ct_v, int64_t count, uint64_t* d_ref, uint64_t* d_sign,
                       uint64_t* small, hipStream_t st) {
  const fhe_params& p = ctx->p;
  const int P = p.msg_bits;
  HIPCHK(ctx, hipMemsetAsync(d_ref, 0, 8 * (size_t)count * fhe_big_lwe_words(&p), st));
  for (int i = 0; i < P; ++i) {
    int rc = fhe_keyswitch_batch(ctx, d_ct_v, count, P - 1 - i, 1ull << 62, small, st);
    if (rc) return rc;
    rc = launch_br(ctx, small, count, BrTv{1ull << (63 - P + i), 0, 0}, 1, nullptr, d_ct_v, d_ref,
                   (i == P - 1) ? d_sign : nullptr, st);
    if (rc) return rc;
  }
  return FHE_OK;
}

// Sign of the msg_bits-bit value v in d_ct_v (consumed) with d-bit digits
// (DESIGN.md §3.4): the low m = P - d bits are cleared LSB-first, each full
// digit [b, b+c) by two bootstraps (its top bit by a sign bootstrap; then,
// with a zero padding bit, its c-1 low bits by a 2^(c-1)-slot staircase LUT),
// a leftover of 1-2 bits by single-bit rounds; the sign of the top d bits is
// the sign of v.
int fhe_sign_digit_bits(const fhe_params* params) {
  std::string why;
  if (validate(params, why)) return -1;
  return sign_digits(*params);
}

int fhe_sign_pbs_count(const fhe_params* params) {
  std::string why;
  if (validate(params, why)) return -1;
  const int P = params->msg_bits, d = sign_digits(*params);
  if (P < 4) return P;
  const int m = P - d, r = m % d;
  return 2 * (m / d) + (r >= 3 ? 2 : r) + 1;
}

static int sign_extract(fhe_ctx* ctx, uint64_t* d_ct_v, int64_t count, uint64_t* d_sign, uint64_t* small,
                        hipStream_t st) {
  const fhe_params& p = ctx->p;
  const int P = p.msg_bits, logN = log2i(p.N);
  int rc;
  if (P < 4) {
    for (int i = 0; i < P; ++i) {
      if ((rc = fhe_keyswitch_batch(ctx, d_ct_v, count, P - 1 - i, 1ull << 62, small, st))) return rc;
      if ((rc = launch_br(ctx, small, count, BrTv{1ull << (63 - P + i), 0, 0}, 1, nullptr, d_ct_v, nullptr,
                          (i == P - 1) ? d_sign : nullptr, st)))
        return rc;
    }
    return FHE_OK;
  }
  const int d = sign_digits(p), m = P - d;
  // one c-bit digit at bit b: the pair of rounds on v << (P-b-c) centred by 2^(63-c)
  auto digit = [&](int b, int c) -> int {
    int r;
    // digit MSB (bit b+c-1): sign bootstrap, ct_v -= [bit] * 2^(b+c-1) * Delta
    if ((r = fhe_keyswitch_batch(ctx, d_ct_v, count, P - b - c, 1ull << (63 - c), small, st))) return r;
    if ((r = launch_br(ctx, small, count, BrTv{1ull << (62 - P + b + c), 0, 0}, 1, nullptr, d_ct_v, nullptr,
                       nullptr, st)))
      return r;
    // bits [b, b+c-1): top bit is now 0 -> 2^(c-1)-slot staircase, output D' * 2^b * Delta
    if ((r = fhe_keyswitch_batch(ctx, d_ct_v, count, P - b - c, 1ull << (63 - c), small, st))) return r;
    return launch_br(ctx, small, count, BrTv{0, 1ull << (64 - P + b), logN - (c - 1)}, 2, nullptr, d_ct_v,
                     nullptr, nullptr, st);
  };
  int b = 0;
  for (; b + d <= m; b += d)
    if ((rc = digit(b, d))) return rc;
  if (m - b >= 3) {
    if ((rc = digit(b, m - b))) return rc;
    b = m;
  }
  for (; b < m; ++b) {
    if ((rc = fhe_keyswitch_batch(ctx, d_ct_v, count, P - b - 1, 1ull << 62, small, st))) return rc;
    if ((rc = launch_br(ctx, small, count, BrTv{1ull << (63 - P + b), 0, 0}, 1, nullptr, d_ct_v, nullptr, nullptr,
                        st)))
      return rc;
  }
  // sign = MSB of the top digit [P-d, P)
  if ((rc = fhe_keyswitch_batch(ctx, d_ct_v, count, 0, 1ull << (63 - d), small, st))) return rc;
  return launch_br(ctx, small, count, BrTv{1ull << 62, 0, 0}, 1, nullptr, d_ct_v, nullptr, d_sign, st);
}

int fhe_sign_batch(fhe_ctx* ctx, uint64_t* d_ct_v, int64_t count, uint64_t* d_sign, void* stream) {
  int rc = need_keys(ctx);
  if (rc) return rc;
  if (count < 0 || (count > 0 && (!d_ct_v || !d_sign))) return fail(ctx, FHE_E_ARG, "bad sign arguments");
  if (count == 0) return FHE_OK;
  rc = ensure_ws(ctx, 8 * (size_t)count * fhe_small_lwe_words(&ctx->p));
  if (rc) return rc;
  return sign_extract(ctx, d_ct_v, count, d_sign, (uint64_t*)ctx->ws, (hipStream_t)stream);
}

int fhe_bit_extract_batch(fhe_ctx* ctx, uint64_t* d_ct_v, int64_t count, uint64_t* d_refreshed, uint64_t* d_sign,
                          void* stream) {
  int rc = need_keys(ctx);
  if (rc) return rc;
  if (count < 0 || (count > 0 && (!d_ct_v || !d_refreshed || !d_sign)))
    return fail(ctx, FHE_E_ARG, "bad bit-extract arguments");
  if (count == 0) return FHE_OK;
  rc = ensure_ws(ctx, 8 * (size_t)count * fhe_small_lwe_words(&ctx->p));
  if (rc) return rc;
  return bit_extract(ctx, d_ct_v, count, d_refreshed, d_sign, (uint64_t*)ctx->ws, (hipStream_t)stream);
}

int fhe_compare_batch(fhe_ctx* ctx, const int64_t* d_qx, int64_t B, int32_t D, const int64_t* d_w, int64_t cst,
                      int64_t T, uint64_t enc_seed, uint64_t id0, int64_t* d_acc, int64_t* d_below, void* stream) {
  int rc = need_keys(ctx);
  if (rc) return rc;
  if (B < 0 || D <= 0 || (B > 0 && (!d_qx || !d_w || !d_acc || !d_below)))
    return fail(ctx, FHE_E_ARG, "bad compare arguments");
  if (B == 0) return FHE_OK;
  const fhe_params& p = ctx->p;
  hipStream_t st = (hipStream_t)stream;
  const size_t Wb = fhe_big_lwe_words(&p), Ws = fhe_small_lwe_words(&p);
  // workspace: inputs (B*D big) | ct_v (B big) | sign (B big) | small (B) | v (B)
  const size_t bytes = 8 * ((size_t)B * D * Wb + 2 * (size_t)B * Wb + (size_t)B * Ws + (size_t)B);
  rc = ensure_ws(ctx, bytes);
  if (rc) return rc;
  u64* cin = (u64*)ctx->ws;
  u64* ctv = cin + (size_t)B * D * Wb;
  u64* sgn = ctv + (size_t)B * Wb;
  u64* small = sgn + (size_t)B * Wb;
  int64_t* v = (int64_t*)(small + (size_t)B * Ws);
  rc = fhe_encrypt_batch(ctx, d_qx, B * D, enc_seed, id0, cin, stream);
  if (rc) return rc;
  for (int64_t b0 = 0; b0 < B; b0 += 65535) {
    const int64_t nb = std::min<int64_t>(65535, B - b0);
    rc = fhe_linear_batch(ctx, cin + (size_t)b0 * D * Wb, nb, D, d_w, cst - T, ctv + (size_t)b0 * Wb, stream);
    if (rc) return rc;
  }
  // The score comes from the leveled accumulator ciphertext (noise ~2^20,
  // as in the reference's leveled Concrete circuit); the PBS chain then
  // computes the encrypted threshold bit [acc < T] exactly.
  rc = fhe_decrypt_batch(ctx, ctv, B, v, stream);
  if (rc) return rc;
  rc = sign_extract(ctx, ctv, B, sgn, small, st);
  if (rc) return rc;
  rc = fhe_decrypt_bits_batch(ctx, sgn, B, d_below, stream);
  if (rc) return rc;
  hipLaunchKernelGGL(k_add_scalar, dim3((unsigned)((B + 255) / 256)), dim3(256), 0, st, v, B, T, d_acc);
  HIPCHK(ctx, hipGetLastError());
  return FHE_OK;
}

int fhe_compare_seeded_batch(fhe_ctx* ctx, const uint64_t* d_body, const uint64_t* d_id0, int64_t B, int32_t D,
                             const uint32_t h_mask_key[8], const int64_t* d_w, int64_t cst, int64_t T,
                             int64_t* d_acc, int64_t* d_below, void* stream) {
  int rc = need_keys(ctx);
  if (rc) return rc;
  if ((rc = seeded_args(ctx, B, D, d_body, d_id0, d_w))) return rc;
  if (!h_mask_key || (B > 0 && (!d_acc || !d_below))) return fail(ctx, FHE_E_ARG, "bad seeded compare arguments");
  if (B == 0) return FHE_OK;
  const fhe_params& p = ctx->p;
  hipStream_t st = (hipStream_t)stream;
  const size_t Wb = fhe_big_lwe_words(&p), Ws = fhe_small_lwe_words(&p);
  // workspace: ct_v (B big) | sign (B big) | small (B) | v (B)
  rc = ensure_ws(ctx, 8 * (2 * (size_t)B * Wb + (size_t)B * Ws + (size_t)B));
  if (rc) return rc;
  u64* ctv = (u64*)ctx->ws;
  u64* sgn = ctv + (size_t)B * Wb;
  u64* small = sgn + (size_t)B * Wb;
  int64_t* v = (int64_t*)(small + (size_t)B * Ws);
  rc = fhe_linear_seeded_batch(ctx, d_body, d_id0, B, D, h_mask_key, d_w, cst - T, ctv, stream);
  if (rc) return rc;
  rc = fhe_decrypt_batch(ctx, ctv, B, v, stream);
  if (rc) return rc;
  rc = sign_extract(ctx, ctv, B, sgn, small, st);
  if (rc) return rc;
  rc = fhe_decrypt_bits_batch(ctx, sgn, B, d_below, stream);
  if (rc) return rc;
  hipLaunchKernelGGL(k_add_scalar, dim3((unsigned)((B + 255) / 256)), dim3(256), 0, st, v, B, T, d_acc);
  HIPCHK(ctx, hipGetLastError());
  return FHE_OK;
}

void fhe_key_from_seed(uint64_t seed, uint32_t h_key_out[8]) {
  const ChaKey K = key_from_seed(seed);
  for (int i = 0; i < 8; ++i) h_key_out[i] = K.w[i];
}

int fhe_quantize_pairs(fhe_ctx* ctx, const void* d_query, int32_t query_is_f64, const void* d_docs,
                       int32_t docs_is_f64, int64_t B, int32_t D, double scale, int64_t zero_point, int64_t qmin,
                       int64_t qmax, int64_t* d_qx, void* stream) {
  int rc = need_device(ctx);
  if (rc) return rc;
  if (B < 0 || D <= 0 || (B > 0 && (!d_docs || !d_qx)) || !(scale > 0) || qmin > qmax)
    return fail(ctx, FHE_E_ARG, "bad quantize arguments");
  if (B == 0) return FHE_OK;
  const int64_t total = B * D;
  const dim3 g((unsigned)((total + 255) / 256)), b(256);
  hipStream_t st = (hipStream_t)stream;
  const double z = (double)zero_point, lo = (double)qmin, hi = (double)qmax;
#define QLAUNCH(QT, DT) \
  hipLaunchKernelGGL((k_pair_quantize<QT, DT>), g, b, 0, st, (const QT*)d_query, (const DT*)d_docs, B, D, scale, z, lo, hi, d_qx)
  if (query_is_f64 && docs_is_f64) QLAUNCH(double, double);
  else if (query_is_f64) QLAUNCH(double, float);
  else if (docs_is_f64) QLAUNCH(float, double);
  else QLAUNCH(float, float);
#undef QLAUNCH
  HIPCHK(ctx, hipGetLastError());
  return FHE_OK;
}

int fhe_dequantize(fhe_ctx* ctx, const int64_t* d_acc, int64_t B, double out_scale, double* d_score, void* stream) {
  int rc = need_device(ctx);
  if (rc) return rc;
  if (B < 0 || (B > 0 && (!d_acc || !d_score))) return fail(ctx, FHE_E_ARG, "bad dequantize arguments");
  if (B == 0) return FHE_OK;
  hipLaunchKernelGGL(k_dequantize, dim3((unsigned)((B + 255) / 256)), dim3(256), 0, (hipStream_t)stream, d_acc, B,
                     out_scale, d_score);
  HIPCHK(ctx, hipGetLastError());
  return FHE_OK;
}

int fhe_topk(fhe_ctx* ctx, const int64_t* d_acc, const int64_t* d_below, int64_t B, int64_t base_idx, int32_t k,
             int64_t* d_out_acc, int64_t* d_out_idx, void* stream) {
  int rc = need_device(ctx);
  if (rc) return rc;
  if (B < 0 || k < 0 || (k > 0 && (!d_out_acc || !d_out_idx)) || (B > 0 && !d_acc))
    return fail(ctx, FHE_E_ARG, "bad topk arguments");
  if (k == 0) return FHE_OK;
  hipLaunchKernelGGL(k_topk, dim3(1), dim3(1024), 0, (hipStream_t)stream, d_acc, d_below, B, base_idx, k, d_out_acc,
                     d_out_idx);
  HIPCHK(ctx, hipGetLastError());
  return FHE_OK;
}

int fhe_dev_alloc(fhe_ctx* ctx, size_t bytes, void** d_out) {
  int rc = need_device(ctx);
  if (rc) return rc;
  if (!d_out) return fail(ctx, FHE_E_ARG, "null output pointer");
  *d_out = nullptr;
  if (bytes == 0) return FHE_OK;
  if (hipMalloc(d_out, bytes) != hipSuccess) {
    *d_out = nullptr;
    return fail(ctx, FHE_E_NOMEM, "hipMalloc failed");
  }
  return FHE_OK;
}

int fhe_dev_free(fhe_ctx* ctx, void* d_ptr) {
  int rc = need_device(ctx);
  if (rc) return rc;
  if (d_ptr) HIPCHK(ctx, hipFree(d_ptr));
  return FHE_OK;
}

int fhe_memcpy_h2d(fhe_ctx* ctx, void* d_dst, const void* h_src, size_t bytes, void* stream) {
  int rc = need_device(ctx);
  if (rc) return rc;
  if (bytes == 0) return FHE_OK;
  if (!d_dst || !h_src) return fail(ctx, FHE_E_ARG, "null copy pointer");
  HIPCHK(ctx, hipMemcpyAsync(d_dst, h_src, bytes, hipMemcpyHostToDevice, (hipStream_t)stream));
  return FHE_OK;
}

int fhe_memcpy_d2h(fhe_ctx* ctx, void* h_dst, const void* d_src, size_t bytes, void* stream) {
  int rc = need_device(ctx);
  if (rc) return rc;
  if (bytes == 0) return FHE_OK;
  if (!h_dst || !d_src) return fail(ctx, FHE_E_ARG, "null copy pointer");
  HIPCHK(ctx, hipMemcpyAsync(h_dst, d_src, bytes, hipMemcpyDeviceToHost, (hipStream_t)stream));
  HIPCHK(ctx, hipStreamSynchronize((hipStream_t)stream));
  return FHE_OK;
}

int fhe_stream_sync(fhe_ctx* ctx, void* stream) {
  int rc = need_device(ctx);
  if (rc) return rc;
  HIPCHK(ctx, hipStreamSynchronize((hipStream_t)stream));
  return FHE_OK;
}

int fhe_debug_v4_stamps(fhe_ctx* ctx, uint64_t* h_out) {
  int rc = need_device(ctx);
  if (rc) return rc;
  if (!h_out) return fail(ctx, FHE_E_ARG, "null output");
  HIPCHK(ctx, hipDeviceSynchronize());
  HIPCHK(ctx, hipMemcpyFromSymbol(h_out, HIP_SYMBOL(g_v4_stamps), sizeof(unsigned long long) * 64));
  HIPCHK(ctx, hipMemcpyFromSymbol(h_out + 64, HIP_SYMBOL(g_v4_span), sizeof(unsigned long long) * 2048 * 3));
  return FHE_OK;
}

int fhe_profile_enable(fhe_ctx* ctx, int enable) {
  if (!ctx) return fail(nullptr, FHE_E_ARG, "null ctx");
  ctx->prof = enable != 0;
  return FHE_OK;
}

int fhe_profile_read(fhe_ctx* ctx, const char* kernel, double* total_ms, int64_t* launches, int64_t* items) {
  int rc = need_device(ctx);
  if (rc) return rc;
  if (!kernel) return fail(ctx, FHE_E_ARG, "null kernel name");
  ProfAcc* a = nullptr;
  if (!strcmp(kernel, "blind_rotate")) a = &ctx->prof_br;
  else if (!strcmp(kernel, "keyswitch")) a = &ctx->prof_ks;
  else return fail(ctx, FHE_E_ARG, "unknown kernel name");
  double ms = 0;
  for (auto& e : a->ev) {
    HIPCHK(ctx, hipEventSynchronize(e.second));
    float x = 0;
    HIPCHK(ctx, hipEventElapsedTime(&x, e.first, e.second));
    ms += x;
  }
  if (total_ms) *total_ms = ms;
  if (launches) *launches = a->launches;
  if (items) *items = a->items;
  free_ev(*a);
  a->launches = 0;
  a->items = 0;
  return FHE_OK;
}

}  // extern "C"
