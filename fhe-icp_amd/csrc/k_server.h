// Server-side kernels: leveled linear layer, key switch (VALU and i8 MFMA), quantisation, top-k.
// Part of libfheicp (one translation unit: fheicp.hip includes it).
#pragma once

#include "common.h"

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

// The key switch uses every KSK word rounded to a multiple of 2^R (R =
// ks_round_bits): the rounding error (2^R / sqrt(12)) is
// 2^-7 of the KSK's own noise, and the i8 MFMA form then needs 8 - R / 8
// byte planes instead of 8.
__device__ __forceinline__ u64 ks_round(u64 x, int R) {
  return R ? (x + (1ull << (R - 1))) & ~((1ull << R) - 1) : x;
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
                                                   int R, u64* __restrict__ out) {
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
        // zero-mean digits in [-B/2, B/2] (as k_ks_digits), offset by B/2
        const int prec = KL * kbeta;
        u64 v = ((a >> (63 - prec)) + 1) >> 1;
        const u64 B = 1ull << kbeta;
        for (int l = KL; l >= 1; --l) {
          const u64 low = v & (B - 1);
          v >>= kbeta;
          int64_t d = (int64_t)low;
          if (low > half || (low == half && ((a >> (62 - prec - (KL - l))) & 1))) {
            d -= (int64_t)B;
            v += 1;
          }
          dig[ii][l - 1][q] = (uint8_t)(d + (int64_t)half);
        }
      } else {
        for (int l = 0; l < KL; ++l) dig[ii][l][q] = (uint8_t)half;  // digit 0
      }
    }
    __syncthreads();
    if (col <= n) {
      const int cnt = min(KS_IC, iend_all - i0);
      for (int ii = 0; ii < cnt; ++ii) {
        for (int l = 0; l < KL; ++l) {
          const u64 kv = ks_round(ksk[((size_t)(i0 + ii) * KL + l) * (n + 1) + col], R);
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

// colsum[t] = sum over all KSK rows of the rounded KSK[row][t] (mod 2^64)
__global__ void k_ksk_colsum(const u64* __restrict__ ksk, int rows, int n, int R, u64* __restrict__ colsum) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t > n) return;
  u64 s = 0;
  for (int r = 0; r < rows; ++r) s += ks_round(ksk[(size_t)r * (n + 1) + t], R);
  colsum[t] = s;
}

// Test vector of a bootstrap: TV_j = base + (j >> shift) * step for
// j in [0, N) (a staircase; step = 0 gives the constant TV of a sign
// bootstrap), extended negacyclically: coefficient t of X^{-b} TV is
// TV_{(t+b) mod 2N} with a minus sign when (t + b) mod 2N >= N.
// ---- key switch on the i8 matrix cores (v_mfma_i32_16x16x64_i8) ----------
// out[c] = (0, .., 0, b'[c]) - sum_r D[c][r] * KSK[r], r = i * ks_level + l,
// a GEMM [count x K] (digits in [-2^(b-1), 2^(b-1))) x [K x (n+1)] over
// Z_2^64. The rounded key (ks_round) is split into QP = 8 - R / 8 balanced
// radix-256 byte planes, KSK = sum_q s_q 2^(R + 8q) with s_q in [-128, 127],
// each an i8 GEMM with i32 accumulation (|sum| <= K * 2^(b-1) * 128 < 2^31);
// the epilogue recombines sum_q acc_q << (R + 8q) modulo 2^64 (exact:
// DESIGN.md §4.3).
// Fragment layouts (checked by tools/mfma_i8_probe.hip): lane l holds
// A[row l&15][k = 16 (l>>4) + j] and B[k = 16 (l>>4) + j][col l&15] in byte j;
// C/D: row 4 (l>>4) + reg, col l&15.
typedef int v4i __attribute__((ext_vector_type(4)));
constexpr int KSM_NB_COLS = 16;  // columns per block

// key planes: [kb][nb][q][lane][16 B], q < QP. The GEMM's K runs level-major,
// k = l * big + i (a k-block of 64 is 64 consecutive input coefficients of
// one level, for any ks_level); the KSK itself is stored [i][l][n+1].
__global__ void k_ksk_to_i8(const u64* __restrict__ ksk, int K, int big, int levels, int n1, int NB, int R, int QP,
                            int8_t* __restrict__ out) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (int64_t)K * NB * 16) return;
  const int row = (int)(e / (NB * 16)), col = (int)(e % (NB * 16));
  const int l = row / big, i = row - l * big;
  u64 x = col < n1 ? ks_round(ksk[((size_t)i * levels + l) * n1 + col], R) >> R : 0;
  const int kb = row >> 6, g = (row >> 4) & 3, j = row & 15;
  const int nb = col >> 4, lane = (col & 15) + 16 * g;
  for (int q = 0; q < QP; ++q) {
    const int8_t sq = (int8_t)(x & 0xff);
    x = (x - (u64)(int64_t)sq) >> 8;
    out[((((size_t)kb * NB + nb) * QP + q) * 64 + lane) * 16 + j] = sq;
  }
}

// digits in A-fragment order [cb][kb][lane][16 B] with K level-major (as
// k_ksk_to_i8), and b' = (b << shift) + add_body. A thread takes 4
// consecutive coefficients of one ciphertext and writes one packed word (4
// digits, one byte each) per level; grid (big / 64, ceil(count / 16)), 256
// threads: 16 ciphertexts x 64 coefficients. Needs big % 64 == 0,
// levels <= 8 and levels * beta <= 32 (fhe_ctx_create). With zero_n1 > 0 it
// also zeroes the key switch's output rows of its 16 ciphertexts (zero_n1
// words each, a slice of columns per block), for the split-K atomics of
// k_keyswitch_mfma (one launch fewer than a memset).
__global__ void __launch_bounds__(256) k_ks_digits(const u64* __restrict__ in, int64_t count, int big, int beta,
                                                   int levels, int shift, u64 add_body, int KB,
                                                   uint32_t* __restrict__ D, u64* __restrict__ body, int zero_n1,
                                                   u64* __restrict__ zero_out) {
  const int t = threadIdx.x, cl = t >> 4, iq = t & 15;
  const int64_t cb = blockIdx.y, c = cb * 16 + cl;
  const int i0 = blockIdx.x * 64 + iq * 4;
  if (zero_n1 > 0) {
    const int per = (zero_n1 + (int)gridDim.x - 1) / (int)gridDim.x;
    for (int e = t; e < 16 * per; e += 256) {
      const int q = e / per, col = (int)blockIdx.x * per + (e - q * per);
      const int64_t cz = cb * 16 + q;
      if (cz < count && col < zero_n1) zero_out[(size_t)cz * zero_n1 + col] = 0;
    }
  }
  if (c >= count) return;
  const u64* src = in + (size_t)c * (big + 1);
  if (blockIdx.x == 0 && iq == 0) body[c] = (src[big] << shift) + add_body;
  const int prec = levels * beta;
  const uint32_t half = 1u << (beta - 1);
  uint32_t packed[8];
#pragma unroll
  for (int s = 0; s < 8; ++s) packed[s] = 0;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const u64 x = src[i0 + q] << shift;
    uint32_t r = (uint32_t)(((x >> (63 - prec)) + 1) >> 1);
    // coins for the ties: the bits of x just below the rounding bit
    const uint32_t coins = (uint32_t)(x >> (63 - prec - 8));
#pragma unroll
    for (int s = 0; s < 8; ++s) {  // LSB-first: digit s is level levels - 1 - s
      if (s >= levels) break;
      // zero-mean digits in [-B/2, B/2] (oracle decompose_ks): a tie at B/2
      // is -B/2 (with a carry) when bit 62 - prec - s of x is set
      const uint32_t low = __builtin_amdgcn_ubfe(r, s * beta, beta);
      const uint32_t coin = (coins >> (7 - s)) & 1u;
      const int d = (low > half || (low == half && coin)) ? (int)low - (1 << beta) : (int)low;
      r -= (uint32_t)d << (s * beta);
      packed[s] |= (uint32_t)(uint8_t)(int8_t)d << (8 * q);
    }
  }
  const int lane = cl + 16 * ((i0 >> 4) & 3);
  const int kbi = i0 >> 6, kbl = big >> 6;
#pragma unroll
  for (int s = 0; s < 8; ++s) {
    if (s >= levels) break;
    const int kb = (levels - 1 - s) * kbl + kbi;
    D[(((size_t)cb * KB + kb) * 64 + lane) * 4 + ((i0 & 15) >> 2)] = packed[s];
  }
}

// workgroup = 4 waves = 128 ciphertexts x CB * 16 columns x QP byte planes x
// one slice of K: each wave two 16-ciphertext groups, so every key fragment
// read from LDS feeds two MFMAs (one per group: with one, the four waves'
// fragment reads, 1 KB per MFMA, saturate the LDS). The key tile of each
// k-block (CB * QP KB) is shared through LDS; the tiles and the digit
// fragments stream through a register ring 4 k-blocks deep (the loads of
// k-block k + 4 are issued at k-block k; the compiler counts their vmcnt),
// and the tiles pass through 3 LDS buffers of two k-blocks each with one
// barrier per two k-blocks: the next step's tiles are written while the
// slowest wave may still read the previous step's (one barrier per k-block:
// 81.3 vs 76.2 us per 1024 ciphertexts at (3,5), 8 planes). KB % 4 == 0 for
// every supported parameter set (kN / 64 is a multiple of 4).
// The digit fragments are the stream that bounds it: every column group
// re-reads all of D, so a 16-column tile of 3 planes (the rounded key) ran no
// faster than 8 planes (85 vs 80 us, docs/AB_LOG_r06.md); CB = 3 column
// blocks per workgroup read D a third as often, and the K range split over
// S workgroups (slice kslice k-blocks each, partial sums added with 64-bit
// vector atomics into a zeroed output: exact and order-independent modulo
// 2^64) keeps ~2 workgroups per CU at 1024 ciphertexts.
constexpr int KSM_RING = 4, KSM_CTS = 128;  // ciphertexts per workgroup
template <int QP, int CB>
__global__ void __launch_bounds__(256, 2) k_keyswitch_mfma(const v4i* __restrict__ D, const v4i* __restrict__ K8,
                                                        const u64* __restrict__ body, int64_t count, int n1, int NB,
                                                        int KB, int R, int S, int kslice, u64* __restrict__ out) {
#ifndef FHEICP_KS_KP
#define FHEICP_KS_KP 2  // k-blocks per barrier (1: one barrier per k-block, A/B builds)
#endif
  constexpr int KP = FHEICP_KS_KP;
  constexpr int TV = CB * QP * 64;          // v4i per key tile (one k-block, CB column blocks)
  constexpr int TL = (TV + 255) / 256;      // tile words per thread
  __shared__ v4i bt[3][KP][TV];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  // XCD-aware order over the (column group, ciphertext block, K slice) grid:
  // block b runs on XCD b % 8, and each XCD takes a contiguous run of column
  // groups with all their ciphertext blocks and slices, so a column group's
  // key tiles come into one XCD's L2 once for every block (the blocks of one
  // column block dispatched round-robin over the XCDs made each XCD stream
  // the whole key)
  const int nblk = (int)gridDim.x, bid = (int)blockIdx.x, xcd = bid & 7, q8 = nblk >> 3, r8 = nblk & 7;
  const int t = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  const int NG = NB / CB;                   // column groups (NB padded to a multiple of CB)
  const int per = nblk / NG;                // ciphertext blocks x slices per column group
  const int ng = t / per, rest = t - ng * per, ctb = rest / S, sl = rest - ctb * S;
  const int kb_lo = sl * kslice, kb_hi = min(KB, kb_lo + kslice);
  const int64_t ncb = (count + 15) / 16;   // 16-ciphertext groups (digit rows)
  const int64_t cb0 = (int64_t)ctb * (KSM_CTS / 16) + 2 * w;
  // a group past the batch streams group 0's digits and stores nothing
  const v4i* Dv0 = D + (size_t)(cb0 < ncb ? cb0 : 0) * KB * 64 + lane;
  const v4i* Dv1 = D + (size_t)(cb0 + 1 < ncb ? cb0 + 1 : 0) * KB * 64 + lane;
  const v4i* Kv = K8 + (size_t)ng * TV;
  const size_t kstride = (size_t)NB * QP * 64;  // v4i per k-block of the key
  v4i acc[2][CB][QP];
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int c = 0; c < CB; ++c)
#pragma unroll
      for (int q = 0; q < QP; ++q) acc[h][c][q] = (v4i){0, 0, 0, 0};
  v4i rk[KSM_RING][TL], rd[KSM_RING][2];
  auto tile_load = [&](v4i(&r)[TL], int kb) {
#pragma unroll
    for (int e = 0; e < TL; ++e)
      if (e * 256 + tid < TV) r[e] = Kv[kb * kstride + e * 256 + tid];
  };
  auto tile_store = [&](v4i* dst, const v4i(&r)[TL]) {
#pragma unroll
    for (int e = 0; e < TL; ++e)
      if (e * 256 + tid < TV) dst[e * 256 + tid] = r[e];
  };
  // prologue: k-blocks lo..lo+3 in flight, the first step's tiles into LDS
#pragma unroll
  for (int j = 0; j < KSM_RING; ++j) {
    tile_load(rk[j], kb_lo + j);
    rd[j][0] = Dv0[(size_t)(kb_lo + j) * 64];
    rd[j][1] = Dv1[(size_t)(kb_lo + j) * 64];
  }
#pragma unroll
  for (int h = 0; h < KP; ++h) tile_store(bt[0][h], rk[h]);
  // steps of KP k-blocks, one barrier each; the ring slots of a step's
  // k-blocks (in LDS since the previous step) reload k-block k + 4, and the
  // next step's tiles (loaded one or two steps ago) go into its LDS buffer
  for (int kb = kb_lo; kb < kb_hi; kb += KSM_RING) {
#pragma unroll
    for (int j0 = 0; j0 < KSM_RING; j0 += KP) {
      const int k0 = kb + j0, step = (k0 - kb_lo) / KP;
#pragma unroll
      for (int h = 0; h < KP; ++h) tile_load(rk[j0 + h], min(k0 + h + KSM_RING, kb_hi - 1));  // clamped: reloads
      if (k0 + KP < kb_hi) {
#pragma unroll
        for (int h = 0; h < KP; ++h) tile_store(bt[(step + 1) % 3][h], rk[(j0 + KP + h) % KSM_RING]);
      }
      __syncthreads();
#pragma unroll
      for (int h = 0; h < KP; ++h) {
        const v4i a0 = rd[j0 + h][0], a1 = rd[j0 + h][1];
#pragma unroll
        for (int c = 0; c < CB; ++c)
#pragma unroll
          for (int q = 0; q < QP; ++q) {
            const v4i bq = bt[step % 3][h][(c * QP + q) * 64 + lane];
            acc[0][c][q] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a0, bq, acc[0][c][q], 0, 0, 0);
            acc[1][c][q] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a1, bq, acc[1][c][q], 0, 0, 0);
          }
        const int kn = min(k0 + h + KSM_RING, kb_hi - 1);
        rd[j0 + h][0] = Dv0[(size_t)kn * 64];
        rd[j0 + h][1] = Dv1[(size_t)kn * 64];
      }
    }
  }
#pragma unroll
  for (int c = 0; c < CB; ++c) {
    const int col = (ng * CB + c) * KSM_NB_COLS + (lane & 15);
    if (col >= n1) continue;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      if (cb0 + h >= ncb) continue;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t ci = (cb0 + h) * 16 + 4 * (lane >> 4) + r;
        if (ci >= count) continue;
        u64 v = 0;
#pragma unroll
        for (int q = 0; q < QP; ++q) v += (u64)(int64_t)acc[h][c][q][r] << (R + 8 * q);
        const u64 o = (col == n1 - 1 && sl == 0 ? body[ci] : (u64)0) - v;
        if (S == 1)
          out[(size_t)ci * n1 + col] = o;
        else
          atomicAdd((unsigned long long*)&out[(size_t)ci * n1 + col], (unsigned long long)o);
      }
    }
  }
}

// Blind rotation + sample extraction. One 64-lane wavefront (= workgroup)
// per ciphertext; the GLWE accumulator ((K+1) x N u64) lives in LDS, the
// external-product partial sums in registers.
// Test vector and epilogue modes: BrTv / br_emit above.

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


__global__ void k_add_scalar(const int64_t* __restrict__ v, int64_t B, int64_t T, int64_t* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < B) out[i] = v[i] + T;
}

// out = mul * ct + trivial(add) for count LWEs of W words (in place allowed):
// every word times mul mod 2^64, `add` on the body
__global__ void k_lwe_affine(const u64* in, int64_t count, int W, u64 mul, u64 add, u64* out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= count * W) return;
  const u64 x = in[i] * mul;
  out[i] = (i % W == W - 1) ? x + add : x;
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

// PCA transform of the embedding stage (dimension_reduction.py:67-72, sklearn
// PCA.transform without whitening): out[b][d] = sum_k (x[b][k] - mean[k]) *
// comp[d][k], accumulated in f64 (a fixed summation order: deterministic, and
// at least as accurate as the reference's float32 BLAS), stored as float32 as
// the reference stores embeddings (batch_operations.py:175-178). One 256-thread
// workgroup per row; the row (K <= 1024 floats, centred) is staged in LDS and
// each thread owns outputs d = tid, tid + 256, ...; the components (D x K)
// stay L2-resident across rows.
__global__ void __launch_bounds__(256) k_pca_transform(const float* __restrict__ x, int K,
                                                       const float* __restrict__ mean,
                                                       const float* __restrict__ comp, int D,
                                                       float* __restrict__ out) {
  __shared__ double row[1024];
  const int64_t b = blockIdx.x;
  for (int k = threadIdx.x; k < K; k += 256) row[k] = (double)x[(size_t)b * K + k] - (double)mean[k];
  __syncthreads();
  for (int d = threadIdx.x; d < D; d += 256) {
    const float* c = comp + (size_t)d * K;
    double acc = 0.0;
    for (int k = 0; k < K; ++k) acc = __fma_rn(row[k], (double)c[k], acc);
    out[(size_t)b * D + d] = (float)acc;
  }
}
