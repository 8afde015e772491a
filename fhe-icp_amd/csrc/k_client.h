// Key generation, encryption / decryption and the seeded (stored) corpus kernels.
// Part of libfheicp (one translation unit: fheicp.hip includes it).
#pragma once

#include "common.h"

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
                                                    u64* __restrict__ bsk, uint32_t tag_mask, uint32_t tag_noise) {
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
      stream_block(K, tag_mask, sid, (uint32_t)blk, w);
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
    u64 b = body[q] + (u64)tuniform(stream_word(K, tag_noise, (u64)row, (u64)t), noise_bits);
    dst[(size_t)k * N + t] = b;
  }
  __syncthreads();
  if (threadIdx.x == 0 && s_small[i]) dst[(size_t)c_in * N] += 1ull << (64 - lvl * beta);
}

// Messages of the multi-bit bootstrapping key: pair j of the
// small secret (s1, s2) = (s[2j], s[2j+1]) (s2 = 0 past n) gets three GGSWs,
// of the indicators s1(1-s2), (1-s1)s2 and s1 s2 (subsets {1}, {2}, {1,2}).
// k_keygen_bsk then runs with these as its "small secret" (GGSW i = 3j + S).
__global__ void k_mb_msgs(const u64* __restrict__ s_small, int n, u64* __restrict__ msg) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= (n + 1) / 2) return;
  const u64 s1 = s_small[2 * j], s2 = 2 * j + 1 < n ? s_small[2 * j + 1] : 0;
  msg[3 * j] = s1 & (1 - s2);
  msg[3 * j + 1] = (1 - s1) & s2;
  msg[3 * j + 2] = s1 & s2;
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
// ---- packed features: the leveled circuit's inputs as GLWE messages --------
//  The D features of pair b are the first coefficients of
// G = ceil(D / N) GLWE messages M_g = sum_t x[b, gN + t] Delta X^t; GLWE g of
// pair b has stream id id0 + b G + g: mask A_i[t] = word iN + t of
// stream(TAG_ENC_MASK, id), noise E[t] = TUniform(word t of
// stream(TAG_ENC_NOISE, id)), body B = sum_i A_i S_i + M + E mod X^N + 1.
// The leveled dot product multiplies GLWE g by W_g = sum_t w[gN + t] X^-t and
// sample-extracts coefficient 0 (sum_t w_t m_t), an LWE under the flattened
// key (kN): with C_i = A_i W_g the extracted mask is a_{i,0} = C_i[0],
// a_{i,u} = -C_i[N - u], i.e.
//     a_{i,u} = sum_t w_t Ahat_i[t - u],  Ahat[m] = A[m] (m >= 0), -A[m + N] (m < 0),
// and the body coefficient 0 of B W_g is sum_t w_t B[t]. One mask of kN words
// per pair instead of one per feature: 16x fewer ChaCha20 blocks at D = 16.

// acc[r] += sum_{t < Dg} w[t] Ahat[t - u0 - r] for r < 8: Ahat of one component
// (A: N words in LDS), windows of 16 words slid by 8 features at a time (all
// register indices static); features past Dg weigh 0.
__device__ __forceinline__ u64 ahat(const u64* A, int m, int N) { return m >= 0 ? A[m] : (u64)0 - A[m + N]; }
// branch-free Ahat[m] for m in [-N, 2N), 0 from m = N on (features past the
// chunk): one LDS read at m mod N and selects (the branchy form above made
// every read its own divergent block, with its latency exposed)
__device__ __forceinline__ u64 ahat_w(const u64* A, int m, int N) {
  const u64 v = A[m & (N - 1)];
  const u64 r = m < 0 ? (u64)0 - v : v;
  return m < N ? r : 0;
}
__device__ __forceinline__ u64 readlane64(u64 v, int lane) {
  return ((u64)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), lane) << 32) |
         (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, lane);
}
// Weights: lane l of the wave holds w[64 c + l] of the current 64-feature
// block c (one coalesced load per 64 features; whole waves call this, all 64
// lanes active: packed_chunk_mask) and feature j's weight is broadcast by
// v_readlane into scalar registers, so the MAC loop touches no memory but the
// window's LDS reads (a clamped global load per feature instead: 38 us per
// 1024 pairs against 26, docs/AB_LOG_r04.md). The u64 product is the
// compiler's v_mad_u64_u32 + two v_mul_lo_u32 + v_add3_u32: splitting it by
// the halves of the mask word into two v_mad_u64_u32 measured slower (the MAC
// phase 5,740 cycles against 5,010, docs/AB_LOG_r04.md).
__device__ __forceinline__ void packed_mac8(const u64* A, int N, int u0, const int64_t* __restrict__ w, int Dg,
                                            u64 acc[8]) {
  u64 win[16];
#pragma unroll
  for (int q = 0; q < 8; ++q) win[q] = ahat_w(A, q - u0 - 7, N);
  u64 wreg = 0;
  const int lane = threadIdx.x & 63;
  for (int j0 = 0; j0 < Dg; j0 += 8) {
    if ((j0 & 63) == 0) {
      const int jl = j0 + lane;
      wreg = jl < Dg ? (u64)w[jl] : 0;  // 0 past Dg: those features weigh nothing
    }
#pragma unroll
    for (int q = 8; q < 16; ++q) win[q] = ahat_w(A, j0 + q - u0 - 7, N);
#pragma unroll
    for (int jj = 0; jj < 8; ++jj) {
      const u64 wj = readlane64(wreg, (j0 & 63) + jj);
#pragma unroll
      for (int r = 0; r < 8; ++r) acc[r] += wj * win[jj + 7 - r];
    }
#pragma unroll
    for (int q = 0; q < 8; ++q) win[q] = win[q + 8];
  }
}

// Client side: GLWE encryption of the packed features (fhe_encrypt_packed_batch).
// One 256-thread workgroup per GLWE (pair b, chunk g); the body's negacyclic
// products with the binary key run as in k_keygen_bsk. glwe: [B][G][(k+1)N].
__global__ void __launch_bounds__(256) k_encrypt_packed(ChaKey K, int N, int k, int msg_bits, int noise_bits,
                                                        const u64* __restrict__ s_big, const int64_t* __restrict__ x,
                                                        int D, int G, u64 id0, u64* __restrict__ glwe) {
  extern __shared__ u64 shm[];
  u64* A = shm;                                              // kN
  unsigned char* S = reinterpret_cast<unsigned char*>(shm + (size_t)k * N);  // kN
  const int64_t bg = blockIdx.x, b = bg / G;
  const int g = (int)(bg - b * G), Dg = min(D - g * N, N);
  const u64 id = id0 + (u64)bg;
  u64* o = glwe + (size_t)bg * (k + 1) * N;
  for (int blk = threadIdx.x; blk < k * N / 8; blk += 256) {
    u64 m[8];
    stream_block(K, TAG_ENC_MASK, id, (uint32_t)blk, m);
#pragma unroll
    for (int q = 0; q < 8; ++q) A[8 * blk + q] = o[8 * blk + q] = m[q];
  }
  for (int t = threadIdx.x; t < k * N; t += 256) S[t] = (unsigned char)s_big[t];
  __syncthreads();
  const int per = N / 256, t0 = per * threadIdx.x;  // this thread's body coefficients [t0, t0 + per)
  u64 body[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int i = 0; i < k; ++i) {
    const u64* Ai = A + (size_t)i * N;
    for (int v = 0; v < N; ++v) {
      if (!S[i * N + v]) continue;  // uniform across the workgroup
#pragma unroll
      for (int q = 0; q < 8; ++q)
        if (q < per) body[q] += ahat(Ai, t0 + q - v, N);
    }
  }
  u64 e[8];
  stream_block(K, TAG_ENC_NOISE, id, (uint32_t)(t0 >> 3), e);
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    if (q >= per) break;
    const int t = t0 + q;
    const u64 msg = t < Dg ? (u64)x[(size_t)b * D + g * N + t] << (64 - msg_bits) : 0;
    o[(size_t)k * N + t] = body[q] + msg + (u64)tuniform(e[(t & 7)], noise_bits);
  }
}

// The per-pair extraction shared by the two kernels below: thread t owns mask
// words [8t, 8t + 8) of the output LWE (component i = 8t / N), with A of the
// chunk in LDS. Returns nothing; accumulates into acc.
// packed_mac8 broadcasts the weights by v_readlane from every lane of the
// wave, so the condition is per wave: a wave with any owned word runs it on
// all 64 lanes (kN = 256 leaves lanes 32-63 of wave 0 without words); the
// lanes past kN work on a clamped position and their acc is never stored.
__device__ __forceinline__ void packed_chunk_mask(const u64* A, int N, int k, const int64_t* __restrict__ wg, int Dg,
                                                  u64 acc[8]) {
  const int t8 = 8 * threadIdx.x;
  if (8 * (int)(threadIdx.x & ~63u) < k * N) {
    const int tc = min(t8, k * N - 8);
    const int i = tc / N;
    packed_mac8(A + (size_t)i * N, N, tc - i * N, wg, Dg, acc);
  }
}

// k_encrypt_linear's LDS form of a chunk's mask: per component i, Ahat_i over
// m in [-N, N) stored at e = m + N, so the negacyclic sign is in the data
// (E[e] = -A[e] for e < N, A[e - N] from N on) and a window read is a plain
// load; one pad word per 8 (physical e + e / 8), so the lanes' windows,
// 8 words apart, start 9 words apart: 2-way instead of 16-way LDS bank
// conflicts. 2N * 9 / 8 words per component.
__host__ __device__ __forceinline__ constexpr int el_region(int N) { return 2 * N / 8 * 9; }
// mask block blk (words [8 blk, 8 blk + 8) of the chunk's kN mask words) into E
__device__ __forceinline__ void el_store_block(u64* E, int N, int blk, const u64 m[8]) {
  const int i = 8 * blk / N, b = blk - i * (N / 8);
  u64* pos = E + i * el_region(N) + 9 * (N / 8 + b);
  u64* neg = E + i * el_region(N) + 9 * b;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    pos[j] = m[j];
    neg[j] = (u64)0 - m[j];
  }
}
// packed_mac8 on the E form: acc[r] += sum_{t < Dg} w[t] Ahat[t - u0 - r]; the
// window of iteration j0 is E[e0 + q], e0 = N - u0 - 7 + j0 = 8 b0 + 1, read
// fresh (15 words, constant offsets from one per-lane base advancing 9 words
// per iteration); the weights are wave-uniform, loaded into scalar registers
__device__ __forceinline__ void packed_mac8_e(const u64* E, int N, int u0, const int64_t* __restrict__ w, int Dg,
                                              u64 acc[8]) {
  const u64* p = E + 9 * (N / 8 - u0 / 8 - 1);
  for (int j0 = 0; j0 < Dg; j0 += 8, p += 9) {
    u64 win[15];
#pragma unroll
    for (int q = 0; q < 15; ++q) win[q] = p[1 + q + ((1 + q) >> 3)];
#pragma unroll
    for (int jj = 0; jj < 8; ++jj) {
      const u64 wj = j0 + jj < Dg ? (u64)w[j0 + jj] : 0;  // past Dg: those features weigh nothing
#pragma unroll
      for (int r = 0; r < 8; ++r) acc[r] += wj * win[jj + 7 - r];
    }
  }
}

// Server side: the leveled dot product over packed GLWE inputs
// (fhe_linear_packed_batch): out[b] = sum_g Extract_0(GLWE_g W_g) +
// trivial(cst Delta). One workgroup per pair, A of each chunk staged in LDS.
__global__ void __launch_bounds__(256) k_linear_packed(int N, int k, const u64* __restrict__ glwe, int D, int G,
                                                       const int64_t* __restrict__ w, u64 cst_scaled,
                                                       u64* __restrict__ out) {
  extern __shared__ u64 shm[];
  __shared__ u64 red[4];
  const int64_t b = blockIdx.x;
  u64 acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  u64 bpart = 0;
  for (int g = 0; g < G; ++g) {
    const u64* in = glwe + ((size_t)b * G + g) * (k + 1) * N;
    const int Dg = min(D - g * N, N);
    __syncthreads();  // the previous chunk's readers are done
    for (int t = threadIdx.x; t < k * N; t += 256) shm[t] = in[t];
    for (int t = threadIdx.x; t < Dg; t += 256) bpart += (u64)w[g * N + t] * in[(size_t)k * N + t];
    __syncthreads();
    packed_chunk_mask(shm, N, k, w + g * N, Dg, acc);
  }
  const int t8 = 8 * threadIdx.x;
  u64* o = out + (size_t)b * (k * N + 1);
  if (t8 < k * N) {
#pragma unroll
    for (int q = 0; q < 8; ++q) o[t8 + q] = acc[q];
  }
  const u64 bs = block_sum_u64<256>(bpart, red);
  if (threadIdx.x == 0) o[k * N] = bs + cst_scaled;
}

// Fused client encryption + leveled dot product (fhe_encrypt_linear_batch):
// k_encrypt_packed then k_linear_packed without materialising the GLWEs. The
// mask of each chunk is generated into LDS (one ChaCha20 block per thread of
// waves 0-3), the extracted mask accumulated in registers, and the body
// computed from it: Extract_0(B W_g) = <a_g, s> + sum_t w_t (m_t + e_t)
// exactly (mod 2^64), so
//   b = <a, s> + sum_j w_j (x_j Delta + e_j) + cst Delta,
// bit-identical to the two kernels. The features' noise blocks (ceil(Dg / 8)
// of them) follow the mask blocks, each on the four lanes of a quad
// (chacha20_block_quad: 300 instructions instead of a second 976-instruction
// pass of a wave for two blocks at D = 16), spread over the four waves. The key words of the thread's eight mask
// words are loaded at the start, behind the ChaCha20 work.
// Phase stamps (tools/el_stamps.py): a launch of 1024 pairs puts exactly four
// workgroups on every CU and one wave of each on every SIMD; the four run
// 19k to 47k cycles as the SIMDs issue by wave age, so a CU's span is set by
// its total VALU work. That work is priced by tools/valu_probe.hip: the
// half-rate v_alignbit_b32 (a third of ChaCha20) and the u64 MAC's VOP3
// multiplies (bench.py leveled_score.roofline.valu_mix_floor_ms).
constexpr int EL_THREADS = 256;
// A/B builds (FHEICP_AB): per wave of the first 1024 workgroups, {s_memrealtime
// at start, s_memtime at start / after the mask blocks / after the noise blocks
// / after the barrier / after the MAC loop / at the end, s_memrealtime at the
// end, HW_ID, XCC_ID} (tools/el_stamps.py, fhe_debug_el_stamps)
#ifdef FHEICP_AB
__device__ unsigned long long g_el_stamps[1024][4][10];
#define EL_STAMP(k, t)                  \
  do {                                  \
    __builtin_amdgcn_sched_barrier(0);  \
    st_[k] = (t);                       \
    __builtin_amdgcn_sched_barrier(0);  \
  } while (0)
#else
#define EL_STAMP(k, t) \
  do {                 \
  } while (0)
#endif
__global__ void __launch_bounds__(EL_THREADS) k_encrypt_linear(ChaKey K, int N, int k, int msg_bits, int noise_bits,
                                                        const u64* __restrict__ s_big, const int64_t* __restrict__ x,
                                                        int D, int G, const int64_t* __restrict__ w, u64 cst_scaled,
                                                        u64 id0, u64* __restrict__ out) {
  extern __shared__ u64 shm[];
  __shared__ u64 red[EL_THREADS / 64];
  const int64_t b = blockIdx.x;
  [[maybe_unused]] unsigned long long st_[8];
  EL_STAMP(0, __builtin_amdgcn_s_memrealtime());
  EL_STAMP(1, __builtin_amdgcn_s_memtime());
  const int t8 = 8 * threadIdx.x;
  u64 key[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) key[q] = t8 < k * N ? s_big[t8 + q] : 0;
  u64 acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  u64 bpart = 0;
  for (int g = 0; g < G; ++g) {
    const u64 id = id0 + (u64)b * G + g;
    const int Dg = min(D - g * N, N);
    __syncthreads();  // the previous chunk's readers are done
    // the features' noise words, 8 per block, each block on a quad of lanes
    // (chacha20_block_quad): noise block nb on quad nb / 4 of wave nb mod 4;
    // the even lanes of the quad hold the low words of u64 words
    // j = (q + 4 r) / 2, the odd ones the high words
    const int q = (int)(threadIdx.x & 3), wv = (int)(threadIdx.x >> 6), qd = (int)((threadIdx.x & 63) >> 2);
    auto noise_words = [&](int nb, const uint32_t e4[4]) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const uint32_t hi = quad_mov<QP_XOR1>(e4[r]);
        const int t = 8 * nb + ((q + 4 * r) >> 1);
        if ((q & 1) == 0 && t < Dg) {
          const u64 e = (u64)e4[r] | ((u64)hi << 32);
          bpart += (u64)w[g * N + t] * (((u64)x[(size_t)b * D + g * N + t] << (64 - msg_bits)) + (u64)tuniform(e, noise_bits));
        }
      }
    };
    const int nblk = k * N / 8;
    int blk = threadIdx.x, nb = 4 * qd + wv;
    // a wave whose first quad has a noise block and whose lanes all have a
    // mask block computes the quad blocks of its first noise pass inside its
    // mask blocks (chacha20_block_with_quad): at D = 16 the two noise blocks
    // ran as their own latency-bound pass on waves 0-1 (9.5k of a wave's 33k
    // cycles) while the other waves waited at the barrier (docs/AB_LOG_r06.md)
    if ((wv + 1) * 64 <= nblk && 8 * wv < Dg) {
      uint32_t o[16], e4[4];
      chacha20_block_with_quad(K, (uint32_t)blk, TAG_ENC_MASK, id, o, (uint32_t)nb, TAG_ENC_NOISE, id, q, e4);
      u64 m[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) m[j] = (u64)o[2 * j] | ((u64)o[2 * j + 1] << 32);
      el_store_block(shm, N, blk, m);
      if (8 * nb < Dg) noise_words(nb, e4);
      blk += 256;
      nb += 64;
    }
    for (; blk < nblk; blk += 256) {
      u64 m[8];
      stream_block(K, TAG_ENC_MASK, id, (uint32_t)blk, m);
      el_store_block(shm, N, blk, m);
    }
    EL_STAMP(2, __builtin_amdgcn_s_memtime());
    for (; 8 * nb < Dg; nb += 64) {
      uint32_t e4[4];
      chacha20_block_quad(K, (uint32_t)nb, TAG_ENC_NOISE, id, q, e4);
      noise_words(nb, e4);
    }
    EL_STAMP(3, __builtin_amdgcn_s_memtime());
    __syncthreads();
    EL_STAMP(4, __builtin_amdgcn_s_memtime());
    if (t8 < k * N) {
      const int i = t8 / N;
      packed_mac8_e(shm + i * el_region(N), N, t8 - i * N, w + g * N, Dg, acc);
    }
    EL_STAMP(5, __builtin_amdgcn_s_memtime());
  }
  u64* o = out + (size_t)b * (k * N + 1);
  u64 sdot = 0;
  if (t8 < k * N) {
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      o[t8 + q] = acc[q];
      sdot += acc[q] & (0 - key[q]);
    }
  }
  const u64 tot = block_sum_u64<EL_THREADS>(sdot + bpart, red);
  if (threadIdx.x == 0) o[k * N] = tot + cst_scaled;
#ifdef FHEICP_AB
  EL_STAMP(6, __builtin_amdgcn_s_memtime());
  EL_STAMP(7, __builtin_amdgcn_s_memrealtime());
  if ((threadIdx.x & 63) < 10 && b < 1024) {
    unsigned long long v = 0;
#pragma unroll
    for (int q = 0; q < 8; ++q) v = (int)(threadIdx.x & 63) == q ? st_[q] : v;
    // HW_ID (wave, SIMD, CU, SE fields) and XCC_ID
    v = (threadIdx.x & 63) == 8 ? (unsigned long long)__builtin_amdgcn_s_getreg(4 | (31 << 11)) : v;
    v = (threadIdx.x & 63) == 9 ? (unsigned long long)__builtin_amdgcn_s_getreg(20 | (31 << 11)) : v;
    g_el_stamps[b][threadIdx.x >> 6][threadIdx.x & 63] = v;
  }
#endif
}

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

// The rotation exponent a blind rotation will apply to small LWE c, i.e. its
// phase modulus-switched to 2N exactly as the rotation rounds it (measurement
// only: it reads the small secret key, like k_decrypt): phi = b~ - sum a~_S
// mod 2N, the test-vector index coefficient 0 ends up reading. group 1
// (classic): a~_i = round(a_i 2N / 2^64) for every set key bit (oracle pbs1g);
// group 2 (multi-bit pairs): the exponent of the pair's active subset, a~_1,
// a~_2, or the switch of the exact sum a_1 + a_2 when both bits are set
// (oracle pbs1_mb, k_blind_rotate_mb's atab). One wave per ciphertext.
__global__ void __launch_bounds__(64) k_ms_phase(int n, int log2n2, int group, const u64* __restrict__ s,
                                                 const u64* __restrict__ small, int64_t count,
                                                 uint32_t* __restrict__ out) {
  const int64_t c = blockIdx.x;
  if (c >= count) return;
  const u64* x = small + (size_t)c * (n + 1);
  uint32_t part = 0;
  if (group == 2) {
    for (int j = threadIdx.x; 2 * j < n; j += 64) {
      const bool s1 = s[2 * j] != 0, s2 = 2 * j + 1 < n && s[2 * j + 1] != 0;
      if (s1 && s2) part += modswitch_2n(x[2 * j] + x[2 * j + 1], log2n2);
      else if (s1) part += modswitch_2n(x[2 * j], log2n2);
      else if (s2) part += modswitch_2n(x[2 * j + 1], log2n2);
    }
  } else {
    for (int i = threadIdx.x; i < n; i += 64)
      if (s[i]) part += modswitch_2n(x[i], log2n2);
  }
  for (int off = 32; off > 0; off >>= 1) part += __shfl_down(part, off, 64);
  if (threadIdx.x == 0) out[c] = (modswitch_2n(x[n], log2n2) - part) & ((1u << log2n2) - 1);
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
