// The embedding stage's encoder on gfx950 (include/fhe_bert.h, SURVEY.md
// §8 f4): BertEmbedder.get_embeddings_batch
// (bert_embeddings.py:103-158) from token ids to the pooled float32
// embedding. Second translation unit of libfheicp.so.
//
// Layout in HBM: the residual stream h in fp32 [M][H] (M = B * S tokens) with
// a bf16 copy hb feeding the GEMMs; weights bf16 in torch's [out][in] layout
// (so both GEMM operands are K-contiguous: A = activations [M][K], B^T =
// W [N][K]); Q, K and V of a layer come out of ONE GEMM against the stacked
// [3H][H] weight. Per layer: QKV GEMM -> fused attention -> output GEMM with
// the residual add fused -> LayerNorm -> FFN GEMM with GELU fused -> FFN
// output GEMM with the residual fused -> LayerNorm.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cmath>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/fhe_bert.h"
#include "../../include/fhe_icp.h"

namespace fbert {
typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

// ---- GEMM: out[M][N] = A[M][K] . W[N][K]^T + bias (+ epilogue) ------------
// Shared pieces of the GEMM below: the 256-row block tile and K step, the
// epilogues, and the erf of BERT's GELU.
constexpr int BM = 256, BK = 64;
enum { EPI_BF16 = 0, EPI_GELU_BF16 = 1, EPI_RESID_F32 = 2 };

// erf by Abramowitz & Stegun 7.1.26 (|error| <= 1.5e-7, far below the bf16
// rounding of the GELU output): one reciprocal, one exp and five FMAs against
// the library erff's ~3x the instructions, which made the FFN GEMM's epilogue
// as long as its main loop. The reciprocal is the hardware v_rcp_f32 (1 ulp):
// __frcp_rn's correctly rounded form is a ten-instruction division sequence
// (div_scale x2, div_fmas, div_fixup, FMAs) per element.
__device__ __forceinline__ float erf_fast(float x) {
  const float ax = fabsf(x);
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, ax, 1.0f));
  const float p = fmaf(fmaf(fmaf(fmaf(1.061405429f, t, -1.453152027f), t, 1.421413741f), t, -0.284496736f), t,
                       0.254829592f) * t;
  return copysignf(1.0f - p * __expf(-ax * ax), x);
}

// ---- GEMM, LDS-DMA form: 256 x 128 tiles, three stages -------------------
// The operands go global -> LDS directly (global_load_lds_dwordx4, no staging
// registers) into three stage buffers, so the loads of K step kt + 2 are in
// flight while step kt computes. An LDS-DMA instruction writes 64 lanes x 16
// bytes contiguously, so the rows are unpadded (128 B) and the bank spread
// comes from an XOR swizzle applied on the global side: LDS chunk c' of row r
// holds the row's chunk c' ^ (r & 7). Waits are counted by hand (vmcnt(6):
// one stage of six loads per wave left in flight) before a raw s_barrier.
constexpr int G3_BN = 128, G3_STAGE = (BM + G3_BN) * BK;  // bf16 elements per stage (48 KB)
constexpr int G3_LDS = 3 * G3_STAGE * (int)sizeof(bf16);   // 147456 B
typedef __attribute__((address_space(3))) void lds_void;

template <int EPI>
__global__ void __launch_bounds__(512) k_gemm3(const bf16* __restrict__ A, const bf16* __restrict__ W,
                                               const float* __restrict__ bias, const float* __restrict__ resid,
                                               void* __restrict__ out, int M, int N, int K, int tiles_n, int nblk) {
  constexpr int BN = G3_BN, WN = 2, FM = 4;  // 8 waves in 4 x 2, each 64 x 64
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16* st = reinterpret_cast<bf16*>(smem);
  const int tid = threadIdx.x, l = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = w / WN, wn = w - wm * WN;
  const int b = blockIdx.x, xcd = b & 7, q = nblk >> 3, r = nblk & 7;
  const int t = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (b >> 3);
  const int m0 = (t / tiles_n) * BM, n0 = (t - (t / tiles_n) * tiles_n) * BN;
  const int KT = K / BK;
  auto issue = [&](int kt, int s) {
    bf16* la = st + s * G3_STAGE;
    bf16* lb = la + BM * BK;
#pragma unroll
    for (int i = 0; i < 4; ++i) {  // A: 32 pieces of 8 rows x 128 B, four per wave
      const int pc = 4 * w + i, row = 8 * pc + (l >> 3), c = (l & 7) ^ (row & 7);
      const int gm = min(m0 + row, M - 1);  // rows past M: loaded, never stored
      __builtin_amdgcn_global_load_lds(A + (size_t)gm * K + kt * BK + 8 * c, (lds_void*)(la + pc * 8 * BK), 16, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {  // B: 16 pieces, two per wave
      const int pc = 2 * w + i, row = 8 * pc + (l >> 3), c = (l & 7) ^ (row & 7);
      const int gn = min(n0 + row, N - 1);
      __builtin_amdgcn_global_load_lds(W + (size_t)gn * K + kt * BK + 8 * c, (lds_void*)(lb + pc * 8 * BK), 16, 0, 0);
    }
  };
  f32x4 acc[FM][4];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  issue(0, 0);
  if (KT > 1) issue(1, 1);
  for (int kt = 0; kt < KT; ++kt) {
    if (kt + 1 < KT)
      asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    else
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (kt + 2 < KT) issue(kt + 2, (kt + 2) % 3);
    const bf16* la = st + (kt % 3) * G3_STAGE;
    const bf16* lb = la + BM * BK;
#pragma unroll
    for (int ks = 0; ks < BK / 32; ++ks) {
      const int c = 4 * ks + (l >> 4);
      bf16x8 bv[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int n = wn * 64 + 16 * j + (l & 15);
        bv[j] = *reinterpret_cast<const bf16x8*>(lb + n * BK + 8 * (c ^ (n & 7)));
      }
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        const int m = wm * (FM * 16) + 16 * i + (l & 15);
        const bf16x8 av = *reinterpret_cast<const bf16x8*>(la + m * BK + 8 * (c ^ (m & 7)));
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bv[j], av, acc[i][j], 0, 0, 0);
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this step's reads retire before the next barrier
  }
#ifdef FBERT_AB_NOEPI
  float sum = 0.f;
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) sum += acc[i][j][0] + acc[i][j][1] + acc[i][j][2] + acc[i][j][3];
  if (sum == 12345.678f) reinterpret_cast<float*>(out)[tid] = sum;
  return;
#endif
  // Epilogue through LDS: each wave writes its 64 x 64 tile (bias added, GELU
  // applied) row-major into a private region, then stores whole 128-byte row
  // pieces, 16 bytes per lane (written straight from the fragments, a lane's
  // four columns made 32-byte row pieces and the FFN GEMM's epilogue ran at
  // 1.4 TB/s). Rows are padded by 16 bytes against bank conflicts.
  __syncthreads();  // every wave is done with the stage buffers
  const int colw = n0 + wn * 64, roww = m0 + wm * 64;
  if (colw >= N) return;  // N % 64 == 0: a wave's columns are all in or all out
  constexpr bool F32 = EPI == EPI_RESID_F32;
  constexpr int EPL = F32 ? 68 : 72;  // row pitch in elements (272 / 144 bytes)
  char* ep = smem + (size_t)w * (64 * 68 * 4);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int c = 16 * j + 4 * (l >> 4);
    const float4 bv4 = *reinterpret_cast<const float4*>(bias + colw + c);
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const int rl = 16 * i + (l & 15);
      float v[4] = {acc[i][j][0] + bv4.x, acc[i][j][1] + bv4.y, acc[i][j][2] + bv4.z, acc[i][j][3] + bv4.w};
      if constexpr (F32) {
        *reinterpret_cast<float4*>(reinterpret_cast<float*>(ep) + rl * EPL + c) = make_float4(v[0], v[1], v[2], v[3]);
      } else {
        if constexpr (EPI == EPI_GELU_BF16) {
#pragma unroll
          for (int rr = 0; rr < 4; ++rr) v[rr] = 0.5f * v[rr] * (1.0f + erf_fast(v[rr] * 0.70710678118654752f));
        }
        typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
        *reinterpret_cast<bf16x4*>(reinterpret_cast<bf16*>(ep) + rl * EPL + c) =
            (bf16x4){(bf16)v[0], (bf16)v[1], (bf16)v[2], (bf16)v[3]};
      }
    }
  }
  constexpr int CPR = F32 ? 16 : 8;  // 16-byte pieces per 64-column row
#pragma unroll
  for (int it = 0; it < 64 * CPR / 64; ++it) {
    const int pc = l + 64 * it, rl = pc / CPR, cp = pc - rl * CPR;
    const int row = roww + rl;
    if (row >= M) continue;
    if constexpr (F32) {
      const float4 v = *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(ep) + rl * EPL + 4 * cp);
      const size_t o = (size_t)row * N + colw + 4 * cp;
      const float4 rs = *reinterpret_cast<const float4*>(resid + o);
      *reinterpret_cast<float4*>(reinterpret_cast<float*>(out) + o) = make_float4(v.x + rs.x, v.y + rs.y, v.z + rs.z, v.w + rs.w);
    } else {
      const uint4 v = *reinterpret_cast<const uint4*>(reinterpret_cast<const bf16*>(ep) + rl * EPL + 8 * cp);
      *reinterpret_cast<uint4*>(reinterpret_cast<bf16*>(out) + (size_t)row * N + colw + 8 * cp) = v;
    }
  }
}

template <int EPI>
static void gemm3_launch(const bf16* A, const bf16* W, const float* bias, const float* resid, void* out, int M, int N,
                         int K, hipStream_t st) {
  const int tiles_n = (N + G3_BN - 1) / G3_BN, nblk = tiles_n * ((M + BM - 1) / BM);
  hipLaunchKernelGGL(k_gemm3<EPI>, dim3((unsigned)nblk), dim3(512), G3_LDS, st, A, W, bias, resid, out, M, N, K,
                     tiles_n, nblk);
}

// ---- GEMM in the reference's arithmetic: f32 operands, f32 MFMA ----------
// v_mfma_f32_32x32x2_f32 is an exact f32 fma chain (one rounding per
// product, f32 accumulation), i.e. the arithmetic of torch's fp32 Linear in
// another summation order. The K step is 32 floats, so a row of a stage is
// the 128 bytes of the bf16 kernel's (eight 16-byte chunks, the same XOR
// swizzle and LDS-DMA pieces). W is the MFMA's A operand (D = W . A^T: a lane
// holds four consecutive output columns per register group); within a K step
// the MFMA's two k slots take the halves of the step (lane half h supplies
// k = 16 h + t at step t), so a lane's operands of a group are one b128 read
// per 32-row tile.
constexpr int F_BK = 32;
enum { EPI_F32 = 3, EPI_GELU_F32 = 4 };  // (+ EPI_RESID_F32)
typedef float f32x16 __attribute__((ext_vector_type(16)));

// BERT's exact GELU in f32 (x * 0.5 * (1 + erf(x / sqrt(2))), transformers'
// GELUActivation): the library erff, not the bf16 path's 1.5e-7 approximation
__device__ __forceinline__ float gelu_erf(float x) { return 0.5f * x * (1.0f + erff(x * 0.70710678118654752f)); }

// 128 x 128 blocks of four waves (2 x 2, each 64 x 64 as 2 x 2 tiles of
// 32 x 32) with two LDS stages (64 KB; the epilogue's 68 KB bound the
// allocation), so two blocks share a CU and one's barriers and epilogue
// overlap the other's MFMAs. Against the bf16 kernel's 256 x 128 blocks of
// eight waves with three stages, in f32 (tools/gemm_probe.hip, docs/
// AB_LOG_r04.md): +7-8% on all four encoder shapes (121.7 / 116.6 / 120.6 /
// 123.0 TF against 113.5 / 108.4 / 111.4 / 114.4 at its best column width).
// Group u (k = 16 h + 4 u .. + 3) is read one group ahead into the other
// register set, behind group u's first MFMA (that MFMA's wait then covers
// group u's reads only); fragments are f32x4 ext_vectors: with HIP's float4
// struct hipcc waited vmcnt(0) before the first ds_read of every K step (the
// DMA just issued), draining the pipeline (tools/isa_lint.py checks).
constexpr int F2_BM = 128, F2_BN = 128, F2_STAGE = (F2_BM + F2_BN) * F_BK;
constexpr int F2_LDS = 4 * 64 * 68 * (int)sizeof(float);  // epilogue 69632 B >= 2 stages (65536 B)
template <int EPI>
__global__ void __launch_bounds__(256, 2) k_gemm2_f32(const float* __restrict__ A, const float* __restrict__ W,
                                                      const float* __restrict__ bias, const float* __restrict__ resid,
                                                      float* __restrict__ out, int M, int N, int K, int tiles_n,
                                                      int nblk) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* st = reinterpret_cast<float*>(smem);
  const int tid = threadIdx.x, l = tid & 63, h = l >> 5;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = w >> 1, wn = w & 1;
  const int b = blockIdx.x, xcd = b & 7, q = nblk >> 3, r = nblk & 7;
  const int t = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (b >> 3);
  const int m0 = (t / tiles_n) * F2_BM, n0 = (t - (t / tiles_n) * tiles_n) * F2_BN;
  const int KT = K / F_BK;
  auto issue = [&](int kt, int s) {
    float* la = st + s * F2_STAGE;
    float* lb = la + F2_BM * F_BK;
#pragma unroll
    for (int i = 0; i < 4; ++i) {  // A: 16 pieces of 8 rows x 128 B, four per wave
      const int pc = 4 * w + i, row = 8 * pc + (l >> 3), c = (l & 7) ^ (row & 7);
      const int gm = min(m0 + row, M - 1);
      __builtin_amdgcn_global_load_lds(A + (size_t)gm * K + kt * F_BK + 4 * c, (lds_void*)(la + pc * 8 * F_BK), 16, 0,
                                       0);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {  // W: 16 pieces, four per wave
      const int pc = 4 * w + i, row = 8 * pc + (l >> 3), c = (l & 7) ^ (row & 7);
      const int gn = min(n0 + row, N - 1);
      __builtin_amdgcn_global_load_lds(W + (size_t)gn * K + kt * F_BK + 4 * c, (lds_void*)(lb + pc * 8 * F_BK), 16, 0,
                                       0);
    }
  };
  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.0f;
  issue(0, 0);
  for (int kt = 0; kt < KT; ++kt) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's pieces of stage kt
    __builtin_amdgcn_s_barrier();                     // everyone's, and stage kt - 1 fully read
    if (kt + 1 < KT) issue(kt + 1, (kt + 1) & 1);
    const float* la = st + (kt & 1) * F2_STAGE;
    const float* lb = la + F2_BM * F_BK;
    f32x4 wv[2][2], av[2][2];
    auto rd = [&](int u, int bsel) {
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int m = wm * 64 + 32 * j + (l & 31);
        av[bsel][j] = *reinterpret_cast<const f32x4*>(la + m * F_BK + 4 * ((4 * h + u) ^ (m & 7)));
        const int n = wn * 64 + 32 * j + (l & 31);
        wv[bsel][j] = *reinterpret_cast<const f32x4*>(lb + n * F_BK + 4 * ((4 * h + u) ^ (n & 7)));
      }
    };
    rd(0, 0);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(wv[u & 1][0][0], av[u & 1][0][0], acc[0][0], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
      if (u < 3) rd(u + 1, (u + 1) & 1);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
            if (e | i | j)
              acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(wv[u & 1][i][e], av[u & 1][j][e], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
  __syncthreads();
  const int colw = n0 + wn * 64, roww = m0 + wm * 64;
  if (colw >= N) return;
  constexpr int EPL = 68;
  float* ep = reinterpret_cast<float*>(smem) + (size_t)w * (64 * EPL);
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int gq = 0; gq < 4; ++gq) {
      const int c = 32 * i + 8 * gq + 4 * h;
      const float4 bv4 = *reinterpret_cast<const float4*>(bias + colw + c);
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int rl = 32 * j + (l & 31);
        float v[4] = {acc[i][j][4 * gq] + bv4.x, acc[i][j][4 * gq + 1] + bv4.y, acc[i][j][4 * gq + 2] + bv4.z,
                      acc[i][j][4 * gq + 3] + bv4.w};
        if constexpr (EPI == EPI_GELU_F32) {
#pragma unroll
          for (int rr = 0; rr < 4; ++rr) v[rr] = gelu_erf(v[rr]);
        }
        *reinterpret_cast<float4*>(ep + rl * EPL + c) = make_float4(v[0], v[1], v[2], v[3]);
      }
    }
#pragma unroll
  for (int it = 0; it < 16; ++it) {
    const int pc = l + 64 * it, rl = pc >> 4, cp = pc & 15;
    const int row = roww + rl;
    if (row >= M) continue;
    float4 v = *reinterpret_cast<const float4*>(ep + rl * EPL + 4 * cp);
    const size_t o = (size_t)row * N + colw + 4 * cp;
    if constexpr (EPI == EPI_RESID_F32) {
      const float4 rs = *reinterpret_cast<const float4*>(resid + o);
      v = make_float4(v.x + rs.x, v.y + rs.y, v.z + rs.z, v.w + rs.w);
    }
    *reinterpret_cast<float4*>(out + o) = v;
  }
}
template <int EPI>
static void gemm2_f32_launch(const float* A, const float* W, const float* bias, const float* resid, float* out, int M,
                             int N, int K, hipStream_t st) {
  const int tiles_n = (N + F2_BN - 1) / F2_BN, nblk = tiles_n * ((M + F2_BM - 1) / F2_BM);
  hipLaunchKernelGGL(k_gemm2_f32<EPI>, dim3((unsigned)nblk), dim3(256), F2_LDS, st, A, W, bias, resid, out, M, N, K,
                     tiles_n, nblk);
}

// ---- fused attention (flash-style) ------------------------------------------
// One workgroup per (sequence, head) and 128 query rows (k_attention<8>; 64 rows of 4 waves beyond 256 tokens), 16 rows per wave.
// K ([Sp][72]) and V transposed ([64][Sp + 8]) of the head are staged in LDS
// once; each wave walks the keys in chunks of 64: S = Q K^T by MFMA (scale
// 1/8, key mask as -inf), online softmax (running max and sum per row), P
// (bf16) through a wave-private LDS tile into the A operand of O += P V.
// Rows: 4 (lane >> 4) + reg of the 16x16 C layout, so a row's 16 keys of a
// tile sit on the 16 lanes of one lane group (xor-shuffle reductions).
constexpr int HD = 64, KLD = HD + 8;

__device__ __forceinline__ float group16_max(float v) {
#pragma unroll
  for (int o = 1; o < 16; o <<= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ float group16_sum(float v) {
#pragma unroll
  for (int o = 1; o < 16; o <<= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// NW waves of 16 query rows each: 8 (128 rows) up to Sp = 256, so a
// sequence of <= 128 tokens stages its head's K and V once instead of once per
// 64 query rows; 4 beyond (the LDS of Sp = 512).
template <int NW>
__global__ void __launch_bounds__(NW * 64) k_attention(const bf16* __restrict__ qkv, const int32_t* __restrict__ mask,
                                                       bf16* __restrict__ ctx, int S, int Sp, int nh, int H) {
  constexpr int NT = NW * 64;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int VLD = Sp + 8;
  bf16* Ks = reinterpret_cast<bf16*>(smem);       // [Sp][KLD]
  bf16* Vt = Ks + Sp * KLD;                        // [HD][VLD]
  bf16* Ps = Vt + HD * VLD;                        // [NW][16][KLD]
  float* madd = reinterpret_cast<float*>(Ps + NW * 16 * KLD);  // [Sp]
  const int tid = threadIdx.x, l = tid & 63, w = tid >> 6;
  const int b = blockIdx.x / nh, h = blockIdx.x - b * nh;
  const int H3 = 3 * H;
  const bf16* base = qkv + (size_t)b * S * H3 + h * HD;
  for (int idx = tid; idx < Sp * 8; idx += NT) {
    const int s = idx >> 3, c = (idx & 7) * 8;
    uint4 kv = make_uint4(0, 0, 0, 0), vv = make_uint4(0, 0, 0, 0);
    if (s < S) {
      kv = *reinterpret_cast<const uint4*>(base + (size_t)s * H3 + H + c);
      vv = *reinterpret_cast<const uint4*>(base + (size_t)s * H3 + 2 * H + c);
    }
    *reinterpret_cast<uint4*>(Ks + s * KLD + c) = kv;
    const bf16* ve = reinterpret_cast<const bf16*>(&vv);
#pragma unroll
    for (int j = 0; j < 8; ++j) Vt[(c + j) * VLD + s] = ve[j];
  }
  for (int s = tid; s < Sp; s += NT) madd[s] = (s < S && mask[(size_t)b * S + s] != 0) ? 0.0f : -INFINITY;
  __syncthreads();
  const int q0 = blockIdx.y * (16 * NW) + w * 16;
  if (q0 >= S) return;  // no barrier below
  const int qr = q0 + (l & 15);
  bf16x8 qa[2];
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) {
    const uint4 z = qr < S ? *reinterpret_cast<const uint4*>(base + (size_t)qr * H3 + 32 * ks + 8 * (l >> 4))
                           : make_uint4(0, 0, 0, 0);
    qa[ks] = __builtin_bit_cast(bf16x8, z);
  }
  float m[4], lsum[4];
  f32x4 o[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) m[r] = -INFINITY, lsum[r] = 0.0f;
#pragma unroll
  for (int d = 0; d < 4; ++d) o[d] = (f32x4){0.f, 0.f, 0.f, 0.f};
  bf16* pw = Ps + w * 16 * KLD;
  for (int c0 = 0; c0 < Sp; c0 += 64) {
    f32x4 s[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      s[t] = (f32x4){0.f, 0.f, 0.f, 0.f};
      const bf16* kr = Ks + (c0 + 16 * t + (l & 15)) * KLD + 8 * (l >> 4);
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
        s[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(qa[ks], *reinterpret_cast<const bf16x8*>(kr + 32 * ks), s[t], 0,
                                                       0, 0);
      const float ma = madd[c0 + 16 * t + (l & 15)];
#pragma unroll
      for (int r = 0; r < 4; ++r) s[t][r] = s[t][r] * 0.125f + ma;
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float mc = fmaxf(fmaxf(s[0][r], s[1][r]), fmaxf(s[2][r], s[3][r]));
      mc = group16_max(mc);
      const float mn = fmaxf(m[r], mc);
      // chunk 0 holds key 0 ([CLS], never masked), so mn is finite from it on
      const float alpha = __expf(m[r] - mn);
      m[r] = mn;
      float ps = 0.0f;
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const float p = __expf(s[t][r] - mn);
        s[t][r] = p;
        ps += p;
      }
      lsum[r] = lsum[r] * alpha + ps;
#pragma unroll
      for (int d = 0; d < 4; ++d) o[d][r] *= alpha;
    }
    // P -> the wave's LDS tile (rows 4 (l >> 4) + r, keys 16 t + (l & 15)),
    // read back as A fragments; one wave's DS operations complete in order
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) pw[(4 * (l >> 4) + r) * KLD + 16 * t + (l & 15)] = (bf16)s[t][r];
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const bf16x8 pa = *reinterpret_cast<const bf16x8*>(pw + (l & 15) * KLD + 32 * ks + 8 * (l >> 4));
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        const bf16x8 vb =
            *reinterpret_cast<const bf16x8*>(Vt + (16 * d + (l & 15)) * VLD + c0 + 32 * ks + 8 * (l >> 4));
        o[d] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pa, vb, o[d], 0, 0, 0);
      }
    }
    __builtin_amdgcn_wave_barrier();  // the next chunk's P writes follow these reads
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const float inv = 1.0f / group16_sum(lsum[r]);
    const int row = q0 + 4 * (l >> 4) + r;
    if (row >= S) continue;
    bf16* dst = ctx + ((size_t)b * S + row) * H + h * HD + (l & 15);
#pragma unroll
    for (int d = 0; d < 4; ++d) dst[16 * d] = (bf16)(o[d][r] * inv);
  }
}

// ---- attention in f32 (the reference's arithmetic) --------------------------
// One workgroup per (sequence, head, 128 query rows), four waves of 32 rows.
// Keys stream through LDS in blocks of 64 (K and V rows, pitch 68 floats).
// Per 32-key tile a wave forms S^T = K . Q^T on v_mfma_f32_32x32x2_f32 (key on
// the register, query on the lane: lane half h takes head dims 32 h + t at
// step t, its Q row slice lives in 32 VGPRs), so the softmax's per-query max
// and sum run over a lane's own registers plus one xor-32 exchange, and P^T
// stays in registers as the B operand of O^T += V^T . P^T (register r of the
// S^T tile is the k slot of one MFMA: keys (r & 3) + 8 (r >> 2) + 4 h).
// Scale 1/8 and the mask (-inf) as BertSelfAttention; f32 exp.
constexpr int FA_KB = 64, FA_LD = HD + 4;

__global__ void __launch_bounds__(256) k_attention_f32(const float* __restrict__ qkv, const int32_t* __restrict__ mask,
                                                       float* __restrict__ ctx, int S, int nh, int H) {
  __shared__ __attribute__((aligned(16))) float Ks[FA_KB * FA_LD];
  __shared__ __attribute__((aligned(16))) float Vs[FA_KB * FA_LD];
  __shared__ float madd[FA_KB];
  const int tid = threadIdx.x, l = tid & 63, h = l >> 5, w = tid >> 6;
  const int b = blockIdx.x / nh, hd = blockIdx.x - b * nh;
  const int H3 = 3 * H;
  const float* base = qkv + (size_t)b * S * H3 + hd * HD;
  const int q0 = blockIdx.y * 128 + w * 32, qr = q0 + (l & 31);
  float qv[32];
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    const float4 z = qr < S ? *reinterpret_cast<const float4*>(base + (size_t)qr * H3 + 32 * h + 4 * u)
                            : make_float4(0.f, 0.f, 0.f, 0.f);
    qv[4 * u] = z.x, qv[4 * u + 1] = z.y, qv[4 * u + 2] = z.z, qv[4 * u + 3] = z.w;
  }
  float m = -INFINITY, lsum = 0.0f;
  f32x16 o[2];
#pragma unroll
  for (int e = 0; e < 16; ++e) o[0][e] = o[1][e] = 0.0f;
  for (int k0 = 0; k0 < S; k0 += FA_KB) {
    __syncthreads();  // the previous block's reads are done
    for (int idx = tid; idx < FA_KB * 16; idx += 256) {
      const int s = idx >> 4, c = (idx & 15) * 4;
      float4 kv = make_float4(0.f, 0.f, 0.f, 0.f), vv = kv;
      if (k0 + s < S) {
        kv = *reinterpret_cast<const float4*>(base + (size_t)(k0 + s) * H3 + H + c);
        vv = *reinterpret_cast<const float4*>(base + (size_t)(k0 + s) * H3 + 2 * H + c);
      }
      *reinterpret_cast<float4*>(Ks + s * FA_LD + c) = kv;
      *reinterpret_cast<float4*>(Vs + s * FA_LD + c) = vv;
    }
    if (tid < FA_KB) madd[tid] = (k0 + tid < S && mask[(size_t)b * S + k0 + tid] != 0) ? 0.0f : -INFINITY;
    __syncthreads();
    if (q0 >= S) continue;  // no work, but this wave keeps joining the barriers
    f32x16 s[2];
#pragma unroll
    for (int kt = 0; kt < 2; ++kt) {
#pragma unroll
      for (int e = 0; e < 16; ++e) s[kt][e] = 0.0f;
      const float* kr = Ks + (32 * kt + (l & 31)) * FA_LD + 32 * h;
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const float4 kk = *reinterpret_cast<const float4*>(kr + 4 * u);
        s[kt] = __builtin_amdgcn_mfma_f32_32x32x2f32(kk.x, qv[4 * u], s[kt], 0, 0, 0);
        s[kt] = __builtin_amdgcn_mfma_f32_32x32x2f32(kk.y, qv[4 * u + 1], s[kt], 0, 0, 0);
        s[kt] = __builtin_amdgcn_mfma_f32_32x32x2f32(kk.z, qv[4 * u + 2], s[kt], 0, 0, 0);
        s[kt] = __builtin_amdgcn_mfma_f32_32x32x2f32(kk.w, qv[4 * u + 3], s[kt], 0, 0, 0);
      }
    }
    float mc = -INFINITY;
#pragma unroll
    for (int kt = 0; kt < 2; ++kt)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int key = 32 * kt + (e & 3) + 8 * (e >> 2) + 4 * h;
        s[kt][e] = s[kt][e] * 0.125f + madd[key];
        mc = fmaxf(mc, s[kt][e]);
      }
    mc = fmaxf(mc, __shfl_xor(mc, 32, 64));
    const float mn = fmaxf(m, mc);  // block 0 holds key 0 ([CLS], never masked): finite from it on
    const float alpha = expf(m - mn);
    m = mn;
    float ps = 0.0f;
#pragma unroll
    for (int kt = 0; kt < 2; ++kt)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        s[kt][e] = expf(s[kt][e] - mn);
        ps += s[kt][e];
      }
    lsum = lsum * alpha + ps;  // this lane half's keys; the halves meet at the end
#pragma unroll
    for (int e = 0; e < 16; ++e) o[0][e] *= alpha, o[1][e] *= alpha;
#pragma unroll
    for (int kt = 0; kt < 2; ++kt)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const float* vr = Vs + (32 * kt + (e & 3) + 8 * (e >> 2) + 4 * h) * FA_LD + (l & 31);
        o[0] = __builtin_amdgcn_mfma_f32_32x32x2f32(vr[0], s[kt][e], o[0], 0, 0, 0);
        o[1] = __builtin_amdgcn_mfma_f32_32x32x2f32(vr[32], s[kt][e], o[1], 0, 0, 0);
      }
  }
  if (qr >= S) return;
  const float inv = 1.0f / (lsum + __shfl_xor(lsum, 32, 64));
  float* dst = ctx + ((size_t)b * S + qr) * H + hd * HD;
#pragma unroll
  for (int dt = 0; dt < 2; ++dt)
#pragma unroll
    for (int gq = 0; gq < 4; ++gq)
      *reinterpret_cast<float4*>(dst + 32 * dt + 8 * gq + 4 * h) =
          make_float4(o[dt][4 * gq] * inv, o[dt][4 * gq + 1] * inv, o[dt][4 * gq + 2] * inv, o[dt][4 * gq + 3] * inv);
}

// ---- LayerNorm, embeddings, pooling ------------------------------------------
// one wave per row of H <= 1024 (H / 64 values per lane), fp32 two-pass
// mean / variance as torch.nn.functional.layer_norm (biased variance)
constexpr int LN_MAXV = 16;
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ void ln_row(float (&v)[LN_MAXV], int nv, const float* g, const float* be, float eps,
                                       int l, float* y, bf16* yb, int H) {
  float s = 0.0f;
  for (int j = 0; j < nv; ++j) s += v[j];
  const float mean = wave_sum(s) / (float)H;
  float q = 0.0f;
  for (int j = 0; j < nv; ++j) {
    const float d = v[j] - mean;
    q += d * d;
  }
  const float rstd = 1.0f / sqrtf(wave_sum(q) / (float)H + eps);
  for (int j = 0; j < nv; ++j) {
    const int c = j * 64 + l;
    const float r = (v[j] - mean) * rstd * g[c] + be[c];
    y[c] = r;
    if (yb) yb[c] = (bf16)r;  // the bf16 GEMM input (bf16 arithmetic only)
  }
}

__global__ void __launch_bounds__(256) k_layernorm(const float* __restrict__ x, const float* __restrict__ g,
                                                   const float* __restrict__ be, float* __restrict__ y,
                                                   bf16* __restrict__ yb, int M, int H, float eps) {
  const int l = threadIdx.x & 63, row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= M) return;
  const int nv = H / 64;
  float v[LN_MAXV];
  for (int j = 0; j < nv; ++j) v[j] = x[(size_t)row * H + j * 64 + l];
  ln_row(v, nv, g, be, eps, l, y + (size_t)row * H, yb ? yb + (size_t)row * H : nullptr, H);
}

// the same LayerNorm with 16-byte accesses (H % 256 == 0): lane l holds
// columns 4l..4l+3 of each 256-column piece, so a row of 768 is three
// float4 loads per lane instead of twelve dword loads
__global__ void __launch_bounds__(256) k_layernorm4(const float* __restrict__ x, const float* __restrict__ g,
                                                    const float* __restrict__ be, float* __restrict__ y,
                                                    bf16* __restrict__ yb, int M, int H, float eps) {
  const int l = threadIdx.x & 63, row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= M) return;
  const int nv = H / 256;  // <= LN_MAXV / 4
  float4 v[LN_MAXV / 4];
  float s = 0.0f;
#pragma unroll
  for (int j = 0; j < LN_MAXV / 4; ++j) {
    if (j >= nv) break;
    v[j] = *reinterpret_cast<const float4*>(x + (size_t)row * H + j * 256 + 4 * l);
    s += (v[j].x + v[j].y) + (v[j].z + v[j].w);
  }
  const float mean = wave_sum(s) / (float)H;
  float q = 0.0f;
#pragma unroll
  for (int j = 0; j < LN_MAXV / 4; ++j) {
    if (j >= nv) break;
    const float a = v[j].x - mean, b = v[j].y - mean, c = v[j].z - mean, d = v[j].w - mean;
    q += (a * a + b * b) + (c * c + d * d);
  }
  const float rstd = 1.0f / sqrtf(wave_sum(q) / (float)H + eps);
#pragma unroll
  for (int j = 0; j < LN_MAXV / 4; ++j) {
    if (j >= nv) break;
    const int c = j * 256 + 4 * l;
    const float4 gg = *reinterpret_cast<const float4*>(g + c), bb = *reinterpret_cast<const float4*>(be + c);
    const float4 r = make_float4((v[j].x - mean) * rstd * gg.x + bb.x, (v[j].y - mean) * rstd * gg.y + bb.y,
                                 (v[j].z - mean) * rstd * gg.z + bb.z, (v[j].w - mean) * rstd * gg.w + bb.w);
    *reinterpret_cast<float4*>(y + (size_t)row * H + c) = r;
    typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
    if (yb) *reinterpret_cast<bf16x4*>(yb + (size_t)row * H + c) = (bf16x4){(bf16)r.x, (bf16)r.y, (bf16)r.z, (bf16)r.w};
  }
}

__global__ void __launch_bounds__(256) k_embed_ln(const int32_t* __restrict__ ids, const int32_t* __restrict__ tt,
                                                  const float* __restrict__ we, const float* __restrict__ pe,
                                                  const float* __restrict__ te, const float* __restrict__ g,
                                                  const float* __restrict__ be, float* __restrict__ y,
                                                  bf16* __restrict__ yb, int M, int S, int H, int vocab, int ntype,
                                                  float eps) {
  const int l = threadIdx.x & 63, row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= M) return;
  const int s = row % S;
  int id = ids[row], t = tt ? tt[row] : 0;
  id = id < 0 ? 0 : (id >= vocab ? vocab - 1 : id);  // the host checks the range; never read out of bounds
  t = t < 0 ? 0 : (t >= ntype ? ntype - 1 : t);
  const int nv = H / 64;
  float v[LN_MAXV];
  for (int j = 0; j < nv; ++j) {
    const int c = j * 64 + l;
    v[j] = we[(size_t)id * H + c] + te[(size_t)t * H + c] + pe[(size_t)s * H + c];
  }
  ln_row(v, nv, g, be, eps, l, y + (size_t)row * H, yb ? yb + (size_t)row * H : nullptr, H);
}

// bert_embeddings.py:140-149: mean over the attention mask, [CLS], or max over
// all S positions; thread per (sequence, feature)
__global__ void k_pool(const float* __restrict__ h, const int32_t* __restrict__ mask, float* __restrict__ out, int B,
                       int S, int H, int mode) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (int64_t)B * H) return;
  const int b = (int)(e / H), c = (int)(e - (int64_t)b * H);
  const float* hb = h + (size_t)b * S * H + c;
  float r;
  if (mode == FHE_BERT_POOL_CLS) {
    r = hb[0];
  } else if (mode == FHE_BERT_POOL_MAX) {
    r = hb[0];
    for (int s = 1; s < S; ++s) r = fmaxf(r, hb[(size_t)s * H]);
  } else {
    float sum = 0.0f, cnt = 0.0f;
    for (int s = 0; s < S; ++s) {
      const float mk = (float)mask[(size_t)b * S + s];
      sum += hb[(size_t)s * H] * mk;
      cnt += mk;
    }
    r = sum / cnt;
  }
  out[e] = r;
}
}  // namespace fbert

// ================================================================ host ======
using namespace fbert;

namespace {
struct Layer {
  bf16 *wqkv = nullptr, *wo = nullptr, *wi = nullptr, *wo2 = nullptr;      // FHE_BERT_BF16
  float *fqkv = nullptr, *fo = nullptr, *fi = nullptr, *fo2 = nullptr;     // FHE_BERT_F32
  float *bqkv = nullptr, *bo = nullptr, *bi = nullptr, *bo2 = nullptr;
  float *ln1w = nullptr, *ln1b = nullptr, *ln2w = nullptr, *ln2b = nullptr;
};
struct Prof {
  std::vector<std::pair<hipEvent_t, hipEvent_t>> ev;
  int64_t launches = 0;
  double flops = 0.0;
};
}  // namespace

struct fhe_bert {
  fhe_bert_config cfg{};
  int device = -1;
  int precision = FHE_BERT_F32;  // the reference's arithmetic unless set otherwise before any tensor
  std::string err;
  float *we = nullptr, *pe = nullptr, *te = nullptr, *elnw = nullptr, *elnb = nullptr;
  std::vector<Layer> layers;
  std::vector<uint64_t> have;  // bit set of tensors loaded, per layer (+1 for the embeddings)
  void* ws = nullptr;
  size_t ws_bytes = 0;
  bool prof = false;
  Prof p_gemm, p_attn, p_other;
};

static int bfail(fhe_bert* h, int code, const std::string& m) {
  if (h) h->err = m;
  return code;
}
#define BCHK(h, call)                                                                  \
  do {                                                                                 \
    hipError_t e_ = (call);                                                            \
    if (e_ != hipSuccess) return bfail(h, FHE_E_DEVICE, std::string(#call ": ") + hipGetErrorString(e_)); \
  } while (0)

static uint16_t to_bf16_bits(float f) {  // round to nearest even (finite inputs)
  uint32_t u;
  std::memcpy(&u, &f, 4);
  if ((u & 0x7f800000u) == 0x7f800000u) return (uint16_t)(u >> 16);
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}

// (the entry points keep the C linkage of their declarations in fhe_bert.h)
int fhe_bert_create(const fhe_bert_config* c, int device, fhe_bert** out) {
  if (!c || !out) return FHE_E_ARG;
  *out = nullptr;
  if (c->hidden_size <= 0 || c->hidden_size % 64 || c->hidden_size > 64 * LN_MAXV || c->num_heads <= 0 ||
      c->hidden_size != 64 * c->num_heads || c->intermediate_size <= 0 || c->intermediate_size % 64 ||
      c->num_layers <= 0 || c->vocab_size <= 0 || c->max_position <= 0 || c->max_position > 512 ||
      c->type_vocab_size <= 0 || !(c->layer_norm_eps > 0.0f))
    return FHE_E_ARG;  // head dim 64, hidden <= 1024, S <= 512 (attention LDS)
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || device < 0 || device >= n) return FHE_E_DEVICE;
  fhe_bert* h = new fhe_bert();
  h->cfg = *c;
  h->device = device;
  h->layers.resize(c->num_layers);
  h->have.assign(c->num_layers + 1, 0);
  // the >64 KB dynamic-LDS attribute of the kernels that need it, set on this
  // handle's device (the attribute is per device; every handle sets it)
  int rc = FHE_OK;
  if (hipSetDevice(device) != hipSuccess ||
      hipFuncSetAttribute((const void*)k_gemm3<EPI_BF16>, hipFuncAttributeMaxDynamicSharedMemorySize, G3_LDS) ||
      hipFuncSetAttribute((const void*)k_gemm3<EPI_GELU_BF16>, hipFuncAttributeMaxDynamicSharedMemorySize, G3_LDS) ||
      hipFuncSetAttribute((const void*)k_gemm3<EPI_RESID_F32>, hipFuncAttributeMaxDynamicSharedMemorySize, G3_LDS) ||
      hipFuncSetAttribute((const void*)k_gemm2_f32<EPI_F32>, hipFuncAttributeMaxDynamicSharedMemorySize, F2_LDS) ||
      hipFuncSetAttribute((const void*)k_gemm2_f32<EPI_GELU_F32>, hipFuncAttributeMaxDynamicSharedMemorySize, F2_LDS) ||
      hipFuncSetAttribute((const void*)k_gemm2_f32<EPI_RESID_F32>, hipFuncAttributeMaxDynamicSharedMemorySize, F2_LDS) ||
      hipFuncSetAttribute((const void*)k_attention<8>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) ||
      hipFuncSetAttribute((const void*)k_attention<4>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024))
    rc = FHE_E_DEVICE;
  if (rc) {
    delete h;
    return rc;
  }
  *out = h;
  return FHE_OK;
}

int fhe_bert_set_precision(fhe_bert* h, int32_t precision) {
  if (!h) return FHE_E_ARG;
  if (precision != FHE_BERT_F32 && precision != FHE_BERT_BF16) return bfail(h, FHE_E_ARG, "unknown precision");
  for (uint64_t m : h->have)
    if (m) return bfail(h, FHE_E_STATE, "set the precision before loading any tensor");
  h->precision = precision;
  return FHE_OK;
}

int fhe_bert_get_precision(const fhe_bert* h) { return h ? h->precision : FHE_E_ARG; }

static void free_all(fhe_bert* h) {
  auto f = [](void* p) {
    if (p) (void)hipFree(p);
  };
  f(h->we), f(h->pe), f(h->te), f(h->elnw), f(h->elnb), f(h->ws);
  for (auto& L : h->layers) {
    f(L.wqkv), f(L.wo), f(L.wi), f(L.wo2), f(L.bqkv), f(L.bo), f(L.bi), f(L.bo2);
    f(L.fqkv), f(L.fo), f(L.fi), f(L.fo2);
    f(L.ln1w), f(L.ln1b), f(L.ln2w), f(L.ln2b);
  }
  for (Prof* p : {&h->p_gemm, &h->p_attn, &h->p_other})
    for (auto& e : p->ev) (void)hipEventDestroy(e.first), (void)hipEventDestroy(e.second);
}

void fhe_bert_destroy(fhe_bert* h) {
  if (!h) return;
  (void)hipSetDevice(h->device);
  (void)hipDeviceSynchronize();
  free_all(h);
  delete h;
}

const char* fhe_bert_last_error(const fhe_bert* h) { return h ? h->err.c_str() : "null handle"; }

template <class T>
static int upload(fhe_bert* h, T** dst, const void* src, size_t bytes) {
  if (!*dst) BCHK(h, hipMalloc((void**)dst, bytes));
  BCHK(h, hipMemcpy(*dst, src, bytes, hipMemcpyHostToDevice));
  return FHE_OK;
}

int fhe_bert_set_tensor(fhe_bert* h, int32_t layer, int32_t which, const float* data, int64_t count) {
  if (!h) return FHE_E_ARG;
  if (!data || count <= 0) return bfail(h, FHE_E_ARG, "no data");
  BCHK(h, hipSetDevice(h->device));
  const fhe_bert_config& c = h->cfg;
  const int64_t H = c.hidden_size, I = c.intermediate_size;
  auto want = [&](int64_t n) { return count == n ? FHE_OK : bfail(h, FHE_E_ARG, "tensor " + std::to_string(which) +
                                                                           ": expected " + std::to_string(n) +
                                                                           " elements, got " + std::to_string(count)); };
  int rc;
  if (layer < 0) {
    switch (which) {
      case FHE_BERT_WORD_EMB: if ((rc = want((int64_t)c.vocab_size * H))) return rc; rc = upload(h, &h->we, data, count * 4); break;
      case FHE_BERT_POS_EMB: if ((rc = want((int64_t)c.max_position * H))) return rc; rc = upload(h, &h->pe, data, count * 4); break;
      case FHE_BERT_TYPE_EMB: if ((rc = want((int64_t)c.type_vocab_size * H))) return rc; rc = upload(h, &h->te, data, count * 4); break;
      case FHE_BERT_EMB_LN_W: if ((rc = want(H))) return rc; rc = upload(h, &h->elnw, data, count * 4); break;
      case FHE_BERT_EMB_LN_B: if ((rc = want(H))) return rc; rc = upload(h, &h->elnb, data, count * 4); break;
      default: return bfail(h, FHE_E_ARG, "unknown embedding tensor id");
    }
    if (rc) return rc;
    h->have[c.num_layers] |= 1ull << which;
    return FHE_OK;
  }
  if (layer >= c.num_layers) return bfail(h, FHE_E_ARG, "layer out of range");
  Layer& L = h->layers[layer];
  // GEMM weights -> bf16 (FHE_BERT_BF16) or as given (FHE_BERT_F32); Q, K and
  // V stack into one [3H][H] matrix
  const bool f32 = h->precision == FHE_BERT_F32;
  auto put_bf16 = [&](bf16** dst, size_t total, size_t off, int64_t n) -> int {
    if ((rc = want(n))) return rc;
    std::vector<uint16_t> t((size_t)n);
    for (int64_t i = 0; i < n; ++i) t[(size_t)i] = to_bf16_bits(data[i]);
    if (!*dst) BCHK(h, hipMalloc((void**)dst, total * 2));
    BCHK(h, hipMemcpy(*dst + off, t.data(), (size_t)n * 2, hipMemcpyHostToDevice));
    return FHE_OK;
  };
  auto put_f32 = [&](float** dst, size_t total, size_t off, int64_t n) -> int {
    if ((rc = want(n))) return rc;
    if (!*dst) BCHK(h, hipMalloc((void**)dst, total * 4));
    BCHK(h, hipMemcpy(*dst + off, data, (size_t)n * 4, hipMemcpyHostToDevice));
    return FHE_OK;
  };
  auto put_w = [&](bf16** db, float** df, size_t total, size_t off, int64_t n) -> int {
    return f32 ? put_f32(df, total, off, n) : put_bf16(db, total, off, n);
  };
  switch (which) {
    case FHE_BERT_Q_W: rc = put_w(&L.wqkv, &L.fqkv, 3 * H * H, 0, H * H); break;
    case FHE_BERT_K_W: rc = put_w(&L.wqkv, &L.fqkv, 3 * H * H, H * H, H * H); break;
    case FHE_BERT_V_W: rc = put_w(&L.wqkv, &L.fqkv, 3 * H * H, 2 * H * H, H * H); break;
    case FHE_BERT_Q_B: rc = put_f32(&L.bqkv, 3 * H, 0, H); break;
    case FHE_BERT_K_B: rc = put_f32(&L.bqkv, 3 * H, H, H); break;
    case FHE_BERT_V_B: rc = put_f32(&L.bqkv, 3 * H, 2 * H, H); break;
    case FHE_BERT_AO_W: rc = put_w(&L.wo, &L.fo, H * H, 0, H * H); break;
    case FHE_BERT_AO_B: rc = put_f32(&L.bo, H, 0, H); break;
    case FHE_BERT_AO_LN_W: rc = put_f32(&L.ln1w, H, 0, H); break;
    case FHE_BERT_AO_LN_B: rc = put_f32(&L.ln1b, H, 0, H); break;
    case FHE_BERT_I_W: rc = put_w(&L.wi, &L.fi, I * H, 0, I * H); break;
    case FHE_BERT_I_B: rc = put_f32(&L.bi, I, 0, I); break;
    case FHE_BERT_O_W: rc = put_w(&L.wo2, &L.fo2, H * I, 0, H * I); break;
    case FHE_BERT_O_B: rc = put_f32(&L.bo2, H, 0, H); break;
    case FHE_BERT_O_LN_W: rc = put_f32(&L.ln2w, H, 0, H); break;
    case FHE_BERT_O_LN_B: rc = put_f32(&L.ln2b, H, 0, H); break;
    default: return bfail(h, FHE_E_ARG, "unknown layer tensor id");
  }
  if (rc) return rc;
  h->have[layer] |= 1ull << which;
  return FHE_OK;
}

int fhe_bert_ready(const fhe_bert* h) {
  if (!h) return 0;
  const uint64_t emb = (1ull << 5) - 1, lay = ((1ull << 16) - 1) << 16;
  if ((h->have[h->cfg.num_layers] & emb) != emb) return 0;
  for (int l = 0; l < h->cfg.num_layers; ++l)
    if ((h->have[l] & lay) != lay) return 0;
  return 1;
}

int fhe_bert_profile_enable(fhe_bert* h, int enable) {
  if (!h) return FHE_E_ARG;
  h->prof = enable != 0;
  return FHE_OK;
}

static void pbegin(fhe_bert* h, Prof& p, hipStream_t st, hipEvent_t* e1) {
  *e1 = nullptr;
  if (!h->prof) return;
  hipEvent_t e0;
  if (hipEventCreate(&e0) != hipSuccess) return;
  if (hipEventCreate(e1) != hipSuccess) {
    (void)hipEventDestroy(e0);
    *e1 = nullptr;
    return;
  }
  (void)hipEventRecord(e0, st);
  p.ev.push_back({e0, *e1});
}
static void pend(fhe_bert* h, Prof& p, hipStream_t st, hipEvent_t e1, double flops) {
  if (!h->prof || !e1) return;
  (void)hipEventRecord(e1, st);
  p.launches += 1;
  p.flops += flops;
}

int fhe_bert_profile_read(fhe_bert* h, const char* kernel, double* total_ms, int64_t* launches, double* flops) {
  if (!h || !kernel) return FHE_E_ARG;
  Prof* p = !strcmp(kernel, "gemm") ? &h->p_gemm : !strcmp(kernel, "attention") ? &h->p_attn
                                                    : !strcmp(kernel, "other") ? &h->p_other : nullptr;
  if (!p) return bfail(h, FHE_E_ARG, "unknown kernel class");
  double ms = 0.0;
  for (auto& e : p->ev) {
    BCHK(h, hipEventSynchronize(e.second));
    float t = 0.0f;
    BCHK(h, hipEventElapsedTime(&t, e.first, e.second));
    ms += t;
    (void)hipEventDestroy(e.first);
    (void)hipEventDestroy(e.second);
  }
  p->ev.clear();
  if (total_ms) *total_ms = ms;
  if (launches) *launches = p->launches;
  if (flops) *flops = p->flops;
  p->launches = 0;
  p->flops = 0.0;
  return FHE_OK;
}

template <int EPI>
static int gemm(fhe_bert* h, const bf16* A, const bf16* W, const float* bias, const float* resid, void* out, int M,
                int N, int K, hipStream_t st) {
  hipEvent_t e1;
  pbegin(h, h->p_gemm, st, &e1);
  // the three-stage LDS-DMA form everywhere (tools/gemm_probe.hip against the
  // register-staged k_gemm: 12-34% faster on the four BERT shapes)
  gemm3_launch<EPI>(A, W, bias, resid, out, M, N, K, st);
  pend(h, h->p_gemm, st, e1, 2.0 * M * N * K);
  BCHK(h, hipGetLastError());
  return FHE_OK;
}

template <int EPI>
static int gemm_f32(fhe_bert* h, const float* A, const float* W, const float* bias, const float* resid, float* out,
                    int M, int N, int K, hipStream_t st) {
  hipEvent_t e1;
  pbegin(h, h->p_gemm, st, &e1);
  gemm2_f32_launch<EPI>(A, W, bias, resid, out, M, N, K, st);
  pend(h, h->p_gemm, st, e1, 2.0 * M * N * K);
  BCHK(h, hipGetLastError());
  return FHE_OK;
}

static int layernorm(fhe_bert* h, const float* x, const float* g, const float* b, float* y, bf16* yb, int M, int H,
                     float eps, hipStream_t st) {
  hipEvent_t e1;
  const unsigned rows4 = (unsigned)((M + 3) / 4);
  pbegin(h, h->p_other, st, &e1);
  if (H % 256 == 0)
    hipLaunchKernelGGL(k_layernorm4, dim3(rows4), dim3(256), 0, st, x, g, b, y, yb, M, H, eps);
  else
    hipLaunchKernelGGL(k_layernorm, dim3(rows4), dim3(256), 0, st, x, g, b, y, yb, M, H, eps);
  pend(h, h->p_other, st, e1, 0.0);
  BCHK(h, hipGetLastError());
  return FHE_OK;
}

// the f32 forward (FHE_BERT_F32): every GEMM and the attention on f32 MFMA,
// workspace h | tmp | qkv | ctx | inter, all f32
static int forward_f32(fhe_bert* h, const int32_t* d_mask, int B, int S, float* hs, hipStream_t st) {
  const fhe_bert_config& c = h->cfg;
  const int H = c.hidden_size, I = c.intermediate_size, nh = c.num_heads, M = B * S;
  float* tmp = hs + (size_t)M * H;
  float* qkv = tmp + (size_t)M * H;
  float* ctx = qkv + (size_t)M * 3 * H;
  float* inter = ctx + (size_t)M * H;
  const float eps = c.layer_norm_eps;
  hipEvent_t e1;
  int rc;
  for (int li = 0; li < c.num_layers; ++li) {
    const Layer& L = h->layers[li];
    if ((rc = gemm_f32<EPI_F32>(h, hs, L.fqkv, L.bqkv, nullptr, qkv, M, 3 * H, H, st))) return rc;
    pbegin(h, h->p_attn, st, &e1);
    hipLaunchKernelGGL(k_attention_f32, dim3((unsigned)(B * nh), (unsigned)((S + 127) / 128)), dim3(256), 0, st, qkv,
                       d_mask, ctx, S, nh, H);
    pend(h, h->p_attn, st, e1, 4.0 * B * nh * (double)S * S * HD);
    BCHK(h, hipGetLastError());
    if ((rc = gemm_f32<EPI_RESID_F32>(h, ctx, L.fo, L.bo, hs, tmp, M, H, H, st))) return rc;
    if ((rc = layernorm(h, tmp, L.ln1w, L.ln1b, hs, nullptr, M, H, eps, st))) return rc;
    if ((rc = gemm_f32<EPI_GELU_F32>(h, hs, L.fi, L.bi, nullptr, inter, M, I, H, st))) return rc;
    if ((rc = gemm_f32<EPI_RESID_F32>(h, inter, L.fo2, L.bo2, hs, tmp, M, H, I, st))) return rc;
    if ((rc = layernorm(h, tmp, L.ln2w, L.ln2b, hs, nullptr, M, H, eps, st))) return rc;
  }
  return FHE_OK;
}

// the bf16 forward (FHE_BERT_BF16): bf16 GEMM operands, f32 accumulation,
// workspace h f32 | tmp f32 | hb bf16 | qkv bf16 | ctx bf16 | inter bf16
static int forward_bf16(fhe_bert* h, const int32_t* d_mask, int B, int S, float* hs, hipStream_t st) {
  const fhe_bert_config& c = h->cfg;
  const int H = c.hidden_size, I = c.intermediate_size, nh = c.num_heads, M = B * S;
  float* tmp = hs + (size_t)M * H;
  bf16* hb = (bf16*)(tmp + (size_t)M * H);
  bf16* qkv = hb + (size_t)M * H;
  bf16* ctx = qkv + (size_t)M * 3 * H;
  bf16* inter = ctx + (size_t)M * H;
  const float eps = c.layer_norm_eps;
  const int Sp = (S + 63) / 64 * 64;
  const int anw = Sp <= 256 ? 8 : 4;  // waves per attention workgroup (k_attention)
  const size_t attn_lds = (size_t)Sp * KLD * 2 + (size_t)HD * (Sp + 8) * 2 + (size_t)anw * 16 * KLD * 2 + (size_t)Sp * 4;
  hipEvent_t e1;
  int rc;
  for (int li = 0; li < c.num_layers; ++li) {
    const Layer& L = h->layers[li];
    if ((rc = gemm<EPI_BF16>(h, hb, L.wqkv, L.bqkv, nullptr, qkv, M, 3 * H, H, st))) return rc;
    pbegin(h, h->p_attn, st, &e1);
    if (anw == 8)
      hipLaunchKernelGGL(k_attention<8>, dim3((unsigned)(B * nh), (unsigned)((Sp + 127) / 128)), dim3(512), attn_lds, st,
                         qkv, d_mask, ctx, S, Sp, nh, H);
    else
      hipLaunchKernelGGL(k_attention<4>, dim3((unsigned)(B * nh), (unsigned)(Sp / 64)), dim3(256), attn_lds, st, qkv,
                         d_mask, ctx, S, Sp, nh, H);
    pend(h, h->p_attn, st, e1, 4.0 * B * nh * (double)S * S * HD);
    BCHK(h, hipGetLastError());
    if ((rc = gemm<EPI_RESID_F32>(h, ctx, L.wo, L.bo, hs, tmp, M, H, H, st))) return rc;
    if ((rc = layernorm(h, tmp, L.ln1w, L.ln1b, hs, hb, M, H, eps, st))) return rc;
    if ((rc = gemm<EPI_GELU_BF16>(h, hb, L.wi, L.bi, nullptr, inter, M, I, H, st))) return rc;
    if ((rc = gemm<EPI_RESID_F32>(h, inter, L.wo2, L.bo2, hs, tmp, M, H, I, st))) return rc;
    if ((rc = layernorm(h, tmp, L.ln2w, L.ln2b, hs, hb, M, H, eps, st))) return rc;
  }
  return FHE_OK;
}

int fhe_bert_forward(fhe_bert* h, const int32_t* d_ids, const int32_t* d_type, const int32_t* d_mask, int32_t B,
                     int32_t S, int32_t pooling, float* d_out, void* stream) {
  if (!h) return FHE_E_ARG;
  const fhe_bert_config& c = h->cfg;
  if (B < 0 || S < 1 || S > c.max_position || pooling < 0 || pooling > FHE_BERT_POOL_NONE ||
      (B > 0 && (!d_ids || !d_mask || !d_out)))
    return bfail(h, FHE_E_ARG, "bad forward arguments (1 <= S <= max_position)");
  if (!fhe_bert_ready(h)) return bfail(h, FHE_E_STATE, "weights not loaded (fhe_bert_set_tensor)");
  if (B == 0) return FHE_OK;
  BCHK(h, hipSetDevice(h->device));
  hipStream_t st = (hipStream_t)stream;
  const int H = c.hidden_size, I = c.intermediate_size;
  const int64_t M64 = (int64_t)B * S;
  if (M64 > (1 << 24)) return bfail(h, FHE_E_ARG, "B * S too large: split the call");
  const int M = (int)M64;
  const bool f32 = h->precision == FHE_BERT_F32;
  // workspace: h f32 | tmp f32 | hb bf16 | qkv bf16 | ctx bf16 | inter bf16,
  // or (f32) h | tmp | qkv | ctx | inter, all f32
  const size_t need = f32 ? (size_t)M * 4 * (H + H + 3 * H + H + I)
                          : (size_t)M * (4 * H + 4 * H + 2 * H + 6 * H + 2 * H + 2 * I);
  if (need > h->ws_bytes) {
    if (h->ws) {
      BCHK(h, hipDeviceSynchronize());
      BCHK(h, hipFree(h->ws));
      h->ws = nullptr;
      h->ws_bytes = 0;
    }
    BCHK(h, hipMalloc(&h->ws, need));
    h->ws_bytes = need;
  }
  float* hs = (float*)h->ws;
  bf16* hb = (bf16*)(hs + 2 * (size_t)M * H);  // bf16: the GEMM copy of the embeddings' LayerNorm
  const float eps = c.layer_norm_eps;
  const unsigned rows4 = (unsigned)((M + 3) / 4);
  hipEvent_t e1;
  pbegin(h, h->p_other, st, &e1);
  hipLaunchKernelGGL(k_embed_ln, dim3(rows4), dim3(256), 0, st, d_ids, d_type, h->we, h->pe, h->te, h->elnw, h->elnb,
                     hs, f32 ? nullptr : hb, M, S, H, c.vocab_size, c.type_vocab_size, eps);
  pend(h, h->p_other, st, e1, 0.0);
  BCHK(h, hipGetLastError());
  int rc;
  if ((rc = f32 ? forward_f32(h, d_mask, B, S, hs, st) : forward_bf16(h, d_mask, B, S, hs, st))) return rc;
  if (pooling == FHE_BERT_POOL_NONE) {
    BCHK(h, hipMemcpyAsync(d_out, hs, (size_t)M * H * 4, hipMemcpyDeviceToDevice, st));
  } else {
    const int64_t tot = (int64_t)B * H;
    hipLaunchKernelGGL(k_pool, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, st, hs, d_mask, d_out, B, S, H,
                       pooling);
    BCHK(h, hipGetLastError());
  }
  return FHE_OK;
}
