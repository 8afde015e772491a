// Blind rotation kernels: v1 (one wave), v2 (br_m512.h), v4 (br_v4.h, the default).
// Part of libfheicp (one translation unit: fheicp.hip includes it).
#pragma once

#include <type_traits>

#include "common.h"
#include "br_m512.h"
#include "br_v4.h"

template <int LOGM, int K, class TV = BrTv>
__global__ void __launch_bounds__(64) k_blind_rotate(const u64* __restrict__ small, int n, int L, int beta,
                                                     const c64* __restrict__ bsk, const c64* __restrict__ tw,
                                                     const c64* __restrict__ twist, TV tv, int mode,
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

// ---- blind rotation for N = 1024, several waves per ciphertext -------------
// V = V2 (br_m512.h: 2 waves, 4 complex/lane).
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

template <class V, int K, int MINW, class TV = BrTv>
__global__ void __launch_bounds__(V::NT, MINW) k_blind_rotate_mw(const u64* __restrict__ small, int n, int L, int beta,
                                                              const c64* __restrict__ bsk, const c64* __restrict__ tw,
                                                              const c64* __restrict__ twist, TV tv, int mode,
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
// scale = 2^-64 / M: both accumulator widths (br_v4.h Acc) read the torus
// from z - floor(z) or z - rint(z), so the products arrive already scaled
// perm != 0 (the multi-bit keys of the gadgets mb_rotate runs with mb_xpose): the
// value of output point (slot u, lane) goes to [2 (lane >> 4) + (u & 1)]
// [16 (u >> 1) + (lane & 15)], so the product wave of quarter g, which loads
// key slot 2g + t at its lane l, gets point (slot 2 (l >> 4) + t, lane
// 16 g + (l & 15)).
__global__ void __launch_bounds__(64) k_bsk_to_fft_v4(const u64* __restrict__ bsk, int npoly,
                                                      const c64* __restrict__ tw4, c64* __restrict__ out,
                                                      double scale, int perm) {
  using namespace v4;
  __shared__ c64 twl[NTW];
  __shared__ c64 scr[SCR];
  const int lane = threadIdx.x;
  fill_tables(twl, tw4, lane, 64);
  __syncthreads();
  const double inv = scale;
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
    for (int u = 0; u < S; ++u) {
      const int pos = perm ? (2 * (lane >> 4) + (u & 1)) * 64 + 16 * (u >> 1) + (lane & 15) : u * 64 + lane;
      dst[pos] = {v[u].x * inv, v[u].y * inv};
    }
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
    // x is a whole number of 2^32 units: ties (x at exactly half a step) are
    // frequent, so round them to even, or the rounding error has a mean that
    // the key-weighted sum would turn into a phase bias
    const int sh = 32 - prec;
    uint32_t r = (x + ((1u << (sh - 1)) - 1u) + ((x >> sh) & 1u)) >> sh;
#pragma unroll
    for (int i = 0; i < L; ++i) {
      const int di = __builtin_amdgcn_sbfe((int)r, i * beta, beta);
      d[L - 1 - i] = di;
      if (i + 1 < L) r -= (uint32_t)di << (i * beta);
    }
  } else {
    // the same digits (round half up, then balanced), read without the
    // carry chain: adding 2^(63-prec) (the rounding) and the balancing offset
    // sum_i (B/2) B^i at bit 64-prec makes each digit its plain beta-bit field
    // minus B/2 (the representation mod B^L is unique; a carry out of bit 63
    // is a multiple of B^L). One 64-bit add, then a shift, mask and subtract
    // per digit, against a shift pair, a 64-bit subtract and more per digit.
    u64 k = (u64)1 << (63 - prec);
#pragma unroll
    for (int i = 0; i < L; ++i) k += (u64)1 << (64 - prec + i * beta + beta - 1);
    const u64 sx = x + k;
#pragma unroll
    for (int i = 0; i < L; ++i)
      d[L - 1 - i] = (int)((uint32_t)(sx >> (64 - prec + i * beta)) & ((1u << beta) - 1u)) - (1 << (beta - 1));
  }
}

// Phase timestamps (DBG bit 7): wave 0 of workgroup 0 records s_memtime at
// the phase boundaries of steps 100..103 (tools/prof_br.py --stamps).
__device__ unsigned long long g_v4_stamps[4][16];
// ... and every workgroup's {s_memrealtime at start, at end, HW_ID} (first 2048)
__device__ unsigned long long g_v4_span[2048][3];
#define V4_STAMP(k)                                                                        \
  do {                                                                                     \
    if constexpr ((DBG & 128) != 0) {                                                      \
      __builtin_amdgcn_sched_barrier(0);                                                   \
      stamp_[k] = __builtin_amdgcn_s_memtime();                                            \
      __builtin_amdgcn_sched_barrier(0);                                                   \
    }                                                                                      \
  } while (0)

// DBG != 0 only for timing experiments (tools/prof_br.py, FHEICP_V4_DBG):
// 1 twiddles from a register, 2 no BSK loads, 4 no barriers, 8 no FFT
// relayout, 16 no LDS rotation, 32 no LDS reads of the other components,
// 128 phase timestamps (results correct).
constexpr int FL_SYNC = 1;
// Wave priorities across the barriers of a step (k_blind_rotate_v4 / _mb /
// _v4s): raised right after each barrier and lowered half-way through the two
// long phases (after the inverse transform; after the first of two product
// halves), so the waves of a SIMD that are behind issue first and the three
// reach the next barrier together instead of the last one running alone.
// FHEICP_{V4,MB,V4S}_PRIO = 0 turns it off (A/B builds).
#ifndef FHEICP_MB_PRIO
#define FHEICP_MB_PRIO 1
#endif
#ifndef FHEICP_V4S_PRIO
#define FHEICP_V4S_PRIO 1
#endif
#ifndef FHEICP_V4_PRIO
#define FHEICP_V4_PRIO 1
#endif
#define BR_PRIO(EN, p)                                 \
  do {                                                 \
    if constexpr ((EN) != 0) __builtin_amdgcn_s_setprio(p); \
  } while (0)
#define MB_PRIO(p) BR_PRIO(FHEICP_MB_PRIO, p)
#define V4S_PRIO(p) BR_PRIO(FHEICP_V4S_PRIO, p)
#define V4_PRIO(p) BR_PRIO(FHEICP_V4_PRIO, p)
// Finer steps down the long phase (2 after the inverse, 1 after the digits)
// pay at L = 2, 3 (v4 (15,2) 9.26 -> 9.13, mb (15,2) 6.56 -> 6.48, v4s (12,3)
// 13.96 -> 13.72 ms) and cost at L = 1 and L >= 4 (mb (23,1) 3.81 -> 3.83,
// v4s (8,5) 20.27 -> 20.53, (6,7) 26.8 -> 27.2); FHEICP_PRIO_FINE = 0 / 1
// forces either (A/B builds)
#ifndef FHEICP_PRIO_FINE
#define FHEICP_PRIO_FINE -1
#endif
template <int L>
__device__ constexpr bool br_prio_fine() {
  return FHEICP_PRIO_FINE < 0 ? (L == 2 || L == 3) : FHEICP_PRIO_FINE != 0;
}

template <int L, bool A32, int DBG = 0, int G = 2, bool FL = false, int BETA = 0>
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
  // BSK rows through buffer loads: the lane's offset is fixed, the row's
  // (uniform: step, level, components) goes in the scalar offset; BETA != 0
  // fixes the base log at compile time (the shipped gadgets)
  const int bta = BETA ? BETA : beta;
  const __amdgpu_buffer_rsrc_t krs = __builtin_amdgcn_make_buffer_rsrc((void*)bsk, (short)0, 0x7fffffff, 0x00020000);
  const int klane = lane * (int)sizeof(c64);
  auto krow = [&](int row_c64, int u) -> c64 {  // element u * 64 + lane of the row at row_c64
    return __builtin_bit_cast(c64, __builtin_amdgcn_raw_buffer_load_b128(krs, klane, (row_c64 + u * 64) * (int)sizeof(c64), 0));
  };
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
        decompose_v4<L, A32>((T)(r - acc[s + h * S]), bta, d[h]);
      }
      v[s] = {(double)d[0][0], (double)d[1][0]};
#pragma unroll
      for (int l = 1; l < L; ++l) dg[l - 1][s] = (uint32_t)(d[0][l] & 0xffff) | ((uint32_t)d[1][l] << 16);
    }

    V4_STAMP(1);
    if constexpr (br_prio_fine<L>()) V4_PRIO(1);
    c64 mac[S];
#pragma unroll
    for (int u = 0; u < S; ++u) mac[u] = {0.0, 0.0};
    const int Gi = i * R * WPC * M;  // this step's GGSW, in c64 from bsk
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
      const int gpo = Gi + ((comp * L + lv) * WPC + comp) * M;
      c64 kb[PF ? S : 1];
      if constexpr (PF) {
#pragma unroll
        for (int u = 0; u < S; ++u) kb[u] = (DBG & 2) ? c64{wf.x + u, wf.y} : krow(gpo, u);
      }
      // the 32-bit-accumulator kernels also start one of the two other rows'
      // loads before the transform, at the first level (the MAC accumulator
      // is not live yet): 7.78 -> 7.02 ms per 1024 bootstraps at (23,1) (166
      // VGPRs), 11.92 -> 11.11 ms at (15,2) (168 VGPRs and a 20-byte spill;
      // loading only half the row early, without the spill, measured the same)
      constexpr bool EARLY_CT = A32 && PF;
      const bool EARLY = EARLY_CT && lv == 0;
      c64 ke[EARLY_CT ? S : 1];
      if (EARLY_CT && EARLY) {
        const int cin = comp + 1 >= WPC ? comp + 1 - WPC : comp + 1;
        const int gp = Gi + ((cin * L + lv) * WPC + comp) * M;
#pragma unroll
        for (int u = 0; u < S; ++u) ke[u] = (DBG & 2) ? c64{wf.x, wf.y + u} : krow(gp, u);
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
        else cmac(mac[u], v[u], (DBG & 2) ? c64{wf.x + u, wf.y} : krow(gpo, u));
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
          const int gp = Gi + ((cin * L + lv) * WPC + comp) * M;
#pragma unroll
          for (int u = 0; u < S; ++u) {
            if (EARLY && ci == 0) kx[ci][u] = ke[u];
            else kx[ci][u] = (DBG & 2) ? c64{wf.x + ci, wf.y + u} : krow(gp, u);
          }
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
      V4_PRIO(3);
      V4_STAMP(4 + 5 * lv);
#pragma unroll
      for (int ci = 0; ci < K; ++ci) {
        if (ci == 1) V4_PRIO(0);
        const int cin = comp + 1 + ci >= WPC ? comp + 1 + ci - WPC : comp + 1 + ci;
        const c64* fs = ctslots + cin * SCR;
        const int gp = Gi + ((cin * L + lv) * WPC + comp) * M;
#pragma unroll
        for (int hh = 0; hh < 2; ++hh) {  // F in halves: bounds register use at the peak
          c64 fv[S / 2], kv[S / 2];
#pragma unroll
          for (int u = 0; u < S / 2; ++u) {
            fv[u] = (DBG & 32) ? v[hh * 4 + u] : fs[(hh * 4 + u) * 64 + lane];
            if constexpr (PF) kv[u] = kx[ci][hh * 4 + u];
            else kv[u] = (DBG & 2) ? c64{wf.x + ci, wf.y + u} : krow(gp, hh * 4 + u);
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
      V4_PRIO(3);
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
    V4_PRIO(br_prio_fine<L>() ? 2 : 0);
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

// ---- multi-bit blind rotation (grouping factor 2) on the v4 layout ---------
// DESIGN.md §4.5. The LWE mask coefficients go in pairs (a1, a2) with secret
// bits (s1, s2); the key holds, per pair, GGSWs of the three indicators
// m_S = [s1 s2 pattern = S] for S = {1}, {2}, {1,2} (k_mb_msgs). One step per
// pair:
//   ACC += ExtProd(ACC, sum_S (X^{a_S} - 1) GGSW(m_S)),
// which rotates ACC by a_S of the one m_S that is 1 (none when s1 = s2 = 0).
// Each exponent is switched to 2N from its exact sum: a_{1,2} = round((A1 +
// A2) 2N / 2^64), not round(A1) + round(A2), so a pair with both bits set
// adds one rounding error to the phase instead of two (ms_var).
// The monomials act in the FFT domain: output position j of the forward
// transform holds the evaluation at psi^{e_j}, psi = exp(i pi / N),
// e_j = 4 bitrev9(j) + 1 (mb_exponent), so X^a multiplies it by psi^{a e_j}
// (a 2N-entry table in LDS). Per pair and wave: the digits of its own ACC
// component (no rotation and no LDS round trip), L forward transforms, the
// 3 x 3L row products per subset for its output component, the (psi^{a_S e}
// - 1) factors, one inverse: about the work of one classic step for two LWE
// coefficients, at half the barriers.
namespace fhei {
// The product wave of quarter g works on source lanes 16g..16g+15, all eight
// slots (lane l: slots 2 (l >> 4) + t), so that after its products two lane
// swaps give each lane all eight slots of one ciphertext: the wave runs the
// inverse's first DFT-8 pass itself and writes straight to the owner's
// relayout positions (8 LDS stores and 8 reads per wave and pair fewer).
// 0: quarter = slots 2g, 2g+1 of all lanes, products handed off as they are.
// Level-1 gadgets only (mb_xpose): mb<1,0,23> -1.0 to -1.5% per launch, while
// mb<2,0,15> was unchanged and mb64<4> 2.7% slower (docs/AB_LOG_r03.md).
#ifndef FHEICP_MB_XPOSE
#define FHEICP_MB_XPOSE 1
#endif
__host__ __device__ constexpr bool mb_xpose(int level) { return FHEICP_MB_XPOSE == 2 || (FHEICP_MB_XPOSE == 1 && level == 1); }
namespace mb {
constexpr int NP_MAX = (v4::NMAX + 1) / 2;  // pairs
__host__ __device__ constexpr int bitrev9(int j) {
  int r = 0;
  for (int b = 0; b < 9; ++b) r |= ((j >> b) & 1) << (8 - b);
  return r;
}
// exponent of output slot u of lane `lane` (layout LC): slot bits are index
// bits 0-2, so e = ebase(lane) + 256 bitrev3(u), ebase = 4 bitrev9(j(lane, 0)) + 1
__host__ __device__ constexpr int exponent(int lane, int u) {
  return (4 * bitrev9(v4::jof(v4::LC, lane, u)) + 1) & 2047;
}
// The table holds psi^x - 1 (the factor the products take; cos - 1 as
// -2 sin^2 for accuracy), stored swizzled, entry x at x ^ ((x >> 4) & 15): the
// gathers psi^(a e) of a 16-lane group otherwise pile onto a few bank quads
// (e mod 16 takes 4 values over a group): 38.7 LDS cycles per ds_read_b128
// on average over a, 8.9 swizzled (4 conflict-free; tools/psi_banks.py).
__host__ __device__ constexpr int psi_pos(int x) { return x ^ ((x >> 4) & 15); }
}  // namespace mb
}  // namespace fhei

// Key-stationary external product: in the product phase wave (g, c) works
// for output component c of ALL four ciphertexts of the workgroup, on the
// slot quarter {2g, 2g+1}. Every key element is then loaded once per CU
// instead of once per ciphertext (4x less L1 traffic, 18 instead of 72 load
// instructions per wave and level); the products go back to the owning waves
// through LDS (one more barrier per pair). Measured at 1024 bootstraps:
// 4.15 ms at (23,1) and 7.4 ms at (15,2), against 5.2 and 12.8 ms with
// per-ciphertext products and 6.0 / 10.1 ms for the classic v4 kernels.
//   per pair: digits -> [forward -> F to slot -> barrier -> products for the
//   quarter -> barrier] x L -> products to the owners' slots -> barrier ->
//   own slot -> inverse
// DBG != 0 only in A/B timing builds (wrong results): 2 = no key loads, 16 = no
// psi gathers, 32 = no F reads, 64 = no F stores; 128 = phase timestamps of
// wave DBG >> 8 of workgroup 0, pairs 100..103 (results correct).
// BETA != 0: the gadget base log as a constant (the shipped fast gadgets),
// which folds the digit shifts and widths into inline operands; 0 = `beta`.
// Key rows come through buffer loads: a per-lane offset fixed for the kernel
// and a scalar offset per row, so the loads take no VALU address arithmetic.
// AW = 1: 32-bit accumulators (L * beta <= 31, k_blind_rotate_mb); else wide
// ones (k_blind_rotate_mb64, the deep gadgets) that carry the rounding and
// balancing offset coff of decompose_v4's offset form from the start, so each
// level's digits are plain bit fields of the accumulator word (minus B/2),
// read when the level starts; the level loop is rolled from L = 3:
// AW = 0 u64 words with v4s's two-word rounding; AW = 2 48-bit words, the
// high 32 bits in acc[] and bits 16-31 of acc[u] and acc[u + S] packed in
// alo[u] (24 VGPRs instead of 32), each product rounded into them at 2^-48
// (n (1 + kN/2) 2^-96 / 12 = 2^-80 of variance, below the FFT error).
// TV: the test vector, the three-word staircase BrTv of the sign extraction
// or the table BrTvLut of fhe_pbs_table_batch (its own instantiations, so the
// hot kernels keep the narrow argument)
template <int L, int DBG, int BETA, int AW, class TV = BrTv>
__device__ __forceinline__ void mb_rotate(const u64* __restrict__ small, int64_t count, int n, int beta,
                                          const c64* __restrict__ bsk, const c64* __restrict__ tw4,
                                          const c64* __restrict__ psi, TV tv, int mode, u64* __restrict__ out,
                                          u64* __restrict__ ct_v, u64* __restrict__ refreshed, u64* __restrict__ sign) {
  using namespace v4;
  constexpr bool A32 = AW == 1, A48 = AW == 2;
  using AT = Acc<A32>;
  using T = std::conditional_t<A48, uint32_t, typename AT::T>;
#ifndef FHEICP_MB64_ROLL
#define FHEICP_MB64_ROLL 99  // fully unrolled (rolled from L: A/B builds)
#endif
  constexpr bool ROLL = !A32 && L >= FHEICP_MB64_ROLL;
  constexpr int G = 4, NT = nthreads(G), NPSI = 2 * N;
  constexpr int OFF_TW = NPSI, OFF_X = OFF_TW + NTW, NC64 = OFF_X + G * WPC * SCR;
  __shared__ c64 lds[NC64];
  // per pair and ciphertext: a1 | e << 11 | a2 << 16, with e - 1 = a12 - a1 - a2
  // (mod 2N) in {-1, 0, 1}: the pair's third exponent a12 is the switch of
  // the exact sum of its two mask words (one rounding, not two, when both key
  // bits are set: 3/4 of the pair's modulus-switch variance, ms_var)
  __shared__ uint32_t atab[mb::NP_MAX][G];
  c64* psil = lds;
  c64* twl = lds + OFF_TW;
  c64* xbuf = lds + OFF_X;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = w / WPC, comp = w - g * WPC;
  const int64_t c = (int64_t)blockIdx.x * G + g;
  c64* slot = xbuf + (g * WPC + comp) * SCR;
  using TS = std::conditional_t<A48, u64, T>;
  TS* sa = reinterpret_cast<TS*>(slot);
  const int np = (n + 1) >> 1;
  const int bta = BETA ? BETA : beta;
  const __amdgpu_buffer_rsrc_t krs = __builtin_amdgcn_make_buffer_rsrc((void*)bsk, (short)0, 0x7fffffff, 0x00020000);
  const int kvoff = (comp * M + 2 * g * 64 + lane) * (int)sizeof(c64);

  fill_tables(twl, tw4, tid, NT);
  for (int x = tid; x < NPSI; x += NT) psil[x] = psi[x];
#ifndef FHEICP_MB_TREG  // A/B builds only (tools/build_variant.sh)
#define FHEICP_MB_TREG 8
#endif
  // pass-A lane twiddles m < NR held in registers for the whole rotation
  // (L = 1 only). NR = 4: 154 -> 162 VGPRs, 8 fewer LDS reads per step, mb<1,0,23>
  // 4.02 -> 3.97 ms per 1024 (NR = 2 slower, 6 and 8 no better then). With the
  // wave priorities of BR_PRIO the kernel fell to 148 VGPRs, and all eight fit:
  // 3.77 -> 3.73 ms (NR = 6: 3.75; profiles/r02g_treg_ab.txt)
  constexpr int NR = (L == 1 && A32) ? FHEICP_MB_TREG : 0;
  c64 treg[NR > 0 ? NR : 1];
#pragma unroll
  for (int m = 0; m < NR; ++m) treg[m] = tw4[m * 64 + lane];
  for (int x = tid; x < G * np; x += NT) {
    const int gg = x / np, jj = x - gg * np;
    const int64_t cc = (int64_t)blockIdx.x * G + gg;
    uint32_t a1 = 0, a2 = 0, e = 1;
    if (cc < count) {
      const u64* sm = small + (size_t)cc * (n + 1);
      a1 = modswitch_2n(sm[2 * jj], 11);
      if (2 * jj + 1 < n) {
        a2 = modswitch_2n(sm[2 * jj + 1], 11);
        e = (modswitch_2n(sm[2 * jj] + sm[2 * jj + 1], 11) - a1 - a2 + 1) & (2 * N - 1);  // 0, 1 or 2
      }
    }
    atab[jj][gg] = a1 | (e << 11) | (a2 << 16);
  }
  __syncthreads();
  // this wave's product quarter: slots 2g, 2g+1; the exponent of slot 2g in
  // 16-byte units, so a * eb16 holds the table entry's byte offset (before
  // the swizzle) in bits 4-14
  constexpr bool XP = mb_xpose(L);
  const uint32_t eb16 = XP
                            ? ((uint32_t)mb::exponent(16 * g + (lane & 15), 2 * (lane >> 4)) & 2047u) << 4
                            : (((uint32_t)mb::exponent(lane, 0) + 256u * bitrev3(2 * g)) & 2047u) << 4;
  // this lane's F position in the slot regions for t = 0 (+ 64 t)
  const int fpos = XP ? 2 * (lane >> 4) * 64 + 16 * g + (lane & 15) : 0;

  // the offset of decompose_v4's offset form (wide accumulators carry it)
  const int prec = L * bta;
  u64 coff = 0;
  if constexpr (!A32) {
    coff = (u64)1 << (63 - prec);
    for (int l = 0; l < L; ++l) coff += (u64)1 << (64 - prec + l * bta + bta - 1);
  }
  T acc[2 * S];
  uint32_t alo[A48 ? S : 1];
  // the accumulator word s as u64 (A48: its bits 0-15 zero)
  auto word = [&](int s) -> u64 {
    if constexpr (A48)
      return ((u64)acc[s] << 32) | (s < S ? alo[s] << 16 : alo[s - S] & 0xffff0000u);
    else
      return AT::to64(acc[s]);
  };
  // A48: words u and u + S from u64 values whose bits 0-15 are dropped
  auto set48 = [&](int u, u64 a, u64 b) {
    acc[u] = (uint32_t)(a >> 32);
    acc[u + S] = (uint32_t)(b >> 32);
    alo[u] = __builtin_amdgcn_perm((uint32_t)b, (uint32_t)a, 0x07060302u);
  };
  {
    const uint32_t bt = c < count ? modswitch_2n(small[(size_t)c * (n + 1) + n], 11) : 0;
#pragma unroll
    for (int s = 0; s < 2 * S; ++s) {
      const uint32_t idx = (uint32_t)(s * 64 + lane + bt) & (2 * N - 1);
      if constexpr (A48) {
        if (s < S) {
          const uint32_t idx2 = (uint32_t)((s + S) * 64 + lane + bt) & (2 * N - 1);
          // the test vector (a multiple of 2^(64 - P)) plus coff: exact in 48 bits
          set48(s, (comp == K ? tv_rot(tv, idx, N) : 0) + coff, (comp == K ? tv_rot(tv, idx2, N) : 0) + coff);
        }
      } else if constexpr (A32) {
        acc[s] = comp == K ? AT::from64(tv_rot(tv, idx, N)) : (T)0;
      } else {
        acc[s] = (comp == K ? tv_rot(tv, idx, N) : 0) + coff;
      }
    }
  }

  constexpr int R = WPC * L;  // GGSW rows per subset
  // wide accumulators: digit lv of word x is the plain beta-bit field of x
  // (which carries coff) minus B/2
  auto digit_at = [&](int s, int lv) -> double {
    u64 w;
    if constexpr (A48) {
      uint32_t t = s < S ? alo[s] : alo[s - S];
      asm volatile("" : "+v"(t));  // unpacked per level, not hoisted out of the loop as 8 more VGPRs
      // bits 0-15 unused: fields start at 64 - L*beta >= 17 (validate() refuses L*beta > 47 here)
      w = ((u64)acc[s] << 32) | (s < S ? t << 16 : t);
    } else {
      w = (u64)acc[s];
    }
    return (double)((int)((uint32_t)(w >> (64 - prec + (L - 1 - lv) * bta)) & ((1u << bta) - 1u)) -
                    (1 << (bta - 1)));
  };
  for (int j = 0; j < np; ++j) {
    [[maybe_unused]] unsigned long long stamp_[16];
    V4_STAMP(0);
    uint32_t aS[G][3];
#pragma unroll
    for (int gg = 0; gg < G; ++gg) {
      const uint32_t aa = __builtin_amdgcn_readfirstlane(atab[j][gg]);
      aS[gg][0] = aa & 0x7ffu;
      aS[gg][1] = aa >> 16;
      aS[gg][2] = (aS[gg][0] + aS[gg][1] + ((aa >> 11) & 3u) - 1u) & (2 * N - 1);
    }
    c64 v[S];
    uint32_t dg[(L > 1 && A32) ? L - 1 : 1][S];
#pragma unroll
    for (int s = 0; s < S; ++s) {
      if constexpr (A32) {
        int d[2][L];
#pragma unroll
        for (int h = 0; h < 2; ++h) decompose_v4<L, true>(acc[s + h * S], bta, d[h]);
        v[s] = {(double)d[0][0], (double)d[1][0]};
#pragma unroll
        for (int l = 1; l < L; ++l) dg[l - 1][s] = (uint32_t)(d[0][l] & 0xffff) | ((uint32_t)d[1][l] << 16);
      } else {
        v[s] = {digit_at(s, 0), digit_at(s + S, 0)};
      }
    }
    V4_STAMP(1);
    if constexpr (br_prio_fine<L>()) MB_PRIO(1);
    c64 o[G][2];  // products of the quarter, per ciphertext
#pragma unroll
    for (int gg = 0; gg < G; ++gg) o[gg][0] = o[gg][1] = {0.0, 0.0};
    const int kjoff = j * 3 * R * WPC * M * (int)sizeof(c64);  // this pair's key, bytes
    constexpr int UNROLL_LV = ROLL ? 1 : L;
#pragma unroll UNROLL_LV
    for (int lv = 0; lv < L; ++lv) {
      if (lv > 0) {
#pragma unroll
        for (int u = 0; u < S; ++u) {
          if constexpr (A32)
            v[u] = {(double)(int16_t)(dg[lv - 1][u] & 0xffff), (double)((int32_t)dg[lv - 1][u] >> 16)};
          else
            v[u] = {digit_at(u, lv), digit_at(u + S, lv)};
        }
      }
      // key rows of this quarter, slot t: [subset][row] (9 per slot)
      c64 kb[2][3][WPC];
      auto load = [&](int t, c64 (&k)[3][WPC]) {
#pragma unroll
        for (int Ss = 0; Ss < 3; ++Ss)
#pragma unroll
          for (int r = 0; r < WPC; ++r)
            k[Ss][r] = (DBG & 2) ? c64{0.25 + r, 0.5 * t + Ss}
                                 : __builtin_bit_cast(c64, __builtin_amdgcn_raw_buffer_load_b128(
                                       krs, kvoff, kjoff + (((Ss * R + r * L + lv) * WPC) * M + t * 64) * (int)sizeof(c64), 0));
      };
      // (loading the first slot's rows before the transform instead, at L = 1:
      // 4.06 vs 4.04 ms per 1024, not kept)
      forward<0, NR>(v, twl, slot, lane, {}, treg);
      V4_STAMP(2 + 4 * lv);
      if constexpr ((DBG & 64) == 0) {
#pragma unroll
        for (int u = 0; u < S; ++u) slot[u * 64 + lane] = v[u];
      }
      load(0, kb[0]);
      V4_STAMP(3 + 4 * lv);
      lds_barrier();
      MB_PRIO(3);
      V4_STAMP(4 + 4 * lv);
      // slot 2g+1's exponent is slot 2g's plus 1024 (bitrev3(2g+1) =
      // bitrev3(2g) + 4): its table position is slot 2g's with bit 10
      // flipped when a is odd (the swizzle only reads bits 4-7), so the
      // address is computed once per (ciphertext, subset)
      uint32_t pa[G][3];  // byte offsets into the psi table
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        // the second slot's rows load when it starts: prefetching them with
        // the first slot's spilled at L = 2 (10.25 vs 7.36 ms per 1024)
        if (t == 1) {
          MB_PRIO(0);
          load(1, kb[1]);
        }
        const int u = 2 * g + t;
#pragma unroll
        for (int gg = 0; gg < G; ++gg) {
          c64 F[WPC];
#pragma unroll
          for (int r = 0; r < WPC; ++r)
            F[r] = (DBG & 32) ? c64{v[(gg + r) & 7].x, v[(gg + 2 * r + t) & 7].y}
                              : xbuf[(gg * WPC + r) * SCR + (XP ? fpos + t * 64 : u * 64 + lane)];
#pragma unroll
          for (int Ss = 0; Ss < 3; ++Ss) {
            c64 P = {0.0, 0.0};
#pragma unroll
            for (int r = 0; r < WPC; ++r) cmac(P, F[r], kb[t][Ss][r]);
            if (t == 0) {
              // 16 psi_pos(a e mod 2N) = X ^ ((X >> 4) & 0xf0), X = 16 (a e mod 2N)
              const uint32_t pr = __umul24(aS[gg][Ss], eb16);
              pa[gg][Ss] = (pr & 0x7ff0u) ^ ((pr >> 4) & 0xf0u);
            } else {
              pa[gg][Ss] ^= (aS[gg][Ss] & 1u) << 14;
            }
            // the table holds psi^x - 1
            if constexpr ((DBG & 16) != 0)
              cmac(o[gg][t], c64{__builtin_bit_cast(double, (u64)pa[gg][Ss] | 0x3fe0000000000000ull), 0.25}, P);
            else
              cmac(o[gg][t], *reinterpret_cast<const c64*>(reinterpret_cast<const char*>(psil) + pa[gg][Ss]), P);
          }
        }
      }
      V4_STAMP(5 + 4 * lv);
      lds_barrier();
      MB_PRIO(3);
    }
    c64 ov[S];
    if constexpr (XP) {
      // lane 16 q + s holds o[gg][t] = ciphertext gg, slot 2q + t of source
      // lane 16 g + s; exchanging q with gg (permlane32 / permlane16 swaps)
      // gives lane 16 gg + s the eight slots of ciphertext gg, on which this
      // wave runs the inverse's first pass and writes the owner's relayout
#pragma unroll
      for (int gg = 0; gg < G; ++gg)
#pragma unroll
        for (int t = 0; t < 2; ++t) ov[2 * gg + t] = o[gg][t];
      swap_bit<0, 4>(ov);
      swap_bit<1, 2>(ov);
      idft8(ov);
      c64* own = xbuf + ((lane >> 4) * WPC + comp) * SCR + rpos(R2I, jof(LC, 16 * g + (lane & 15), 0));
#pragma unroll
      for (int u = 0; u < S; ++u) own[rpos(R2I, jof(LC, 0, u))] = ov[u];
      lds_barrier();
      MB_PRIO(3);
      V4_STAMP(10);
#pragma unroll
      for (int u = 0; u < S; ++u) ov[u] = slot[rpos(R2I, jof(LB, lane, u))];
      inverse_post<0, NR>(ov, twl, slot, lane, {}, treg);
    } else {
      // products to the owners: ciphertext gg's component comp, slots 2g, 2g+1
#pragma unroll
      for (int gg = 0; gg < G; ++gg)
#pragma unroll
        for (int t = 0; t < 2; ++t) xbuf[(gg * WPC + comp) * SCR + (2 * g + t) * 64 + lane] = o[gg][t];
      lds_barrier();
      MB_PRIO(3);
      V4_STAMP(10);
#pragma unroll
      for (int u = 0; u < S; ++u) ov[u] = slot[u * 64 + lane];
      inverse<0, NR>(ov, twl, slot, lane, {}, treg);
    }
#pragma unroll
    for (int u = 0; u < S; ++u) {
      if constexpr (A48) {
        // + 2^15: the truncation to 48 bits rounds to nearest
        set48(u, word(u) + Acc<false>::from_f64(ov[u].x, 0x8000u), word(u + S) + Acc<false>::from_f64(ov[u].y, 0x8000u));
      } else {
        acc[u] += AT::from_f64(ov[u].x);
        acc[u + S] += AT::from_f64(ov[u].y);
      }
    }
    MB_PRIO(br_prio_fine<L>() ? 2 : 0);
    V4_STAMP(11);
    if constexpr ((DBG & 128) != 0)
      if (blockIdx.x == 0 && w == (DBG >> 8) && j >= 100 && j < 104 && lane < 16) {
        unsigned long long t_ = 0;
#pragma unroll
        for (int k = 0; k < 12; ++k) t_ = lane == k ? stamp_[k] : t_;
        g_v4_stamps[j - 100][lane] = t_;
      }
  }

  // sample extraction of coefficient 0 (as k_blind_rotate_v4)
  auto sword = [&](int i) -> u64 {
    if constexpr (A48)
      return sa[i] - coff;
    else
      return AT::to64(sa[i]) - coff;
  };
#pragma unroll
  for (int s = 0; s < 2 * S; ++s) {
    if constexpr (A48)
      sa[s * 64 + lane] = word(s);
    else
      sa[s * 64 + lane] = acc[s];
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  if (c < count) {
    const int W = K * N + 1;
    if (comp < K) {
#pragma unroll
      for (int s = 0; s < 2 * S; ++s) {
        const int t = s * 64 + lane;
        const u64 x = t == 0 ? sword(0) : (u64)0 - sword(N - t);
        br_emit(mode, x, false, tv, (size_t)c * W + comp * N + t, out, ct_v, refreshed, sign);
      }
    } else if (lane == 0) {
      br_emit(mode, word(0) - coff, true, tv, (size_t)c * W + K * N, out, ct_v, refreshed, sign);
    }
  }
}

template <int L, int DBG = 0, int BETA = 0, class TV = BrTv>
__global__ void __launch_bounds__(v4::nthreads(4), 1) k_blind_rotate_mb(const u64* __restrict__ small, int64_t count, int n,
                                                                      int beta, const c64* __restrict__ bsk,
                                                                      const c64* __restrict__ tw4,
                                                                      const c64* __restrict__ psi, TV tv, int mode,
                                                                      u64* __restrict__ out, u64* __restrict__ ct_v,
                                                                      u64* __restrict__ refreshed, u64* __restrict__ sign) {
  mb_rotate<L, DBG, BETA, 1, TV>(small, count, n, beta, bsk, tw4, psi, tv, mode, out, ct_v, refreshed, sign);
}
// the deep gadgets (L * beta > 31) on the multi-bit rotation: 48-bit accumulators
// (FHEICP_MB64_AW = 0: 64-bit ones, A/B builds)
#ifndef FHEICP_MB64_AW
#define FHEICP_MB64_AW 2
#endif
template <int L, int DBG = 0, class TV = BrTv>
__global__ void __launch_bounds__(v4::nthreads(4), 1) k_blind_rotate_mb64(const u64* __restrict__ small, int64_t count,
                                                                        int n, int beta, const c64* __restrict__ bsk,
                                                                        const c64* __restrict__ tw4,
                                                                        const c64* __restrict__ psi, TV tv, int mode,
                                                                        u64* __restrict__ out, u64* __restrict__ ct_v,
                                                                        u64* __restrict__ refreshed,
                                                                        u64* __restrict__ sign) {
  mb_rotate<L, DBG, 0, FHEICP_MB64_AW, TV>(small, count, n, beta, bsk, tw4, psi, tv, mode, out, ct_v, refreshed, sign);
}

// ---- classic blind rotation with key-stationary products ---------------------
#ifndef FHEICP_V4S_PARK
#define FHEICP_V4S_PARK 5
#endif
// k_blind_rotate_v4's step (rotation through the own slot, digits, L forward
// transforms, one inverse per wave) with the product phase of
// k_blind_rotate_mb: wave (g, c) forms output component c of all four
// ciphertexts on the slot quarter {2g, 2g+1}, so each key element is loaded
// once per CU (6 loads per wave and level instead of 24) and goes back to the
// owner through LDS (2L + 1 barriers per step instead of 2L). Key rows come
// through buffer loads (scalar row offsets) and BETA != 0 fixes the base log
// at compile time, as in k_blind_rotate_mb.
template <int L, bool A32, int DBG = 0, int BETA = 0>
__global__ void __launch_bounds__(v4::nthreads(4), 1) k_blind_rotate_v4s(const u64* __restrict__ small, int64_t count, int n,
                                                                      int beta, const c64* __restrict__ bsk,
                                                                      const c64* __restrict__ tw4, BrTv tv, int mode,
                                                                      u64* __restrict__ out, u64* __restrict__ ct_v,
                                                                      u64* __restrict__ refreshed, u64* __restrict__ sign) {
  using namespace v4;
  using AT = Acc<A32>;
  using T = typename AT::T;
  constexpr int G = 4, NT = nthreads(G);
  __shared__ c64 xbuf[G * WPC * SCR];
  __shared__ c64 twl[NTW];
  __shared__ uint16_t atab[G][NMAX + 1];
  // 64-bit accumulators from L = 4: PARK of the 16 words per lane wait out the
  // step in LDS (written after the rotation has read them, read back for the
  // update), 10 VGPRs less over the level loop, which otherwise spilled 56 B
  // per step to scratch (FHEICP_V4S_PARK = 0: A/B builds)
  constexpr int PARK = (!A32 && L >= 4) ? FHEICP_V4S_PARK : 0;
  __shared__ u64 park[PARK > 0 ? PARK * G * WPC * 64 : 1];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = w / WPC, comp = w - g * WPC;
  const int64_t c = (int64_t)blockIdx.x * G + g;
  c64* slot = xbuf + (g * WPC + comp) * SCR;
  T* sa = reinterpret_cast<T*>(slot);

  fill_tables(twl, tw4, tid, NT);
  for (int x = tid; x < G * (n + 1); x += NT) {
    const int gg = x / (n + 1), ii = x - gg * (n + 1);
    const int64_t cc = (int64_t)blockIdx.x * G + gg;
    atab[gg][ii] = cc < count ? (uint16_t)modswitch_2n(small[(size_t)cc * (n + 1) + ii], 11) : (uint16_t)0;
  }
  __syncthreads();

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
  const int bta = BETA ? BETA : beta;
  // this wave's key column and slot quarter: a per-lane offset fixed for the
  // kernel, a scalar one per row
  const __amdgpu_buffer_rsrc_t krs = __builtin_amdgcn_make_buffer_rsrc((void*)bsk, (short)0, 0x7fffffff, 0x00020000);
  const int kvoff = (comp * M + 2 * g * 64 + lane) * (int)sizeof(c64);
  auto load = [&](int i, int lv, c64 (&k)[2][WPC]) {
    const int ki = i * R * WPC * M * (int)sizeof(c64);
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int r = 0; r < WPC; ++r)
        k[t][r] = (DBG & 2) ? c64{0.25 + r, 0.5 * t + lv}
                            : __builtin_bit_cast(c64, __builtin_amdgcn_raw_buffer_load_b128(
                                  krs, kvoff, ki + (((r * L + lv) * WPC) * M + t * 64) * (int)sizeof(c64), 0));
  };
  // From L = 3 the level loop stays rolled: unrolled, the compiler hoists
  // work across levels and spills (28 bytes at L = 3, 172-532 at L = 4-7;
  // rolled: 0 at L = 3). From L = 4 the digits are not kept per level but
  // re-extracted from the difference plus the rounding and balancing
  // constant (decompose_v4's offset form): each is a plain beta-bit field
  // minus B/2, the same digits as the sequential balanced decomposition.
  constexpr bool ROLL = L >= 3;
  constexpr bool RECOMP = L >= 4;
  static_assert(!RECOMP || !A32, "re-extracted digits are for the 64-bit accumulators");
  // (decompose_v4's offset form: the rounding and balancing constant added
  // once, each level's digit a plain field of the sum)
  const int prec = L * bta;
  u64 coff = 0;
  if constexpr (RECOMP) {
    coff = (u64)1 << (63 - prec);
    for (int l = 0; l < L; ++l) coff += (u64)1 << (64 - prec + l * bta + bta - 1);
  }
  auto digit_at = [&](u64 rr, int lv) -> double {
    return (double)((int)((uint32_t)(rr >> (64 - prec + (L - 1 - lv) * bta)) & ((1u << bta) - 1u)) -
                    (1 << (bta - 1)));
  };
  c64 kb[2][WPC];  // this level's rows: [slot t][row]
  for (int i = 0; i < n; ++i) {
    [[maybe_unused]] unsigned long long stamp_[16];
    V4_STAMP(0);
    const uint32_t a = __builtin_amdgcn_readfirstlane((uint32_t)atab[g][i]);
#pragma unroll
    for (int s = 0; s < 2 * S; ++s) sa[s * 64 + lane] = acc[s];  // own slot: in-order DS, no wait
    c64 v[S];
    uint32_t dg[(L > 1 && !RECOMP) ? L - 1 : 1][S];
    u64 rr[RECOMP ? 2 * S : 1];
    T rot[2 * S];
#pragma unroll
    for (int s = 0; s < 2 * S; ++s) {
      const uint32_t src = (uint32_t)(s * 64 + lane - (int)a) & (2 * N - 1);
      rot[s] = sa[src & (N - 1)];
    }
#pragma unroll
    for (int s = 0; s < S; ++s) {
      if constexpr (RECOMP) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const uint32_t src = (uint32_t)((s + h * S) * 64 + lane - (int)a) & (2 * N - 1);
          const u64 x = (u64)((src >= (uint32_t)N ? (T)0 - rot[s + h * S] : rot[s + h * S]) - acc[s + h * S]);
          rr[s + h * S] = x + coff;
        }
        v[s] = {digit_at(rr[s], 0), digit_at(rr[s + S], 0)};
      } else {
        int d[2][L];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const uint32_t src = (uint32_t)((s + h * S) * 64 + lane - (int)a) & (2 * N - 1);
          const T r = src >= (uint32_t)N ? (T)0 - rot[s + h * S] : rot[s + h * S];
          decompose_v4<L, A32>((T)(r - acc[s + h * S]), bta, d[h]);
        }
        v[s] = {(double)d[0][0], (double)d[1][0]};
#pragma unroll
        for (int l = 1; l < L; ++l) dg[l - 1][s] = (uint32_t)(d[0][l] & 0xffff) | ((uint32_t)d[1][l] << 16);
      }
    }
    if constexpr (PARK > 0) {
#pragma unroll
      for (int s = 0; s < PARK; ++s) park[(s * G * WPC + w) * 64 + lane] = acc[s];
    }
    V4_STAMP(1);
    if constexpr (br_prio_fine<L>()) V4S_PRIO(1);
    c64 o[G][2];
#pragma unroll
    for (int gg = 0; gg < G; ++gg) o[gg][0] = o[gg][1] = {0.0, 0.0};
    constexpr int UNROLL_LV = ROLL ? 1 : L;
#pragma unroll UNROLL_LV
    for (int lv = 0; lv < L; ++lv) {
      if (lv > 0) {
#pragma unroll
        for (int u = 0; u < S; ++u) {
          if constexpr (RECOMP)
            v[u] = {digit_at(rr[u], lv), digit_at(rr[u + S], lv)};
          else
            v[u] = {(double)(int16_t)(dg[lv - 1][u] & 0xffff), (double)((int32_t)dg[lv - 1][u] >> 16)};
        }
      }
      // (this level's rows loaded before the transform, or the next level's
      // during the products, measured slower: FHEICP_V4S=1 A/B, round 2)
      forward(v, twl, slot, lane);
      // (12,3): a drop after the deeper levels' transforms too (13.67 -> 13.30 ms per
      // 1000 at C5); it costs 1-2% at L = 2 and L >= 4 (profiles/r02h_prio_fwd_ab.txt)
      if (L == 3 && lv > 0) V4S_PRIO(1);
      V4_STAMP(2 + 4 * lv);
#pragma unroll
      for (int u = 0; u < S; ++u) slot[u * 64 + lane] = v[u];
      load(i, lv, kb);
      V4_STAMP(3 + 4 * lv);
      lds_barrier();
      V4S_PRIO(3);
      V4_STAMP(4 + 4 * lv);
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        if (t == 1) V4S_PRIO(0);
        const int u = 2 * g + t;
#pragma unroll
        for (int gg = 0; gg < G; ++gg) {
          c64 F[WPC];
#pragma unroll
          for (int r = 0; r < WPC; ++r) F[r] = xbuf[(gg * WPC + r) * SCR + u * 64 + lane];
#pragma unroll
          for (int r = 0; r < WPC; ++r) cmac(o[gg][t], F[r], kb[t][r]);
#ifdef FHEICP_V4S_SB
          __builtin_amdgcn_sched_barrier(0);  // keep the F reads from all being hoisted (VGPRs)
#endif
        }
      }
      V4_STAMP(5 + 4 * lv);
      lds_barrier();
      V4S_PRIO(3);
    }
    // products to the owners: ciphertext gg's component comp, slots 2g, 2g+1
#pragma unroll
    for (int gg = 0; gg < G; ++gg)
#pragma unroll
      for (int t = 0; t < 2; ++t) xbuf[(gg * WPC + comp) * SCR + (2 * g + t) * 64 + lane] = o[gg][t];
    lds_barrier();
    V4S_PRIO(3);
    V4_STAMP(10);
    c64 ov[S];
#pragma unroll
    for (int u = 0; u < S; ++u) ov[u] = slot[u * 64 + lane];
    inverse(ov, twl, slot, lane);
    if constexpr (PARK > 0) {
#pragma unroll
      for (int s = 0; s < PARK; ++s) acc[s] = park[(s * G * WPC + w) * 64 + lane];
    }
#pragma unroll
    for (int u = 0; u < S; ++u) {
      acc[u] += AT::from_f64(ov[u].x);
      acc[u + S] += AT::from_f64(ov[u].y);
    }
    V4S_PRIO(br_prio_fine<L>() ? 2 : 0);
    V4_STAMP(11);
    if constexpr ((DBG & 128) != 0)
      if (blockIdx.x == 0 && w == (DBG >> 8) && i >= 100 && i < 104 && lane < 16) {
        unsigned long long t_ = 0;
#pragma unroll
        for (int k = 0; k < 12; ++k) t_ = lane == k ? stamp_[k] : t_;
        g_v4_stamps[i - 100][lane] = t_;
      }
  }

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
