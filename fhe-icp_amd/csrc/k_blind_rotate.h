// Blind rotation kernels: v1 (one wave), v2 (br_m512.h), v4 (br_v4.h, the default);
// v3 (br_m512q.h) only in A/B builds (FHEICP_AB, tools/build_variant.sh).
// Part of libfheicp (one translation unit: fheicp.hip includes it).
#pragma once

#include "common.h"
#include "br_m512.h"
#ifdef FHEICP_AB
#include "br_m512q.h"
#endif
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
// scale = 1/M, times 2^-64 for the 32-bit-accumulator kernels (Acc<true>
// reads the torus from fract(z), so the products arrive already scaled)
__global__ void __launch_bounds__(64) k_bsk_to_fft_v4(const u64* __restrict__ bsk, int npoly,
                                                      const c64* __restrict__ tw4, c64* __restrict__ out,
                                                      double scale) {
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
        const c64* gp = Gi + ((size_t)(cin * L + lv) * WPC + comp) * M;
#pragma unroll
        for (int u = 0; u < S; ++u) ke[u] = (DBG & 2) ? c64{wf.x, wf.y + u} : gp[u * 64 + lane];
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
          for (int u = 0; u < S; ++u) {
            if (EARLY && ci == 0) kx[ci][u] = ke[u];
            else kx[ci][u] = (DBG & 2) ? c64{wf.x + ci, wf.y + u} : gp[u * 64 + lane];
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
