// Wave-level negacyclic FFT for TFHE polynomial products on gfx950.
//
// A real polynomial a of size N over Z[X]/(X^N+1) is folded into M = N/2
// complex points  y[t] = (a[t] + i a[t+M]) * w^t,  w = exp(i*pi/N),
// and transformed with an M-point complex FFT (exponent +2*pi*i/M). The
// result holds the evaluations of a at the odd powers of exp(i*pi/N) that
// determine a negacyclic product. Forward is decimation-in-
// frequency (natural order in, bit-reversed out); inverse is the exact
// algebraic inverse (bit-reversed in, natural out, scaled by M). Pointwise
// products happen in the bit-reversed domain, so no reordering pass exists.
//
// Mapping: one 64-lane wavefront owns a transform; every lane holds S = M/64
// complex values. A "layout q" places index bits [q, q+log2 S) in the lane's
// slot u and the remaining 6 bits in the lane id l:
//     j(l, u, q) = (l & (2^q-1)) | (u << q) | ((l >> q) << (q + log2 S)).
// Each pass runs the radix-2 stages of its in-lane bits entirely in
// registers; passes are joined by one LDS transpose (ds_write_b128 /
// ds_read_b128 with a 1-in-8 element pad that keeps 16-lane groups
// bank-conflict free for the three layouts used at N = 1024).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace fhei {

struct alignas(16) c64 {
  double x, y;
};

__device__ __forceinline__ c64 cadd(c64 a, c64 b) { return {a.x + b.x, a.y + b.y}; }
__device__ __forceinline__ c64 csub(c64 a, c64 b) { return {a.x - b.x, a.y - b.y}; }
__device__ __forceinline__ c64 cmul(c64 a, c64 b) {
  return {__fma_rn(a.x, b.x, -a.y * b.y), __fma_rn(a.x, b.y, a.y * b.x)};
}
// a * conj(b)
__device__ __forceinline__ c64 cmulc(c64 a, c64 b) {
  return {__fma_rn(a.x, b.x, a.y * b.y), __fma_rn(a.y, b.x, -a.x * b.y)};
}
// acc += a * b
__device__ __forceinline__ void cmac(c64& acc, c64 a, c64 b) {
  acc.x = __fma_rn(a.x, b.x, __fma_rn(-a.y, b.y, acc.x));
  acc.y = __fma_rn(a.x, b.y, __fma_rn(a.y, b.x, acc.y));
}

__host__ __device__ constexpr int ilog2c(int x) { return x <= 1 ? 0 : 1 + ilog2c(x >> 1); }

// LDS element index with a 1-in-8 pad.
__device__ __forceinline__ int lds_pad(int j) { return j + (j >> 3); }

template <int LOGM>
struct WaveFFT {
  static constexpr int M = 1 << LOGM;
  static constexpr int S = M / 64;
  static constexpr int LOGS = ilog2c(S);
  static_assert(S >= 1 && (S & (S - 1)) == 0, "M must be a power of two >= 64");
  static constexpr int LDS_ELEMS = M + M / 8;  // c64 elements of transpose scratch
  static constexpr int Q_NAT = LOGM - LOGS;    // layout of natural order, j = l + 64 u

  __device__ __forceinline__ static int jidx(int l, int u, int q) {
    return (l & ((1 << q) - 1)) | (u << q) | ((l >> q) << (q + LOGS));
  }

  // Move v from layout qa to layout qb through LDS (one wave).
  __device__ __forceinline__ static void relayout(c64 (&v)[S], int qa, int qb, c64* lds, int l) {
#pragma unroll
    for (int u = 0; u < S; ++u) lds[lds_pad(jidx(l, u, qa))] = v[u];
    __syncthreads();
#pragma unroll
    for (int u = 0; u < S; ++u) v[u] = lds[lds_pad(jidx(l, u, qb))];
    __syncthreads();
  }

  // DIF radix-2 stages for bits top..q (h = 2^bit), data in layout q.
  __device__ __forceinline__ static void dif_pass(c64 (&v)[S], int q, int top, const c64* __restrict__ tw, int l) {
#pragma unroll
    for (int b = LOGS - 1; b >= 0; --b) {
      const int bit = q + b;
      if (bit > top) continue;
      const int h = 1 << bit;
#pragma unroll
      for (int u = 0; u < S; ++u) {
        if (u & (1 << b)) continue;
        const int jm = ((l & ((1 << q) - 1)) | ((u & ((1 << b) - 1)) << q));  // j mod h
        const c64 W = tw[jm * (M / 2 / h)];
        const c64 X = v[u], Y = v[u | (1 << b)];
        v[u] = cadd(X, Y);
        v[u | (1 << b)] = cmul(csub(X, Y), W);
      }
    }
  }

  // Inverse stages for bits q..top in increasing order (DIT, conjugate twiddles).
  __device__ __forceinline__ static void dit_pass(c64 (&v)[S], int q, int top, const c64* __restrict__ tw, int l) {
#pragma unroll
    for (int b = 0; b < LOGS; ++b) {
      const int bit = q + b;
      if (bit > top) continue;
      const int h = 1 << bit;
#pragma unroll
      for (int u = 0; u < S; ++u) {
        if (u & (1 << b)) continue;
        const int jm = ((l & ((1 << q) - 1)) | ((u & ((1 << b) - 1)) << q));
        const c64 W = tw[jm * (M / 2 / h)];
        const c64 X = v[u], Y = cmulc(v[u | (1 << b)], W);
        v[u] = cadd(X, Y);
        v[u | (1 << b)] = csub(X, Y);
      }
    }
  }

  // Pass schedule: pass p covers index bits [q_p, top_p] with
  // top_p = LOGM-1-p*LOGS and q_p = max(LOGM-(p+1)*LOGS, 0).
  static constexpr int NPASS = (LOGM + LOGS - 1) / LOGS;
  __host__ __device__ static constexpr int top_of(int p) { return LOGM - 1 - p * LOGS; }
  __host__ __device__ static constexpr int q_of(int p) { return LOGM - (p + 1) * LOGS > 0 ? LOGM - (p + 1) * LOGS : 0; }

  // Forward: v in natural layout (q = Q_NAT) -> bit-reversed, layout 0.
  __device__ __forceinline__ static void forward(c64 (&v)[S], const c64* __restrict__ tw, c64* lds, int l) {
    int qprev = Q_NAT;
#pragma unroll
    for (int p = 0; p < NPASS; ++p) {
      const int q = q_of(p), top = top_of(p);
      if (q != qprev) relayout(v, qprev, q, lds, l);
      dif_pass(v, q, top, tw, l);
      qprev = q;
    }
    if (qprev != 0) relayout(v, qprev, 0, lds, l);
  }

  // Inverse: v in layout 0 (bit-reversed) -> natural layout Q_NAT, times M.
  __device__ __forceinline__ static void inverse(c64 (&v)[S], const c64* __restrict__ tw, c64* lds, int l) {
    int qprev = 0;
#pragma unroll
    for (int p = NPASS - 1; p >= 0; --p) {
      const int q = q_of(p), top = top_of(p);
      if (q != qprev) relayout(v, qprev, q, lds, l);
      dit_pass(v, q, top, tw, l);
      qprev = q;
    }
    if (qprev != Q_NAT) relayout(v, qprev, Q_NAT, lds, l);
  }
};

// f64 -> u64 modulo 2^64 for an (approximately) integral value of any
// magnitude below 2^1023: subtract the nearest multiple of 2^64 exactly
// (|r| <= 2^63), then split r = hi * 2^32 + lo with hi, lo exact 32-bit
// integers (native v_cvt_i32_f64 / v_cvt_u32_f64 instead of the long
// generic f64 -> i64 sequence).
__device__ __forceinline__ uint64_t f64_to_torus(double v) {
  const double two64 = 18446744073709551616.0;
  const double m = rint(v * (1.0 / two64));
  const double r = rint(__fma_rn(-m, two64, v));      // exact, |r| <= 2^63
  const double hi = floor(r * (1.0 / 4294967296.0));  // |hi| <= 2^31
  const double lo = __fma_rn(-hi, 4294967296.0, r);   // exact, in [0, 2^32)
  const uint32_t hu = (uint32_t)(int32_t)(hi >= 2147483648.0 ? hi - 4294967296.0 : hi);
  return ((uint64_t)hu << 32) + (uint64_t)(uint32_t)lo;
}

}  // namespace fhei
