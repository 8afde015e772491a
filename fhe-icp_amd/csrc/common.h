// Device helpers shared by the kernels: modulus switch, gadget digits, block sums, test vectors.
// Part of libfheicp (one translation unit: fheicp.hip includes it).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include "prng.h"
#include "wave_fft.h"


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


// Test vector of a bootstrap, TV_j for j in [0, N), extended negacyclically:
// a staircase TV_j = base + (j >> shift) * step (step 0: a constant).
struct BrTv {
  u64 base, step;
  int shift;
};
// Table form (fhe_pbs_table_batch): 2^lut_bits boxes of 2^lut_log_box
// coefficients centred on the messages m * N / 2^lut_bits, TV_j = lut[m] *
// delta; the half box below 0 is the negacyclic image of the top half box, so
// a message-0 phase with negative noise still reads lut[0]. Only the v1/v2
// kernels take it: the hot v4 kernels keep the three-word argument (the
// wider one measured 2-3% slower at (23,1), tools/ab_lib2.sh).
struct BrTvLut {
  u64 base, step;
  int shift;
  int lut_log_box;
  int lut_count;
  const int64_t* lut;  // device, lut_count entries
  u64 delta;
};
__device__ __forceinline__ u64 tv_rot(const BrTv& tv, uint32_t idx, int N) {
  const uint32_t j = idx & (uint32_t)(N - 1);
  const u64 v = tv.base + (u64)(j >> tv.shift) * tv.step;
  return idx < (uint32_t)N ? v : (u64)0 - v;
}
__device__ __forceinline__ u64 tv_rot(const BrTvLut& tv, uint32_t idx, int N) {
  const uint32_t j = idx & (uint32_t)(N - 1);
  const uint32_t box = (j + (1u << (tv.lut_log_box - 1))) >> tv.lut_log_box;
  const u64 v = box < (uint32_t)tv.lut_count ? (u64)tv.lut[box] * tv.delta : (u64)0 - (u64)tv.lut[0] * tv.delta;
  return idx < (uint32_t)N ? v : (u64)0 - v;
}
// Output of one extracted LWE word x (word `pos` of ciphertext c):
//   mode 0: out = x
//   mode 1: sign-bit round: bit = trivial(tv.base) - x; ct_v -= bit;
//           refreshed += bit (if given); sign = bit (if given)
//   mode 2: digit round: ct_v -= x; refreshed += x (if given)
template <class TV>
__device__ __forceinline__ void br_emit(int mode, u64 x, bool body, const TV& tv, size_t pos, u64* out, u64* ct_v,
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
