// Blind rotation v2 for N = 1024 (M = 512 complex points): TWO wavefronts
// per ciphertext, S = 4 complex values per lane.
//
// Why: with one wave per ciphertext the accumulator (LDS) and the
// external-product partial sums (VGPRs) allow one wave per SIMD at a
// 1024-ciphertext batch, and rocprof showed 68% of wave-cycles parked in
// s_waitcnt/barriers (profiles/r01_v1_pmc). Splitting a ciphertext over
// two waves halves the per-lane state, so two waves share every SIMD.
//
// FFT index bits (9) live in 2 slot bits, 6 lane bits and 1 wave bit. A
// layout maps each position to an index bit. Radix-2 stages run on slot
// bits in registers; v_permlane32_swap exchanges slot bit 1 with lane bit 5
// (a pure-VALU index-bit transposition), and an LDS relayout moves bits
// between waves. Per FFT: 9 stages, 3 swaps, 2 LDS relayouts (one across
// the two waves with 2 barriers, one inside each wave with none).
//   forward  LA[8,7] -swap-> LAs[6] -lds-> LB[5,4] -swap-> LBs[3] -lds-> LC[2,1] -swap-> LCs[0]
//   inverse  the exact reverse, ending in LA (the coefficient layout).
#pragma once
#include "wave_fft.h"

namespace fhei {
namespace m512 {

constexpr int M = 512, N = 1024, S = 4, NT = 128;

// position -> index bit: [slot0, slot1, lane0..lane5, wave]
struct Lay {
  int p[9];
};
constexpr Lay LA = {{7, 8, 0, 1, 2, 3, 4, 6, 5}};
constexpr Lay LAs = {{7, 6, 0, 1, 2, 3, 4, 8, 5}};
constexpr Lay LB = {{4, 5, 0, 1, 2, 6, 7, 3, 8}};
constexpr Lay LBs = {{4, 3, 0, 1, 2, 6, 7, 5, 8}};
constexpr Lay LC = {{1, 2, 3, 4, 5, 6, 7, 0, 8}};
constexpr Lay LCs = {{1, 0, 3, 4, 5, 6, 7, 2, 8}};

__device__ __forceinline__ int jof(const Lay& L, int tid, int u) {
  const int lane = tid & 63, wave = tid >> 6;
  int j = ((u & 1) << L.p[0]) | (((u >> 1) & 1) << L.p[1]) | (wave << L.p[8]);
#pragma unroll
  for (int b = 0; b < 6; ++b) j |= ((lane >> b) & 1) << L.p[2 + b];
  return j;
}

// swap slot bit 1 with lane bit 5 for the pairs (u, u|2)
__device__ __forceinline__ void swap32(c64 (&v)[S]) {
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    c64& x = v[u];
    c64& y = v[u | 2];
    const uint64_t xr = __builtin_bit_cast(uint64_t, x.x), xi = __builtin_bit_cast(uint64_t, x.y);
    const uint64_t yr = __builtin_bit_cast(uint64_t, y.x), yi = __builtin_bit_cast(uint64_t, y.y);
    auto a0 = __builtin_amdgcn_permlane32_swap((uint32_t)xr, (uint32_t)yr, false, false);
    auto a1 = __builtin_amdgcn_permlane32_swap((uint32_t)(xr >> 32), (uint32_t)(yr >> 32), false, false);
    auto b0 = __builtin_amdgcn_permlane32_swap((uint32_t)xi, (uint32_t)yi, false, false);
    auto b1 = __builtin_amdgcn_permlane32_swap((uint32_t)(xi >> 32), (uint32_t)(yi >> 32), false, false);
    x.x = __builtin_bit_cast(double, (uint64_t)a0[0] | ((uint64_t)a1[0] << 32));
    y.x = __builtin_bit_cast(double, (uint64_t)a0[1] | ((uint64_t)a1[1] << 32));
    x.y = __builtin_bit_cast(double, (uint64_t)b0[0] | ((uint64_t)b1[0] << 32));
    y.y = __builtin_bit_cast(double, (uint64_t)b0[1] | ((uint64_t)b1[1] << 32));
  }
}

// LDS relayouts. Scratch hazards: a cross-wave relayout
// writes or reads positions of BOTH waves' halves (split by index bit 8 in
// LB/LBs/LC); a wave-local one only touches its own half. Barrier placement:
//  - forward cross relayout (LAs -> LB): barrier BEFORE the writes (the
//    other wave may still be reading its half from the previous FFT's
//    wave-local relayout), writes, barrier, then reads of its own half;
//  - inverse cross relayout (LB -> LAs): writes of its own half, barrier,
//    reads across both halves, barrier AFTER (the next wave-local relayout
//    writes into a half the other wave may still be reading).
__device__ __forceinline__ void write_lay(const c64 (&v)[S], const Lay& A, c64* lds, int tid) {
#pragma unroll
  for (int u = 0; u < S; ++u) lds[lds_pad(jof(A, tid, u))] = v[u];
}
__device__ __forceinline__ void read_lay(c64 (&v)[S], const Lay& B, const c64* lds, int tid) {
#pragma unroll
  for (int u = 0; u < S; ++u) v[u] = lds[lds_pad(jof(B, tid, u))];
}
__device__ __forceinline__ void relayout_fwd(c64 (&v)[S], const Lay& A, const Lay& B, c64* lds, int tid) {
  __syncthreads();
  write_lay(v, A, lds, tid);
  __syncthreads();
  read_lay(v, B, lds, tid);
}
__device__ __forceinline__ void relayout_inv(c64 (&v)[S], const Lay& A, const Lay& B, c64* lds, int tid) {
  write_lay(v, A, lds, tid);
  __syncthreads();
  read_lay(v, B, lds, tid);
  __syncthreads();
}
// Relayout inside one wave's half (same wave bit in both layouts): no
// workgroup barrier. lgkmcnt(0) retires the wave's LDS writes before its
// reads; the asm statements also pin the compiler's order.
__device__ __forceinline__ void relayout_wave(c64 (&v)[S], const Lay& A, const Lay& B, c64* lds, int tid) {
  write_lay(v, A, lds, tid);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  read_lay(v, B, lds, tid);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
}
static_assert(LB.p[8] == 8 && LBs.p[8] == 8 && LC.p[8] == 8, "wave halves must be split by index bit 8");
static_assert(LBs.p[8] == LC.p[8], "LBs <-> LC must keep the wave bit");

// Per-lane twiddles for the 9 stages, 2 butterflies each (loaded once).
// Stage on slot bit sb of layout L at index bit k: butterflies (u, u|1<<sb)
// for the two u with that bit clear; W = exp(2 pi i (j mod 2^k) / 2^(k+1)).
struct Tw {
  c64 w[9][2];
};
__device__ __forceinline__ void stage_tw(Tw& T, const Lay& L, int sb, const c64* __restrict__ tw, int tid) {
  const int k = L.p[sb];
  const int h = 1 << k;
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int u = sb == 1 ? q : (q << 1);  // u with bit sb clear
    const int jm = jof(L, tid, u) & (h - 1);
    T.w[k][q] = tw[jm * (M / 2 / h)];
  }
}
__device__ __forceinline__ void load_twiddles(Tw& T, const c64* __restrict__ tw, int tid) {
  stage_tw(T, LA, 1, tw, tid);   // 8
  stage_tw(T, LA, 0, tw, tid);   // 7
  stage_tw(T, LAs, 1, tw, tid);  // 6
  stage_tw(T, LB, 1, tw, tid);   // 5
  stage_tw(T, LB, 0, tw, tid);   // 4
  stage_tw(T, LBs, 1, tw, tid);  // 3
  stage_tw(T, LC, 1, tw, tid);   // 2
  stage_tw(T, LC, 0, tw, tid);   // 1
  stage_tw(T, LCs, 1, tw, tid);  // 0
}

template <int SB>
__device__ __forceinline__ void dif(c64 (&v)[S], const c64 (&W)[2]) {
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int u = SB == 1 ? q : (q << 1), w = u | (1 << SB);
    const c64 X = v[u], Y = v[w];
    v[u] = cadd(X, Y);
    v[w] = cmul(csub(X, Y), W[q]);
  }
}
template <int SB>
__device__ __forceinline__ void dit(c64 (&v)[S], const c64 (&W)[2]) {
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int u = SB == 1 ? q : (q << 1), w = u | (1 << SB);
    const c64 X = v[u], Y = cmulc(v[w], W[q]);
    v[u] = cadd(X, Y);
    v[w] = csub(X, Y);
  }
}

// natural order (layout LA) -> bit-reversed-by-layout (LCs)
__device__ __forceinline__ void forward(c64 (&v)[S], const Tw& T, c64* lds, int tid) {
  dif<1>(v, T.w[8]);
  dif<0>(v, T.w[7]);
  swap32(v);
  dif<1>(v, T.w[6]);
  relayout_fwd(v, LAs, LB, lds, tid);
  dif<1>(v, T.w[5]);
  dif<0>(v, T.w[4]);
  swap32(v);
  dif<1>(v, T.w[3]);
  relayout_wave(v, LBs, LC, lds, tid);
  dif<1>(v, T.w[2]);
  dif<0>(v, T.w[1]);
  swap32(v);
  // stage 0: W = exp(0) = 1
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const c64 X = v[q], Y = v[q | 2];
    v[q] = cadd(X, Y);
    v[q | 2] = csub(X, Y);
  }
}

// LCs -> LA, times M
__device__ __forceinline__ void inverse(c64 (&v)[S], const Tw& T, c64* lds, int tid) {
#pragma unroll
  for (int q = 0; q < 2; ++q) {  // stage 0: W = 1
    const c64 X = v[q], Y = v[q | 2];
    v[q] = cadd(X, Y);
    v[q | 2] = csub(X, Y);
  }
  swap32(v);
  dit<0>(v, T.w[1]);
  dit<1>(v, T.w[2]);
  relayout_wave(v, LC, LBs, lds, tid);
  dit<1>(v, T.w[3]);
  swap32(v);
  dit<0>(v, T.w[4]);
  dit<1>(v, T.w[5]);
  relayout_inv(v, LB, LAs, lds, tid);
  dit<1>(v, T.w[6]);
  swap32(v);
  dit<0>(v, T.w[7]);
  dit<1>(v, T.w[8]);
}

// coefficient index (of the first half, t < M) held by (tid, slot u) in LA
__device__ __forceinline__ int tcoef(int tid, int u) { return jof(LA, tid, u); }
// FFT-domain storage index of (tid, slot u) in LCs: [u][tid], coalesced
__device__ __forceinline__ int fslot(int tid, int u) { return u * NT + tid; }

}  // namespace m512

// Adapter used by the templated blind-rotation kernel (fheicp.hip).
struct V2 {
  static constexpr int M = m512::M, N = m512::N, S = m512::S, NT = m512::NT;
  static constexpr bool MULTI = false;
  static constexpr int SCRATCH = m512::M + m512::M / 8;
  using Tw = m512::Tw;
  __device__ static void load_twiddles(Tw& T, const c64* tw, int tid) { m512::load_twiddles(T, tw, tid); }
  __device__ static void forward(c64 (&v)[S], const Tw& T, c64* lds, int tid) { m512::forward(v, T, lds, tid); }
  __device__ static void inverse(c64 (&v)[S], const Tw& T, c64* lds, int tid) { m512::inverse(v, T, lds, tid); }
  __device__ static int tcoef(int tid, int u) { return m512::tcoef(tid, u); }
  __device__ static int fslot(int tid, int u) { return m512::fslot(tid, u); }
};

}  // namespace fhei
