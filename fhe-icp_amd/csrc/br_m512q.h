// Blind rotation v3 for N = 1024 (M = 512 complex points): FOUR wavefronts
// per ciphertext, S = 2 complex values per lane.
//
// v2 (br_m512.h) runs 2 waves per SIMD at a 1024-ciphertext batch and sits
// near 40% f64-pipe utilisation: there is not enough independent work per
// SIMD to cover f64 and LDS latency. Four waves per ciphertext with <= 128
// VGPRs give 4 waves per SIMD at the same batch.
//
// Positions of the 9 FFT index bits: [slot0, lane0..lane5, wave0, wave1].
// One phase processes 3 bits without LDS: a radix-2 stage on slot0, then
// v_permlane32_swap (slot0 <-> lane5) and v_permlane16_swap (slot0 <->
// lane4) each bring a new bit into the slot. 3 phases, 2 relayouts:
//   forward  A[8] s32 [7] s16 [6] -wave-local-> B[5] s32 [4] s16 [3] -cross-> C[2] s32 [1] s16 [0]
//   inverse  the exact reverse, ending in layout A (coefficient layout).
// A and B keep the wave bits {0, 1} (the A<->B relayout stays inside each
// wave's quarter of the scratch); C uses wave bits {7, 8}.
#pragma once
#include "wave_fft.h"

namespace fhei {
namespace m512q {

constexpr int M = 512, N = 1024, S = 2, NT = 256;
constexpr int LDS_STRIDE = M;  // c64 elements of scratch per polynomial (no padding)
constexpr int NF_MAX = 2;      // polynomials transformed jointly (scratch = NF_MAX * 8 KB)
// XOR swizzle of the scratch index: low 3 bits ^= bits 3-5 ^ bits 6-8. A
// bijection inside each group of 8 elements; simulated over the gfx950
// ds_write_b128 / ds_read_b128 lane groups for every relayout pattern below
// it leaves at most 2-way bank conflicts (the 1-in-8 pad leaves 4-way) and
// needs no extra LDS, which keeps the workgroup at 40 KB = 4 per CU.
__device__ __forceinline__ int swz(int j) { return j ^ ((j >> 3) & 7) ^ ((j >> 6) & 7); }

struct Lay {
  int p[9];  // [slot0, lane0..lane5, wave0, wave1] -> index bit
};
constexpr Lay LA = {{8, 2, 3, 4, 5, 6, 7, 0, 1}};
constexpr Lay LA1 = {{7, 2, 3, 4, 5, 6, 8, 0, 1}};
constexpr Lay LA2 = {{6, 2, 3, 4, 5, 7, 8, 0, 1}};
constexpr Lay LB = {{5, 2, 6, 7, 8, 3, 4, 0, 1}};
constexpr Lay LB1 = {{4, 2, 6, 7, 8, 3, 5, 0, 1}};
constexpr Lay LB2 = {{3, 2, 6, 7, 8, 4, 5, 0, 1}};
constexpr Lay LC = {{2, 3, 4, 5, 6, 0, 1, 7, 8}};
constexpr Lay LC1 = {{1, 3, 4, 5, 6, 0, 2, 7, 8}};
constexpr Lay LC2 = {{0, 3, 4, 5, 6, 1, 2, 7, 8}};

__device__ __forceinline__ int jof(const Lay& L, int tid, int u) {
  const int lane = tid & 63, wave = tid >> 6;
  int j = (u << L.p[0]) | ((wave & 1) << L.p[7]) | ((wave >> 1) << L.p[8]);
#pragma unroll
  for (int b = 0; b < 6; ++b) j |= ((lane >> b) & 1) << L.p[1 + b];
  return j;
}

__device__ __forceinline__ uint64_t bits(double d) { return __builtin_bit_cast(uint64_t, d); }
__device__ __forceinline__ double dbl(uint32_t lo, uint32_t hi) {
  return __builtin_bit_cast(double, (uint64_t)lo | ((uint64_t)hi << 32));
}

// v_permlane32_swap: lanes 32-63 of x <-> lanes 0-31 of y (slot0 <-> lane5)
__device__ __forceinline__ void swap32(c64 (&v)[S]) {
  const uint64_t xr = bits(v[0].x), xi = bits(v[0].y), yr = bits(v[1].x), yi = bits(v[1].y);
  auto a0 = __builtin_amdgcn_permlane32_swap((uint32_t)xr, (uint32_t)yr, false, false);
  auto a1 = __builtin_amdgcn_permlane32_swap((uint32_t)(xr >> 32), (uint32_t)(yr >> 32), false, false);
  auto b0 = __builtin_amdgcn_permlane32_swap((uint32_t)xi, (uint32_t)yi, false, false);
  auto b1 = __builtin_amdgcn_permlane32_swap((uint32_t)(xi >> 32), (uint32_t)(yi >> 32), false, false);
  v[0] = {dbl(a0[0], a1[0]), dbl(b0[0], b1[0])};
  v[1] = {dbl(a0[1], a1[1]), dbl(b0[1], b1[1])};
}
// v_permlane16_swap: odd 16-lane rows of x <-> even rows of y (slot0 <-> lane4)
__device__ __forceinline__ void swap16(c64 (&v)[S]) {
  const uint64_t xr = bits(v[0].x), xi = bits(v[0].y), yr = bits(v[1].x), yi = bits(v[1].y);
  auto a0 = __builtin_amdgcn_permlane16_swap((uint32_t)xr, (uint32_t)yr, false, false);
  auto a1 = __builtin_amdgcn_permlane16_swap((uint32_t)(xr >> 32), (uint32_t)(yr >> 32), false, false);
  auto b0 = __builtin_amdgcn_permlane16_swap((uint32_t)xi, (uint32_t)yi, false, false);
  auto b1 = __builtin_amdgcn_permlane16_swap((uint32_t)(xi >> 32), (uint32_t)(yi >> 32), false, false);
  v[0] = {dbl(a0[0], a1[0]), dbl(b0[0], b1[0])};
  v[1] = {dbl(a0[1], a1[1]), dbl(b0[1], b1[1])};
}

// All transforms below operate on NF independent polynomials at once: each
// stage is applied to all of them before the next, which gives the f64
// pipe NF independent dependency chains per lane and lets the NF transforms
// share every relayout (and its barriers).
template <int NF>
__device__ __forceinline__ void write_lay(const c64 (&v)[NF][S], const Lay& A, c64* lds, int tid) {
#pragma unroll
  for (int f = 0; f < NF; ++f)
#pragma unroll
    for (int u = 0; u < S; ++u) lds[f * LDS_STRIDE + swz(jof(A, tid, u))] = v[f][u];
}
template <int NF>
__device__ __forceinline__ void read_lay(c64 (&v)[NF][S], const Lay& B, const c64* lds, int tid) {
#pragma unroll
  for (int f = 0; f < NF; ++f)
#pragma unroll
    for (int u = 0; u < S; ++u) v[f][u] = lds[f * LDS_STRIDE + swz(jof(B, tid, u))];
}
// Inside one wave's quarter of the scratch (layouts share the wave bits).
template <int NF>
__device__ __forceinline__ void relayout_wave(c64 (&v)[NF][S], const Lay& A, const Lay& B, c64* lds, int tid) {
  write_lay<NF>(v, A, lds, tid);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  read_lay<NF>(v, B, lds, tid);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
}
// Across waves. Writes touch the writer's {0,1}-quarter (B side) or
// {7,8}-quarter (C side) and reads the other quarter system, so a barrier
// separates writes from reads and a trailing barrier keeps the next
// wave-local relayout from overwriting positions another wave still reads.
template <int NF>
__device__ __forceinline__ void relayout_cross(c64 (&v)[NF][S], const Lay& A, const Lay& B, c64* lds, int tid) {
  write_lay<NF>(v, A, lds, tid);
  __syncthreads();
  read_lay<NF>(v, B, lds, tid);
  __syncthreads();
}
static_assert(LA2.p[7] == LB.p[7] && LA2.p[8] == LB.p[8], "A <-> B must keep the wave bits");

struct Tw {
  c64 w[9];
};
__device__ __forceinline__ c64 stage_tw(const Lay& L, const c64* __restrict__ tw, int tid) {
  const int k = L.p[0], h = 1 << k;
  const int jm = jof(L, tid, 0) & (h - 1);
  return tw[jm * (M / 2 / h)];
}
__device__ __forceinline__ void load_twiddles(Tw& T, const c64* __restrict__ tw, int tid) {
  T.w[8] = stage_tw(LA, tw, tid);
  T.w[7] = stage_tw(LA1, tw, tid);
  T.w[6] = stage_tw(LA2, tw, tid);
  T.w[5] = stage_tw(LB, tw, tid);
  T.w[4] = stage_tw(LB1, tw, tid);
  T.w[3] = stage_tw(LB2, tw, tid);
  T.w[2] = stage_tw(LC, tw, tid);
  T.w[1] = stage_tw(LC1, tw, tid);
  T.w[0] = {1.0, 0.0};
}

template <int NF>
__device__ __forceinline__ void dif(c64 (&v)[NF][S], c64 W) {
#pragma unroll
  for (int f = 0; f < NF; ++f) {
    const c64 X = v[f][0], Y = v[f][1];
    v[f][0] = cadd(X, Y);
    v[f][1] = cmul(csub(X, Y), W);
  }
}
template <int NF>
__device__ __forceinline__ void dif1(c64 (&v)[NF][S]) {  // W = 1 (also its own inverse)
#pragma unroll
  for (int f = 0; f < NF; ++f) {
    const c64 X = v[f][0], Y = v[f][1];
    v[f][0] = cadd(X, Y);
    v[f][1] = csub(X, Y);
  }
}
template <int NF>
__device__ __forceinline__ void dit(c64 (&v)[NF][S], c64 W) {
#pragma unroll
  for (int f = 0; f < NF; ++f) {
    const c64 X = v[f][0], Y = cmulc(v[f][1], W);
    v[f][0] = cadd(X, Y);
    v[f][1] = csub(X, Y);
  }
}
template <int NF>
__device__ __forceinline__ void swap32n(c64 (&v)[NF][S]) {
#pragma unroll
  for (int f = 0; f < NF; ++f) swap32(v[f]);
}
template <int NF>
__device__ __forceinline__ void swap16n(c64 (&v)[NF][S]) {
#pragma unroll
  for (int f = 0; f < NF; ++f) swap16(v[f]);
}

template <int NF>
__device__ __forceinline__ void forward(c64 (&v)[NF][S], const Tw& T, c64* lds, int tid) {
  dif<NF>(v, T.w[8]);
  swap32n<NF>(v);
  dif<NF>(v, T.w[7]);
  swap16n<NF>(v);
  dif<NF>(v, T.w[6]);
  relayout_wave<NF>(v, LA2, LB, lds, tid);
  dif<NF>(v, T.w[5]);
  swap32n<NF>(v);
  dif<NF>(v, T.w[4]);
  swap16n<NF>(v);
  dif<NF>(v, T.w[3]);
  relayout_cross<NF>(v, LB2, LC, lds, tid);
  dif<NF>(v, T.w[2]);
  swap32n<NF>(v);
  dif<NF>(v, T.w[1]);
  swap16n<NF>(v);
  dif1<NF>(v);
}

template <int NF>
__device__ __forceinline__ void inverse(c64 (&v)[NF][S], const Tw& T, c64* lds, int tid) {
  dif1<NF>(v);
  swap16n<NF>(v);
  dit<NF>(v, T.w[1]);
  swap32n<NF>(v);
  dit<NF>(v, T.w[2]);
  relayout_cross<NF>(v, LC, LB2, lds, tid);
  dit<NF>(v, T.w[3]);
  swap16n<NF>(v);
  dit<NF>(v, T.w[4]);
  swap32n<NF>(v);
  dit<NF>(v, T.w[5]);
  relayout_wave<NF>(v, LB, LA2, lds, tid);
  dit<NF>(v, T.w[6]);
  swap16n<NF>(v);
  dit<NF>(v, T.w[7]);
  swap32n<NF>(v);
  dit<NF>(v, T.w[8]);
}

__device__ __forceinline__ int tcoef(int tid, int u) { return jof(LA, tid, u); }
__device__ __forceinline__ int fslot(int tid, int u) { return u * NT + tid; }

}  // namespace m512q

// Adapter used by the templated blind-rotation kernel (fheicp.hip).
struct V3 {
  static constexpr int M = m512q::M, N = m512q::N, S = m512q::S, NT = m512q::NT;
  using Tw = m512q::Tw;
  __device__ static void load_twiddles(Tw& T, const c64* tw, int tid) { m512q::load_twiddles(T, tw, tid); }
  static constexpr bool MULTI = true;  // forward/inverse take [NF][S]
  static constexpr int SCRATCH = m512q::NF_MAX * m512q::LDS_STRIDE;
  template <int NF>
  __device__ static void forward(c64 (&v)[NF][S], const Tw& T, c64* lds, int tid) { m512q::forward<NF>(v, T, lds, tid); }
  template <int NF>
  __device__ static void inverse(c64 (&v)[NF][S], const Tw& T, c64* lds, int tid) { m512q::inverse<NF>(v, T, lds, tid); }
  __device__ static int tcoef(int tid, int u) { return m512q::tcoef(tid, u); }
  __device__ static int fslot(int tid, int u) { return m512q::fslot(tid, u); }
};

}  // namespace fhei
