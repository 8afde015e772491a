// Blind rotation v4 for N = 1024, k = 2: one wavefront per
// GLWE component, three per ciphertext, two ciphertexts per workgroup.
//
// Why this split: v2 divides every FFT between two waves, which costs a
// cross-wave LDS relayout (two barriers) per transform — 18 barriers per
// step — and leaves 2 waves per SIMD. Here a wave owns whole transforms
// (8 complex values per lane, S = 8): the 9 index bits live in 3 slot bits
// and 6 lane bits, and a transform needs three v_permlane swaps plus ONE
// relayout through the wave's own LDS slot (no barrier). The waves of a
// ciphertext meet only in the external product: each writes the FFT of its
// component's digit polynomial to LDS, and wave c accumulates output
// component c from all three (2 barriers per gadget level, 4 per step).
// 6 waves x 2 workgroups per CU = 3 waves per SIMD; the two ciphertexts of a
// workgroup stream the same BSK lines, so the second load hits L1.
//
// FFT layouts: positions [slot0, slot1, slot2, lane0..lane5] -> index bit.
//   forward  LA [8,7,6] -swap32,swap16-> LB [5,4] -lds-> LC [3,2,1] -swap32-> LD [0]
// (swap32 exchanges slot bit 1 with lane bit 5, swap16 slot bit 2 with lane
// bit 4, so LB holds index bits 8,7 in lane bits 4,5.)
//   inverse  the exact reverse, ending in LA (natural order: j = lane + 64*slot)
// The accumulator is kept in registers as the top 32 bits of each torus
// coefficient when L*beta <= 31 (ACC32), else as full u64.
#pragma once
#include "wave_fft.h"

namespace fhei {
namespace v4 {
using u64 = uint64_t;

constexpr int M = 512, N = 1024, S = 8, K = 2;
constexpr int G = 2;             // ciphertexts per workgroup
constexpr int WPC = K + 1;       // waves per ciphertext
constexpr int NT = 64 * G * WPC; // 384 threads
constexpr int NTW = 17;          // per-lane twiddle entries (forward stages 8..1)
constexpr int NMAX = 1023;       // max small-LWE dimension (LDS budget: 2 workgroups per CU)

struct Lay {
  int p[9];
};
constexpr Lay LAYS[4] = {{{6, 7, 8, 0, 1, 2, 3, 4, 5}},   // LA
                         {{6, 5, 4, 0, 1, 2, 3, 8, 7}},   // LB
                         {{1, 2, 3, 4, 5, 6, 7, 8, 0}},   // LC
                         {{1, 2, 0, 4, 5, 6, 7, 8, 3}}};  // LD
enum { LA = 0, LB = 1, LC = 2, LD = 3 };

__host__ __device__ constexpr int jof(int li, int lane, int u) {
  int j = 0;
  for (int b = 0; b < 3; ++b) j |= ((u >> b) & 1) << LAYS[li].p[b];
  for (int b = 0; b < 6; ++b) j |= ((lane >> b) & 1) << LAYS[li].p[3 + b];
  return j;
}

// LDS position of FFT index j in the relayout scratch: j + j/16 (one pad
// element per 16). Injective, additive in the lane and slot parts of j (one
// base register plus immediate offsets) and conflict-free: a ds_read_b128
// bank quad is the position mod 16 = (j + j/16) mod 16, so the 16-lane read
// groups (index bits 0..3 and 8 of LB, bits 4..8 of LC) and 8-lane write
// groups (bits 0..2 of LB, 4..6 of LC) land on distinct quads (bit 8 moves a
// position by 272 = 0 mod 16).
constexpr int SCR = M + M / 16;  // scratch elements per wave
__host__ __device__ constexpr int swz(int j) { return j + (j >> 4); }

// Twiddle entries: a DIF stage on slot bit sb of layout li works on index
// bit k = p[sb]; its twiddle W = exp(2 pi i (j mod 2^k) / 2^(k+1)) depends on
// the lane and on the slot bits mapped below k ("relevant" bits).
__host__ __device__ constexpr int stage_k(int li, int sb) { return LAYS[li].p[sb]; }
__host__ __device__ constexpr int n_rel(int li, int sb) {
  int c = 0;
  for (int b = 0; b < 3; ++b)
    if (b != sb && LAYS[li].p[b] < LAYS[li].p[sb]) ++c;
  return c;
}
// entry offset of pair base u within its stage
__host__ __device__ constexpr int ent(int li, int sb, int u) {
  int e = 0, c = 0;
  for (int b = 0; b < 3; ++b)
    if (b != sb && LAYS[li].p[b] < LAYS[li].p[sb]) e |= ((u >> b) & 1) << c++;
  return e;
}
// slot value u whose relevant bits encode entry e (inverse of ent)
__host__ __device__ constexpr int ent_u(int li, int sb, int e) {
  int u = 0, c = 0;
  for (int b = 0; b < 3; ++b)
    if (b != sb && LAYS[li].p[b] < LAYS[li].p[sb]) u |= ((e >> c++) & 1) << b;
  return u;
}
// forward stage list: (layout, slot bit); entry base offsets
constexpr int NST = 8;
constexpr int ST_L[NST] = {LA, LA, LA, LB, LB, LC, LC, LC};
constexpr int ST_B[NST] = {2, 1, 0, 1, 2, 2, 1, 0};
__host__ __device__ constexpr int st_e0(int s) {
  int e = 0;
  for (int t = 0; t < s; ++t) e += 1 << n_rel(ST_L[t], ST_B[t]);
  return e;
}
static_assert(st_e0(NST) == NTW, "twiddle entry count");

// Fill the per-workgroup LDS tables: twl[e][lane] (stage twiddles) and
// twt[u][lane] = twist[lane + 64 u] (the fold's w^j, natural layout).
__device__ __forceinline__ void fill_tables(c64* twl, c64* twt, const c64* __restrict__ tw,
                                            const c64* __restrict__ twist, int tid, int nthr) {
  for (int x = tid; x < NTW * 64; x += nthr) {
    const int e = x >> 6, lane = x & 63;
    int s = 0;
    while (s + 1 < NST && st_e0(s + 1) <= e) ++s;
    const int li = ST_L[s], sb = ST_B[s], k = stage_k(li, sb);
    const int u = ent_u(li, sb, e - st_e0(s));
    const int jm = jof(li, lane, u) & ((1 << k) - 1);
    twl[x] = tw[jm * ((M / 2) >> k)];
  }
  for (int x = tid; x < S * 64; x += nthr) twt[x] = twist[x];
}

// Workgroup barrier for LDS hand-offs only: retire this wave's LDS ops, then
// s_barrier. Outstanding global loads stay in flight across it (the compiler
// sees neither a fence nor a barrier it would drain them for).
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// ---- register-level pieces ---------------------------------------------
template <int SB>
__device__ __forceinline__ void swap32(c64 (&v)[S]) {
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int u = ((q >> SB) << (SB + 1)) | (q & ((1 << SB) - 1)), w = u | (1 << SB);
    uint64_t xr = __builtin_bit_cast(uint64_t, v[u].x), xi = __builtin_bit_cast(uint64_t, v[u].y);
    uint64_t yr = __builtin_bit_cast(uint64_t, v[w].x), yi = __builtin_bit_cast(uint64_t, v[w].y);
    auto a0 = __builtin_amdgcn_permlane32_swap((uint32_t)xr, (uint32_t)yr, false, false);
    auto a1 = __builtin_amdgcn_permlane32_swap((uint32_t)(xr >> 32), (uint32_t)(yr >> 32), false, false);
    auto b0 = __builtin_amdgcn_permlane32_swap((uint32_t)xi, (uint32_t)yi, false, false);
    auto b1 = __builtin_amdgcn_permlane32_swap((uint32_t)(xi >> 32), (uint32_t)(yi >> 32), false, false);
    v[u].x = __builtin_bit_cast(double, (uint64_t)a0[0] | ((uint64_t)a1[0] << 32));
    v[w].x = __builtin_bit_cast(double, (uint64_t)a0[1] | ((uint64_t)a1[1] << 32));
    v[u].y = __builtin_bit_cast(double, (uint64_t)b0[0] | ((uint64_t)b1[0] << 32));
    v[w].y = __builtin_bit_cast(double, (uint64_t)b0[1] | ((uint64_t)b1[1] << 32));
  }
}
template <int SB>
__device__ __forceinline__ void swap16(c64 (&v)[S]) {
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int u = ((q >> SB) << (SB + 1)) | (q & ((1 << SB) - 1)), w = u | (1 << SB);
    uint64_t xr = __builtin_bit_cast(uint64_t, v[u].x), xi = __builtin_bit_cast(uint64_t, v[u].y);
    uint64_t yr = __builtin_bit_cast(uint64_t, v[w].x), yi = __builtin_bit_cast(uint64_t, v[w].y);
    auto a0 = __builtin_amdgcn_permlane16_swap((uint32_t)xr, (uint32_t)yr, false, false);
    auto a1 = __builtin_amdgcn_permlane16_swap((uint32_t)(xr >> 32), (uint32_t)(yr >> 32), false, false);
    auto b0 = __builtin_amdgcn_permlane16_swap((uint32_t)xi, (uint32_t)yi, false, false);
    auto b1 = __builtin_amdgcn_permlane16_swap((uint32_t)(xi >> 32), (uint32_t)(yi >> 32), false, false);
    v[u].x = __builtin_bit_cast(double, (uint64_t)a0[0] | ((uint64_t)a1[0] << 32));
    v[w].x = __builtin_bit_cast(double, (uint64_t)a0[1] | ((uint64_t)a1[1] << 32));
    v[u].y = __builtin_bit_cast(double, (uint64_t)b0[0] | ((uint64_t)b1[0] << 32));
    v[w].y = __builtin_bit_cast(double, (uint64_t)b0[1] | ((uint64_t)b1[1] << 32));
  }
}

// DIF / DIT stage s of the forward list (twiddles from LDS); stage 0 of the
// transform (index bit 0, W = 1) is separate.
// DBG (timing experiments only, results wrong): bit 0 takes every twiddle
// from the register wf instead of LDS; bit 3 skips the relayout's LDS trip.
template <int ST, int DBG = 0>
__device__ __forceinline__ void dif(c64 (&v)[S], const c64* twl, int lane, c64 wf = {}) {
  constexpr int li = ST_L[ST], SB = ST_B[ST], E0 = st_e0(ST), NE = 1 << n_rel(li, SB);
  // the stage's distinct twiddles as one batch of LDS reads (one wait)
  c64 Wt[NE];
#pragma unroll
  for (int e = 0; e < NE; ++e) Wt[e] = (DBG & 1) ? wf : twl[(E0 + e) * 64 + lane];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int u = ((q >> SB) << (SB + 1)) | (q & ((1 << SB) - 1)), w = u | (1 << SB);
    const c64 W = Wt[ent(li, SB, u)];
    const c64 X = v[u], Y = v[w];
    v[u] = cadd(X, Y);
    v[w] = cmul(csub(X, Y), W);
  }
}
template <int ST, int DBG = 0>
__device__ __forceinline__ void dit(c64 (&v)[S], const c64* twl, int lane, c64 wf = {}) {
  constexpr int li = ST_L[ST], SB = ST_B[ST], E0 = st_e0(ST), NE = 1 << n_rel(li, SB);
  // the stage's distinct twiddles as one batch of LDS reads (one wait)
  c64 Wt[NE];
#pragma unroll
  for (int e = 0; e < NE; ++e) Wt[e] = (DBG & 1) ? wf : twl[(E0 + e) * 64 + lane];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int u = ((q >> SB) << (SB + 1)) | (q & ((1 << SB) - 1)), w = u | (1 << SB);
    const c64 W = Wt[ent(li, SB, u)];
    const c64 X = v[u], Y = cmulc(v[w], W);
    v[u] = cadd(X, Y);
    v[w] = csub(X, Y);
  }
}
// index bit 0 on slot bit 2 of LD: W = 1
__device__ __forceinline__ void bfly0(c64 (&v)[S]) {
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const c64 X = v[u], Y = v[u + 4];
    v[u] = cadd(X, Y);
    v[u + 4] = csub(X, Y);
  }
}

// wave-local relayout through the wave's own scratch (no barrier)
template <int LS, int LT, int DBG = 0>
__device__ __forceinline__ void relayout(c64 (&v)[S], c64* scr, int lane) {
  if constexpr ((DBG & 8) != 0) return;
#pragma unroll
  for (int u = 0; u < S; ++u) scr[swz(jof(LS, lane, u))] = v[u];
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
  for (int u = 0; u < S; ++u) v[u] = scr[swz(jof(LT, lane, u))];
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
}

// natural order (LA) -> LD
template <int DBG = 0>
__device__ __forceinline__ void forward(c64 (&v)[S], const c64* twl, c64* scr, int lane, c64 wf = {}) {
  dif<0, DBG>(v, twl, lane, wf);
  dif<1, DBG>(v, twl, lane, wf);
  dif<2, DBG>(v, twl, lane, wf);
  swap32<1>(v);
  swap16<2>(v);
  dif<3, DBG>(v, twl, lane, wf);
  dif<4, DBG>(v, twl, lane, wf);
  relayout<LB, LC, DBG>(v, scr, lane);
  dif<5, DBG>(v, twl, lane, wf);
  dif<6, DBG>(v, twl, lane, wf);
  dif<7, DBG>(v, twl, lane, wf);
  swap32<2>(v);
  bfly0(v);
}
// LD -> natural order (LA), times M
template <int DBG = 0>
__device__ __forceinline__ void inverse(c64 (&v)[S], const c64* twl, c64* scr, int lane, c64 wf = {}) {
  bfly0(v);
  swap32<2>(v);
  dit<7, DBG>(v, twl, lane, wf);
  dit<6, DBG>(v, twl, lane, wf);
  dit<5, DBG>(v, twl, lane, wf);
  relayout<LC, LB, DBG>(v, scr, lane);
  dit<4, DBG>(v, twl, lane, wf);
  dit<3, DBG>(v, twl, lane, wf);
  swap16<2>(v);
  swap32<1>(v);
  dit<2, DBG>(v, twl, lane, wf);
  dit<1, DBG>(v, twl, lane, wf);
  dit<0, DBG>(v, twl, lane, wf);
}

// ---- accumulator word type ------------------------------------------------
template <bool A32>
struct Acc;
template <>
struct Acc<true> {
  using T = uint32_t;
  static __device__ __forceinline__ T from64(u64 x) { return (T)((x + (1ull << 31)) >> 32); }
  static __device__ __forceinline__ u64 to64(T x) { return (u64)x << 32; }
  // round(z / 2^32) mod 2^32 via a magic number: z/2^32 + 1.5*2^55 has an
  // ulp of 8, so its low mantissa word is round(z / 2^35) mod 2^32 for
  // |z| < 2^86 (the product sums here stay below 2^85). The 3 dropped bits
  // add noise far below sigma_pbs.
  static __device__ __forceinline__ T from_f64(double z) {
    const double t = __fma_rn(z, 1.0 / 4294967296.0, 54043195528445952.0);
    return (T)(uint32_t)__builtin_bit_cast(uint64_t, t) << 3;
  }
};
template <>
struct Acc<false> {
  using T = u64;
  static __device__ __forceinline__ T from64(u64 x) { return x; }
  static __device__ __forceinline__ u64 to64(T x) { return x; }
  static __device__ __forceinline__ T from_f64(double z) { return f64_to_torus(z); }
};

}  // namespace v4
}  // namespace fhei
