// Blind rotation v4 for N = 1024, k = 2: one wavefront per
// GLWE component, three per ciphertext, two ciphertexts per workgroup.
//
// Why this split: v2 divides every FFT between two waves, which costs a
// cross-wave LDS relayout (two barriers) per transform — 18 barriers per
// step — and leaves 2 waves per SIMD. Here a wave owns whole transforms
// (8 complex values per lane, S = 8): the 9 index bits live in 3 slot bits
// and 6 lane bits; a transform is three radix-8 passes joined by two
// relayouts through the wave's own LDS slot (no barrier). The waves of a
// ciphertext meet only in the external product: each writes the FFT of its
// component's digit polynomial to LDS, and wave c accumulates output
// component c from all three (2 barriers per gadget level, 4 per step).
// 6 waves x 2 workgroups per CU = 3 waves per SIMD; the two ciphertexts of a
// workgroup stream the same BSK lines, so the second load hits L1.
//
// FFT: forward LA [8,7,6] -lds-> LB [5,4,3] -lds-> LC [2,1,0]; the inverse
// is the exact reverse, ending in LA (natural order: j = lane + 64*slot).
// The accumulator is kept in registers as the top 32 bits of each torus
// coefficient when L*beta <= 31 (ACC32), else as full u64.
#pragma once
#include "wave_fft.h"

namespace fhei {
namespace v4 {
using u64 = uint64_t;

constexpr int M = 512, N = 1024, S = 8, K = 2;
constexpr int WPC = K + 1;       // waves per ciphertext
// ciphertexts per workgroup: G2 = 2 (384 threads, 2 workgroups per CU) or 1
// (192 threads, 4 workgroups per CU: barriers join only one ciphertext's waves)
constexpr int nthreads(int G) { return 64 * G * WPC; }
constexpr int NTA = 8 * 64;      // pass A twiddles: 8 per lane (twist merged)
constexpr int NTB = 7 * 8;       // pass B twiddles: 7 per value of the 3 index bits below the pass
constexpr int NTW = NTA + NTB;   // LDS twiddle table entries (9 KB)
constexpr int NMAX = 1023;       // max small-LWE dimension (LDS budget: 2 workgroups per CU)
constexpr int SCR = 576;         // relayout scratch elements per wave (positions < 573)

// Transform = three radix-8 passes over index bits (8,7,6), (5,4,3), (2,1,0).
// A pass runs a constant DFT-8 network on its 3 slot bits (internal
// twiddles are 8th roots of unity) and then multiplies element u by the lane
// twiddle exp(2 pi i L m / 2^(p0+3)), m = bitrev3(u), L = index bits below
// the pass (the lane-dependent parts of all radix-2 DIF twiddles of the pass,
// deferred to its end). Pass C has L = 0. Two wave-local LDS relayouts move
// the slot bits; there are no lane permutes.
// Layouts: positions [slot0, slot1, slot2, lane0..lane5] -> index bit.
struct Lay {
  int p[9];
};
constexpr Lay LAYS[3] = {{{6, 7, 8, 0, 1, 2, 3, 4, 5}},   // LA: natural, j = lane + 64 u
                         {{3, 4, 5, 0, 1, 2, 6, 7, 8}},   // LB: LA with slot bits k <-> lane bits 3 + k
                         {{0, 1, 2, 4, 5, 8, 3, 6, 7}}};  // LC: transform output
enum { LA = 0, LB = 1, LC = 2 };

__host__ __device__ constexpr int jof(int li, int lane, int u) {
  int j = 0;
  for (int b = 0; b < 3; ++b) j |= ((u >> b) & 1) << LAYS[li].p[b];
  for (int b = 0; b < 6; ++b) j |= ((lane >> b) & 1) << LAYS[li].p[3 + b];
  return j;
}

// Scratch position of index j for each relayout: j + sum_k c_k * bit_{4+k}(j)
// (c superincreasing -> injective; additive in the lane and slot parts, so
// one base register plus immediate offsets). The offsets were searched so
// that the 8-lane ds_write_b128 groups of the source layout and the 16-lane
// ds_read_b128 groups of the target layout hit distinct bank quads.
// LA <-> LB is not an LDS relayout any more: it exchanges the slot bits with
// lane bits 3..5 in registers (swap_lb below); only LB <-> LC goes through
// LDS (offsets from tools/search_relayout.py --lb 0,1,2,6,7,8).
// FHEICP_ABLDS = 1: LA <-> LB through the slot too (R1F / R1I, offsets from
// tools/search_relayout.py; the identity is conflict-free for LB -> LA)
// instead of the permlane / DPP swaps (8.3 and 4.2 SIMD cycles per
// instruction, tools/xlane_probe.hip: 32 + 32 per transform)
#ifndef FHEICP_ABLDS
#define FHEICP_ABLDS 0
#endif
enum { R2F = 0, R2I = 1, R1F = 2, R1I = 3 };  // LB->LC, LC->LB, LA->LB, LB->LA
constexpr int RC[4][5] = {{1, 2, 4, 7, 16}, {2, 4, 8, 16, 31}, {2, 4, 8, 16, 30}, {0, 0, 0, 0, 0}};
__host__ __device__ constexpr int rpos(int r, int j) {
  int p = j;
  for (int k = 0; k < 5; ++k) p += RC[r][k] * ((j >> (4 + k)) & 1);
  return p;
}

__host__ __device__ constexpr int bitrev3(int u) { return ((u & 1) << 2) | (u & 2) | ((u >> 2) & 1); }

// Twiddles, computed on the host in long double (fhe_ctx_create) and copied
// to LDS per workgroup:
//   twl[m * 64 + lane] (m = 0..7): pass A, w^lane * exp(2 pi i lane m / 512)
//        — the lane part w^lane of the fold twist w^(lane + 64 u)
//        (w = exp(i pi / N)) commutes with pass A's DFT-8 and merges into
//        its lane twiddles;
//   twl[NTA + (m - 1) * 8 + L] (m = 1..7): pass B, exp(2 pi i L m / 64),
//        L = index bits 0..2 of the lane in layout LB (lanes sharing L read
//        one address: an LDS broadcast).
// The slot part w^(64 u) = exp(i pi u / 16) is a compile-time constant (fold8).
__host__ __device__ constexpr int lb_low3(int lane) { return jof(1, lane, 0) & 7; }
__device__ __forceinline__ void fill_tables(c64* twl, const c64* __restrict__ tw4, int tid, int nthr) {
  for (int x = tid; x < NTW; x += nthr) twl[x] = tw4[x];
}

// Workgroup barrier for LDS hand-offs only: retire this wave's LDS ops, then
// s_barrier. Outstanding global loads stay in flight across it (the compiler
// sees neither a fence nor a barrier it would drain them for).
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// Per-ciphertext hand-offs without s_barrier (FL kernels): the three waves of
// a ciphertext count their F writes (W) and their reads of the others' F (R)
// in two LDS words. One wave's DS operations are performed in order, so a
// count added after a wave's F writes (or after its reads) is observed only
// once those have been performed; the compiler is kept from moving LDS
// accesses across the add and the poll by "memory" clobbers. Outstanding
// global loads are not waited for. Ciphertexts of a workgroup never wait for
// each other, unlike s_barrier.
// Both are inline asm so that no divergent branch or loop appears in the
// compiler's CFG (a divergent `if (lane == 0)` there made the allocator
// spill the prefetched BSK rows).
__device__ __forceinline__ uint32_t lds_addr(const void* p) { return (uint32_t)(uintptr_t)p; }
__device__ __forceinline__ void ct_signal(uint32_t* f) {
  uint64_t saved;
  asm volatile(
      "s_mov_b64 %0, exec\n\t"
      "s_mov_b64 exec, 1\n\t"
      "ds_add_u32 %1, %2\n\t"
      "s_mov_b64 exec, %0"
      : "=&s"(saved)
      : "v"(lds_addr(f)), "v"(1u)
      : "memory");
}
__device__ __forceinline__ void ct_wait(const uint32_t* f, uint32_t target) {
  uint32_t tv;
  uint32_t ts;
  asm volatile(
      "1:\n\t"
      "ds_read_b32 %0, %2\n\t"
      "s_waitcnt lgkmcnt(0)\n\t"
      "v_readfirstlane_b32 %1, %0\n\t"
      "s_cmp_lt_u32 %1, %3\n\t"
      "s_cbranch_scc0 2f\n\t"
      "s_sleep 1\n\t"
      "s_branch 1b\n"
      "2:"
      : "=&v"(tv), "=&s"(ts)
      : "v"(lds_addr(f)), "s"(target)
      : "memory", "scc");
}

// ---- register-level pieces ---------------------------------------------
constexpr double RH = 0.70710678118654752440;  // sqrt(2)/2

// constant DFT-8 network, DIF (natural -> bit-reversed within the pass).
// The w8 and w8^3 twiddles of elements 5 and 7 are (1 -+ i) * RH: the
// (1 -+ i) part is two adds, and the RH factor is carried through the bit-1
// butterfly (which mixes only 5 and 7) into the bit-0 butterflies as FMAs.
__device__ __forceinline__ void dft8(c64 (&v)[S]) {
#pragma unroll
  for (int u = 0; u < 4; ++u) {  // slot bit 2; twiddles 1, w8, i, w8^3
    const c64 X = v[u], Y = v[u + 4];
    v[u] = cadd(X, Y);
    const c64 D = csub(X, Y);
    if (u == 0) v[4] = D;
    if (u == 1) v[5] = {D.x - D.y, D.x + D.y};        // / RH
    if (u == 2) v[6] = {-D.y, D.x};
    if (u == 3) v[7] = {-(D.x + D.y), D.x - D.y};     // / RH
  }
#pragma unroll
  for (int q = 0; q < 4; ++q) {  // slot bit 1; twiddles 1, i
    const int u = ((q >> 1) << 2) | (q & 1);
    const c64 X = v[u], Y = v[u + 2];
    v[u] = cadd(X, Y);
    const c64 D = csub(X, Y);
    v[u + 2] = (u & 1) ? c64{-D.y, D.x} : D;
  }
#pragma unroll
  for (int u = 0; u < S; u += 2) {  // slot bit 0
    const c64 X = v[u], Y = v[u + 1];
    if (u >= 4) {  // v[5], v[7] still lack their RH factor
      v[u] = {__fma_rn(Y.x, RH, X.x), __fma_rn(Y.y, RH, X.y)};
      v[u + 1] = {__fma_rn(Y.x, -RH, X.x), __fma_rn(Y.y, -RH, X.y)};
    } else {
      v[u] = cadd(X, Y);
      v[u + 1] = csub(X, Y);
    }
  }
}
// its exact inverse up to a factor 8 (DIT, conjugate constants); the RH of
// the exp(-i pi/4) and exp(-3 i pi/4) twiddles goes into the last butterflies
__device__ __forceinline__ void idft8(c64 (&v)[S]) {
#pragma unroll
  for (int u = 0; u < S; u += 2) {
    const c64 X = v[u], Y = v[u + 1];
    v[u] = cadd(X, Y);
    v[u + 1] = csub(X, Y);
  }
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int u = ((q >> 1) << 2) | (q & 1);
    const c64 X = v[u], Y0 = v[u + 2];
    const c64 Y = (u & 1) ? c64{Y0.y, -Y0.x} : Y0;  // * conj(i)
    v[u] = cadd(X, Y);
    v[u + 2] = csub(X, Y);
  }
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const c64 X = v[u], Y0 = v[u + 4];
    if (u == 1 || u == 3) {
      // u = 1: * exp(-i pi/4) = RH (1 - i); u = 3: * exp(-3 i pi/4) = RH (-1 - i)
      const c64 Y = (u == 1) ? c64{Y0.x + Y0.y, Y0.y - Y0.x} : c64{Y0.y - Y0.x, -(Y0.x + Y0.y)};
      v[u] = {__fma_rn(Y.x, RH, X.x), __fma_rn(Y.y, RH, X.y)};
      v[u + 4] = {__fma_rn(Y.x, -RH, X.x), __fma_rn(Y.y, -RH, X.y)};
    } else {
      const c64 Y = (u == 2) ? c64{Y0.y, -Y0.x} : Y0;  // * -i
      v[u] = cadd(X, Y);
      v[u + 4] = csub(X, Y);
    }
  }
}

// lane twiddles of pass PS (0 = A: elements 0..7, entries m; 1 = B: elements
// 1..7, entries 7 + m), in two batches of LDS reads to bound register use;
// DBG bit 0 takes them from wf
// (NR > 0: pass A's first NR entries come from treg, kept in registers)
template <int PS, bool INV, int DBG = 0, int NR = 0>
__device__ __forceinline__ void lane_tw(c64 (&v)[S], const c64* twl, int lane, c64 wf, const c64* treg = nullptr) {
  constexpr int M0 = PS == 0 ? 0 : 1;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int m0 = h ? 4 : M0, m1 = h ? 7 : 3;
    c64 T[4];
#pragma unroll
    for (int m = m0; m <= m1; ++m)
      T[m - m0] = (DBG & 1)            ? wf
                  : (PS == 0 && m < NR) ? treg[m]
                  : PS == 0             ? twl[m * 64 + lane]
                                        : twl[NTA + (m - 1) * 8 + lb_low3(lane)];
#pragma unroll
    for (int u = 0; u < S; ++u) {
      const int m = bitrev3(u);
      if (m < m0 || m > m1) continue;
      v[u] = INV ? cmulc(v[u], T[m - m0]) : cmul(v[u], T[m - m0]);
    }
  }
}

// the slot part of the fold twist, exp(i pi u / 16) (conjugate when INV)
template <bool INV>
__device__ __forceinline__ void fold8(c64 (&v)[S]) {
  constexpr double C[8] = {1.0, 0.98078528040323044913, 0.92387953251128675613, 0.83146961230254523708,
                           0.70710678118654752440, 0.55557023301960222474, 0.38268343236508977173,
                           0.19509032201612826785};
#pragma unroll
  for (int u = 1; u < S; ++u) {
    const c64 c = {C[u], INV ? -C[8 - u] : C[8 - u]};  // sin(pi u/16) = cos(pi (8-u)/16)
    v[u] = cmul(v[u], c);
  }
}

// Wave-local relayout through the wave's own scratch: no barrier and no
// wait between the writes and the reads — one wave's DS operations are
// performed in order, so its reads see its writes (and a later write cannot
// overtake an earlier read); the compiler keeps these possibly-aliasing
// accesses in program order and waits only before the data is used.
template <int R, int LS, int LT, int DBG = 0>
__device__ __forceinline__ void relayout(c64 (&v)[S], c64* scr, int lane) {
  if constexpr ((DBG & 8) != 0) return;
#pragma unroll
  for (int u = 0; u < S; ++u) scr[rpos(R, jof(LS, lane, u))] = v[u];
#pragma unroll
  for (int u = 0; u < S; ++u) v[u] = scr[rpos(R, jof(LT, lane, u))];
}

// LA <-> LB in registers (self-inverse): slot bit 2 <-> lane bit 5 by
// v_permlane32_swap, slot bit 1 <-> lane bit 4 by v_permlane16_swap (both
// exchange half-rows between two registers), slot bit 0 <-> lane bit 3 by
// two DPP row shifts of 8 lanes whose bank masks keep the half-rows that stay.
__device__ __forceinline__ uint32_t dpp_shr8_hi(uint32_t old, uint32_t src) {  // banks 2,3 <- src[lane - 8]
  return (uint32_t)__builtin_amdgcn_update_dpp((int)old, (int)src, 0x118, 0xF, 0xC, false);
}
__device__ __forceinline__ uint32_t dpp_shl8_lo(uint32_t old, uint32_t src) {  // banks 0,1 <- src[lane + 8]
  return (uint32_t)__builtin_amdgcn_update_dpp((int)old, (int)src, 0x108, 0xF, 0x3, false);
}
template <int KIND>  // 0: permlane32 (slot bit 2), 1: permlane16 (slot bit 1), 2: dpp (slot bit 0)
__device__ __forceinline__ void swap_pair(double& x, double& y) {
  const uint64_t xb = __builtin_bit_cast(uint64_t, x), yb = __builtin_bit_cast(uint64_t, y);
  uint32_t x0 = (uint32_t)xb, x1 = (uint32_t)(xb >> 32), y0 = (uint32_t)yb, y1 = (uint32_t)(yb >> 32);
  if constexpr (KIND == 0) {
    auto a = __builtin_amdgcn_permlane32_swap(x0, y0, false, false);
    auto b = __builtin_amdgcn_permlane32_swap(x1, y1, false, false);
    x0 = a[0], y0 = a[1], x1 = b[0], y1 = b[1];
  } else if constexpr (KIND == 1) {
    auto a = __builtin_amdgcn_permlane16_swap(x0, y0, false, false);
    auto b = __builtin_amdgcn_permlane16_swap(x1, y1, false, false);
    x0 = a[0], y0 = a[1], x1 = b[0], y1 = b[1];
  } else {
    const uint32_t nx0 = dpp_shr8_hi(x0, y0), nx1 = dpp_shr8_hi(x1, y1);
    const uint32_t ny0 = dpp_shl8_lo(y0, x0), ny1 = dpp_shl8_lo(y1, x1);
    x0 = nx0, x1 = nx1, y0 = ny0, y1 = ny1;
  }
  x = __builtin_bit_cast(double, (uint64_t)x0 | ((uint64_t)x1 << 32));
  y = __builtin_bit_cast(double, (uint64_t)y0 | ((uint64_t)y1 << 32));
}
template <int KIND, int STRIDE>
__device__ __forceinline__ void swap_bit(c64 (&v)[S]) {
#pragma unroll
  for (int u = 0; u < S; ++u) {
    if (u & STRIDE) continue;
    swap_pair<KIND>(v[u].x, v[u + STRIDE].x);
    swap_pair<KIND>(v[u].y, v[u + STRIDE].y);
  }
}
__device__ __forceinline__ void swap_lb(c64 (&v)[S]) {
  swap_bit<0, 4>(v);
  swap_bit<1, 2>(v);
  swap_bit<2, 1>(v);
}
// folded coefficient pairs (a_t + i a_{t+M}), natural order (LA) -> LC;
// includes the negacyclic twist w^t
template <int DBG = 0, int NR = 0>
__device__ __forceinline__ void forward(c64 (&v)[S], const c64* twl, c64* scr, int lane, c64 wf = {},
                                        const c64* treg = nullptr) {
  fold8<false>(v);
  dft8(v);
  lane_tw<0, false, DBG, NR>(v, twl, lane, wf, treg);
  if constexpr (FHEICP_ABLDS) relayout<R1F, LA, LB, DBG>(v, scr, lane);
  else if constexpr ((DBG & 8) == 0) swap_lb(v);
  dft8(v);
  lane_tw<1, false, DBG>(v, twl, lane, wf);
  relayout<R2F, LB, LC, DBG>(v, scr, lane);
  dft8(v);
}
// LC -> natural order (LA), times M, untwisted
template <int DBG = 0, int NR = 0>
__device__ __forceinline__ void inverse(c64 (&v)[S], const c64* twl, c64* scr, int lane, c64 wf = {},
                                        const c64* treg = nullptr) {
  idft8(v);
  relayout<R2I, LC, LB, DBG>(v, scr, lane);
  lane_tw<1, true, DBG>(v, twl, lane, wf);
  idft8(v);
  if constexpr (FHEICP_ABLDS) relayout<R1I, LB, LA, DBG>(v, scr, lane);
  else if constexpr ((DBG & 8) == 0) swap_lb(v);
  lane_tw<0, true, DBG, NR>(v, twl, lane, wf, treg);
  idft8(v);
  fold8<true>(v);
}

// the inverse from layout LB on (after the C -> B relayout's writes and reads,
// which a caller may have split between waves)
template <int DBG = 0, int NR = 0>
__device__ __forceinline__ void inverse_post(c64 (&v)[S], const c64* twl, c64* scr, int lane, c64 wf = {},
                                             const c64* treg = nullptr) {
  lane_tw<1, true, DBG>(v, twl, lane, wf);
  idft8(v);
  if constexpr (FHEICP_ABLDS) relayout<R1I, LB, LA, DBG>(v, scr, lane);
  else if constexpr ((DBG & 8) == 0) swap_lb(v);
  lane_tw<0, true, DBG, NR>(v, twl, lane, wf, treg);
  idft8(v);
  fold8<true>(v);
}

// ---- accumulator word type ------------------------------------------------
template <bool A32>
struct Acc;
template <>
struct Acc<true> {
  using T = uint32_t;
  static __device__ __forceinline__ T from64(u64 x) { return (T)((x + (1ull << 31)) >> 32); }
  static __device__ __forceinline__ u64 to64(T x) { return (u64)x << 32; }
  // round(z / 2^32) mod 2^32, exact for any z, from t = z / 2^64 (the
  // FFT-domain BSK carries the 2^-64, k_bsk_to_fft_v4): f = fract(t) is
  // exact, and f * 2^32 + 1.5 * 2^52 has an ulp of 1, so its low mantissa
  // word is round(f * 2^32).
  // (Rounding at 2^35 instead, one fma, was measured to double the
  // bootstrap noise: the output rounding is key-weighted like the gadget's.)
  static __device__ __forceinline__ T from_f64(double z) {
#ifdef FHEICP_A32_ROUND35  // A/B build only (tools/build_variant.sh)
    const double t35 = __fma_rn(z, 4294967296.0, 54043195528445952.0);
    return (T)(uint32_t)__builtin_bit_cast(uint64_t, t35) << 3;
#endif
    const double f = __builtin_amdgcn_fract(z);
#ifdef FHEICP_FMA_ROUND
    const double t = __fma_rn(f, 4294967296.0, 6755399441055744.0);
#else
    // f * 2^32 is exact, so the add rounds once as the fma would; the fma's
    // accumulator operand costs two v_mov per coefficient (its destination
    // is the 1.5 * 2^52 constant), ldexp + add with an SGPR constant none
    const double t = __builtin_ldexp(f, 32) + 6755399441055744.0;
#endif
    return (T)(uint32_t)__builtin_bit_cast(uint64_t, t);
  }
};
template <>
struct Acc<false> {
  using T = u64;
  static __device__ __forceinline__ T from64(u64 x) { return x; }
  static __device__ __forceinline__ u64 to64(T x) { return x; }
  // round(z * 2^64) mod 2^64 from t = z (the FFT-domain BSK carries the
  // 2^-64 here too), bit-identical to f64_to_torus(z * 2^64) for any z:
  // f = z - rint(z) is exact, F = f * 2^32 splits into h = rint(F) (the low
  // mantissa word of F + 1.5 * 2^52) and r = F - h (exact, |r| <= 1/2),
  // and bits(r * 2^32 + 1.5 * 2^52) = bits(1.5 * 2^52) + rint(r * 2^32).
  // 8 f64 + 4 integer ops against f64_to_torus's 9 + 6 (split via floor,
  // a sign fix-up and two conversions).
  // (+ add: a constant folded into the subtraction, the A48 rounding bias)
  static __device__ __forceinline__ T from_f64(double z, uint32_t add = 0) {
#ifdef FHEICP_TORUS_SPLIT  // A/B build only (tools/build_variant.sh)
    return f64_to_torus(__builtin_ldexp(z, 64)) + add;
#endif
    constexpr double M = 6755399441055744.0;
    const double F = __builtin_ldexp(z - __builtin_rint(z), 32);
    const double t1 = F + M;
    const double t2 = __builtin_ldexp(F - (t1 - M), 32) + M;
    const u64 hi = (u64)(uint32_t)__builtin_bit_cast(u64, t1) << 32;
    return hi + (__builtin_bit_cast(u64, t2) - (0x4338000000000000ull - add));
  }
};

}  // namespace v4
}  // namespace fhei
