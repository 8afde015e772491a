// f64 matrix-core probe for gfx950: issue rates of v_mfma_f64_16x16x4_f64 and
// v_mfma_f64_4x4x4_4b_f64 (16 or 4 waves per CU), and whether they run beside
// v_fma_f64 streams — in other waves of the SIMD or interleaved in one wave —
// at the sum of the two rates (separate pipes) or share one f64 budget. Decides
// whether the blind rotation's key products can move to the matrix pipe
// (DESIGN.md §9). Not part of the product.
// hipcc --offload-arch=gfx950 -O3 tools/mfma_f64_probe.hip -o tools/mfma_f64_probe
#include <hip/hip_runtime.h>
#include <cstdio>

#define CHK(x)                                                                   \
  do {                                                                           \
    hipError_t e = (x);                                                          \
    if (e != hipSuccess) {                                                       \
      printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__);                    \
      return 1;                                                                  \
    }                                                                            \
  } while (0)

typedef double d4 __attribute__((ext_vector_type(4)));
constexpr int ITERS = 4096;

// MODE 0: VALU only, 8 v_fma_f64 chains per step
// MODE 1: 16x16x4 MFMA only, 4 accumulators, one MFMA per step
// MODE 2: 4x4x4_4b MFMA only, 4 accumulators, one MFMA per step
// MODE 3: one 16x16x4 MFMA + NV v_fma_f64 per step, same wave
// MODE 4: one 4x4x4_4b MFMA + NV v_fma_f64 per step, same wave
// MODE 5: even waves MODE 1, odd waves MODE 0 (other waves of the SIMD)
template <int MODE, int NV>
__global__ void __launch_bounds__(1024) k_probe(double* out, double seed) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  double a = seed + lane * 1e-3, b = 1.0 - lane * 1e-6;
  d4 c16[4];
  double c4[4];
  double v[8];
#pragma unroll
  for (int q = 0; q < 4; ++q) c16[q] = d4{0.1 * q, 0.2, 0.3, 0.4}, c4[q] = 0.5 * q;
#pragma unroll
  for (int q = 0; q < 8; ++q) v[q] = q * 0.25;
  const bool valu_wave = MODE == 5 ? (w & 1) : (MODE == 0 || MODE == 3 || MODE == 4);
  const bool mfma_wave = MODE == 5 ? !(w & 1) : (MODE != 0);
  if (mfma_wave && (MODE == 1 || MODE == 3 || MODE == 5)) {
    for (int i = 0; i < ITERS; i += 4) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        c16[q] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c16[q], 0, 0, 0);
        if constexpr (MODE == 3) {
#pragma unroll
          for (int r = 0; r < NV; ++r) asm volatile("v_fma_f64 %0, %1, %2, %0" : "+v"(v[r & 7]) : "v"(a), "v"(b));
        }
      }
    }
  }
  if (mfma_wave && (MODE == 2 || MODE == 4)) {
    for (int i = 0; i < ITERS; i += 4) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        c4[q] = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c4[q], 0, 0, 0);
        if constexpr (MODE == 4) {
#pragma unroll
          for (int r = 0; r < NV; ++r) asm volatile("v_fma_f64 %0, %1, %2, %0" : "+v"(v[r & 7]) : "v"(a), "v"(b));
        }
      }
    }
  }
  if (valu_wave && (MODE == 0 || MODE == 5)) {
    for (int i = 0; i < ITERS; ++i) {
#pragma unroll
      for (int r = 0; r < 8; ++r) asm volatile("v_fma_f64 %0, %1, %2, %0" : "+v"(v[r]) : "v"(a), "v"(b));
    }
  }
  double s = 0;
#pragma unroll
  for (int q = 0; q < 4; ++q) s += c16[q].x + c16[q].y + c16[q].z + c16[q].w + c4[q];
#pragma unroll
  for (int q = 0; q < 8; ++q) s += v[q];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int MODE, int NV>
static int run(const char* name, int threads, double* d, double mfma_flops_per_inst) {
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0));
  CHK(hipEventCreate(&e1));
  const int blocks = 256 * 4;
  for (int rep = 0; rep < 2; ++rep) {
    CHK(hipEventRecord(e0));
    hipLaunchKernelGGL((k_probe<MODE, NV>), dim3(blocks), dim3(threads), 0, 0, d, 1.0 + rep);
    CHK(hipEventRecord(e1));
    CHK(hipEventSynchronize(e1));
  }
  float ms;
  CHK(hipEventElapsedTime(&ms, e0, e1));
  const double waves = (double)blocks * threads / 64;
  const double mwaves = MODE == 5 ? waves / 2 : (MODE == 0 ? 0 : waves);
  const double vwaves = MODE == 5 ? waves / 2 : ((MODE == 0 || MODE >= 3) ? waves : 0);
  const double mf = mwaves * ITERS * mfma_flops_per_inst;
  const double vi = MODE == 0 || MODE == 5 ? 8.0 * ITERS : (double)NV * ITERS;
  const double vf = vwaves * vi * 64 * 2;
  printf("%-44s %5d thr  %8.3f ms  mfma %6.2f TF  valu %6.2f TF  sum %6.2f TF\n", name, threads, ms,
         mf / ms / 1e9, vf / ms / 1e9, (mf + vf) / ms / 1e9);
  return 0;
}

int main() {
  double* d;
  CHK(hipMalloc(&d, sizeof(double) * 256 * 4 * 1024));
  const double f16 = 2.0 * 16 * 16 * 4, f4 = 2.0 * 4 * 4 * 4 * 4;
  for (int thr : {256, 768, 1024}) {
    run<0, 0>("valu v_fma_f64 x8", thr, d, 0);
    run<1, 0>("mfma f64 16x16x4", thr, d, f16);
    run<2, 0>("mfma f64 4x4x4_4b", thr, d, f4);
    run<3, 4>("16x16x4 + 4 v_fma_f64 same wave", thr, d, f16);
    run<3, 8>("16x16x4 + 8 v_fma_f64 same wave", thr, d, f16);
    run<3, 16>("16x16x4 + 16 v_fma_f64 same wave", thr, d, f16);
    run<4, 2>("4x4x4_4b + 2 v_fma_f64 same wave", thr, d, f4);
    run<4, 4>("4x4x4_4b + 4 v_fma_f64 same wave", thr, d, f4);
    run<5, 0>("16x16x4 waves beside v_fma_f64 waves", thr, d, f16);
  }
  return 0;
}
