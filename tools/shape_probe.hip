// Shape probe: the measured per-point costs behind the
// k = 1, N = 2048 estimate of tools/shape_plans.py. Not part of the product.
//   shape 0: one wave owns a 512-point complex f64 transform, 8 values per lane
//            (the shipped k = 2, N = 1024 rotation's v4 forward + inverse:
//            br_v4.h, relayout through the wave's own LDS slot);
//   shape 1: one wave owns a 1024-point transform, 16 values per lane (what a
//            k = 1, N = 2048 rotation's wave would run): two 512-point v4
//            transforms on the even / odd halves and one radix-2 stage
//            (decimation in time: 8 twiddle multiplies + 16 adds per lane, the
//            twiddles from LDS), and its exact inverse;
//   mac:     the products' complex multiply-accumulate (P += F K, F from LDS
//            as the kernels read it, K from a buffer as the key rows), the
//            instruction both shapes' products are made of.
// Each at 3 waves per SIMD (the shipped kernels' occupancy: 768-thread
// workgroups, one per CU) and shape 1 also at 2 (a 1024-point wave holds
// twice the values; a k = 1 kernel would likely be limited to 2).
// Prints transform points per second chip-wide and ns per point per SIMD.
// hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/shape_probe.hip -o tools/shape_probe
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <vector>

#include "../fhe-icp_amd/csrc/br_v4.h"

using namespace fhei;
using namespace fhei::v4;

#define CHK(x)                                                                   \
  do {                                                                           \
    hipError_t e = (x);                                                          \
    if (e != hipSuccess) {                                                       \
      printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__);                    \
      return 1;                                                                  \
    }                                                                            \
  } while (0)

constexpr int MAXW = 12;  // waves per workgroup (one workgroup per CU)
constexpr int NT2 = 512;  // radix-2 stage twiddles (one per output pair position)

template <int SHAPE, int WAVES>
__global__ void __launch_bounds__(64 * WAVES, 1) k_tf(const c64* __restrict__ tw4, const c64* __restrict__ tw2,
                                                       int iters, double* __restrict__ out) {
  __shared__ c64 twl[NTW];
  __shared__ c64 t2[NT2];
  __shared__ c64 scr[MAXW * SCR];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  fill_tables(twl, tw4, tid, 64 * WAVES);
  for (int x = tid; x < NT2; x += 64 * WAVES) t2[x] = tw2[x];
  __syncthreads();
  c64* slot = scr + w * SCR;
  c64 a[S], b[S];
#pragma unroll
  for (int u = 0; u < S; ++u) {
    a[u] = {1e-3 * (lane + u), 1e-3 * (u - lane)};
    b[u] = {2e-3 * (lane - u), 1e-3 * (u + 2)};
  }
  const double sc = 1.0 / (double)M;
  for (int it = 0; it < iters; ++it) {
    if constexpr (SHAPE == 0) {
      forward(a, twl, slot, lane);
      inverse(a, twl, slot, lane);
#pragma unroll
      for (int u = 0; u < S; ++u) a[u] = {a[u].x * sc, a[u].y * sc};
    } else {
      forward(a, twl, slot, lane);
      forward(b, twl, slot, lane);
      // X_k = A_k + W^k B_k, X_(k+512) = A_k - W^k B_k
#pragma unroll
      for (int u = 0; u < S; ++u) {
        const c64 W = t2[u * 64 + lane];
        const c64 B = cmul(b[u], W);
        b[u] = csub(a[u], B);
        a[u] = cadd(a[u], B);
      }
      // inverse: A = (X + X') / 2, B = (X - X') conj(W) / 2
#pragma unroll
      for (int u = 0; u < S; ++u) {
        const c64 W = t2[u * 64 + lane];
        const c64 X = a[u], Y = b[u];
        a[u] = cadd(X, Y);
        b[u] = cmulc(csub(X, Y), W);
      }
      inverse(a, twl, slot, lane);
      inverse(b, twl, slot, lane);
#pragma unroll
      for (int u = 0; u < S; ++u) {
        a[u] = {a[u].x * sc * 0.5, a[u].y * sc * 0.5};
        b[u] = {b[u].x * sc * 0.5, b[u].y * sc * 0.5};
      }
    }
  }
  double s = 0;
#pragma unroll
  for (int u = 0; u < S; ++u) s += a[u].x + a[u].y + b[u].x - b[u].y;
  out[blockIdx.x * blockDim.x + tid] = s;
}

// P += F[r] K[r] over R rows per point, 8 points per lane per iteration (the
// products of one slot quarter), F from LDS, K by buffer loads of an
// L2-resident key, then the psi factor from an LDS table
template <int WAVES>
__global__ void __launch_bounds__(64 * WAVES, 1) k_mac(const c64* __restrict__ key, int iters, double* __restrict__ out) {
  constexpr int R = 3;
  __shared__ c64 F[8 * R * 64];  // one slot quarter's F, read by every wave
  __shared__ c64 psi[2048];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  for (int x = tid; x < 8 * R * 64; x += 64 * WAVES) F[x] = {1e-3 * x, 2e-3};
  for (int x = tid; x < 2048; x += 64 * WAVES) psi[x] = {std::cos(x * 1e-3), std::sin(x * 1e-3)};
  __syncthreads();
  const __amdgpu_buffer_rsrc_t krs = __builtin_amdgcn_make_buffer_rsrc((void*)key, (short)0, 0x7fffffff, 0x00020000);
  c64 o[8];
#pragma unroll
  for (int p = 0; p < 8; ++p) o[p] = {0.0, 0.0};
  uint32_t e = lane * 37u;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int p = 0; p < 8; ++p) {
      c64 P = {0.0, 0.0};
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const c64 K = __builtin_bit_cast(
            c64, __builtin_amdgcn_raw_buffer_load_b128(krs, (lane * 16), ((it & 63) * 24 + p * R + r) * 1024, 0));
        cmac(P, F[(p * R + r) * 64 + ((lane + w) & 63)], K);
      }
      e = e * 1103515245u + 12345u;
      cmac(o[p], psi[(e >> 8) & 2047], P);
    }
  }
  double s = 0;
#pragma unroll
  for (int p = 0; p < 8; ++p) s += o[p].x + o[p].y;
  out[blockIdx.x * blockDim.x + tid] = s;
}

template <class F>
static float time_ms(F launch) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  launch();
  (void)hipDeviceSynchronize();
  float best = 1e30f;
  for (int rep = 0; rep < 3; ++rep) {
    (void)hipEventRecord(e0);
    launch();
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    best = std::min(best, ms);
  }
  return best;
}

int main() {
  hipDeviceProp_t prop;
  CHK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  printf("%s, %d CUs, clock %d kHz\n", prop.gcnArchName, cus, prop.clockRate);
  // v4 per-lane twiddles as fhe_ctx_create builds them, and the radix-2 stage's
  const long double PI = 3.14159265358979323846264338327950288L;
  std::vector<c64> t4(NTW), t2(NT2);
  for (int m = 0; m < 8; ++m)
    for (int l = 0; l < 64; ++l) {
      const long double ang = PI * (long double)l * (long double)(1 + 4 * m) / 1024.0L;
      t4[m * 64 + l] = {(double)cosl(ang), (double)sinl(ang)};
    }
  for (int m = 1; m < 8; ++m)
    for (int L = 0; L < 8; ++L) {
      const long double ang = 2.0L * PI * (long double)(L * m) / 64.0L;
      t4[NTA + (m - 1) * 8 + L] = {(double)cosl(ang), (double)sinl(ang)};
    }
  for (int x = 0; x < NT2; ++x) t2[x] = {(double)cosl(PI * x / 512.0L), (double)sinl(PI * x / 512.0L)};
  c64 *dtw4, *dtw2, *dkey;
  double* dout;
  CHK(hipMalloc(&dtw4, sizeof(c64) * NTW));
  CHK(hipMalloc(&dtw2, sizeof(c64) * NT2));
  CHK(hipMalloc(&dkey, sizeof(c64) * 64 * 64 * 24 * 8));
  CHK(hipMemset(dkey, 0, sizeof(c64) * 64 * 64 * 24 * 8));
  CHK(hipMalloc(&dout, sizeof(double) * cus * 64 * MAXW));
  CHK(hipMemcpy(dtw4, t4.data(), sizeof(c64) * NTW, hipMemcpyHostToDevice));
  CHK(hipMemcpy(dtw2, t2.data(), sizeof(c64) * NT2, hipMemcpyHostToDevice));
  const int iters = 256;
  const double simds = 4.0 * cus;
  auto report = [&](const char* name, float ms, double waves_per_cu, int points_per_wave_iter, const char* unit) {
    const double pts = (double)cus * waves_per_cu * iters * points_per_wave_iter;
    printf("%-44s %8.3f ms  %9.3f G%s/s  %8.4f ns per %s per SIMD\n", name, ms, pts / ms / 1e6, unit,
           ms * 1e6 * simds / pts, unit);
  };
  // transform points: a forward + inverse pair counts M points (per transform pair)
  float ms;
  ms = time_ms([&] { hipLaunchKernelGGL((k_tf<0, 12>), dim3(cus), dim3(768), 0, 0, dtw4, dtw2, iters, dout); });
  report("512-pt fwd+inv, 3 waves/SIMD", ms, 12, 512, "pt");
  ms = time_ms([&] { hipLaunchKernelGGL((k_tf<1, 12>), dim3(cus), dim3(768), 0, 0, dtw4, dtw2, iters, dout); });
  report("1024-pt fwd+inv, 3 waves/SIMD", ms, 12, 1024, "pt");
  ms = time_ms([&] { hipLaunchKernelGGL((k_tf<1, 8>), dim3(cus), dim3(512), 0, 0, dtw4, dtw2, iters, dout); });
  report("1024-pt fwd+inv, 2 waves/SIMD", ms, 8, 1024, "pt");
  ms = time_ms([&] { hipLaunchKernelGGL((k_tf<0, 8>), dim3(cus), dim3(512), 0, 0, dtw4, dtw2, iters, dout); });
  report("512-pt fwd+inv, 2 waves/SIMD", ms, 8, 512, "pt");
  // MACs: 8 points x (3 row MACs + 1 psi MAC) per lane per iteration
  ms = time_ms([&] { hipLaunchKernelGGL((k_mac<12>), dim3(cus), dim3(768), 0, 0, dkey, iters, dout); });
  report("cmac (F from LDS, key by buffer), 3 w/SIMD", ms, 12, 64 * 8 * 4, "cmac");
  ms = time_ms([&] { hipLaunchKernelGGL((k_mac<8>), dim3(cus), dim3(512), 0, 0, dkey, iters, dout); });
  report("cmac (F from LDS, key by buffer), 2 w/SIMD", ms, 8, 64 * 8 * 4, "cmac");
  CHK(hipGetLastError());
  return 0;
}
