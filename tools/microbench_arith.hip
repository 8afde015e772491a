// Arithmetic throughput probe for gfx950: Goldilocks modmul / modadd vs f64 FMA.
// Informs the NTT-vs-FFT choice in DESIGN.md §4. Not part of the product.
#include <hip/hip_runtime.h>
#include <cstdio>

// Minimal Goldilocks (p = 2^64 - 2^32 + 1) field ops, kept here only for the probe.
namespace gl {
static constexpr uint64_t P = 0xFFFFFFFF00000001ull, EPS = 0xFFFFFFFFull;
__device__ __forceinline__ uint64_t reduce128(uint64_t lo, uint64_t hi) {
  const uint64_t h0 = hi & 0xFFFFFFFFull, h1 = hi >> 32;
  uint64_t t = lo - h1; if (lo < h1) t -= EPS;
  const uint64_t u = (h0 << 32) - h0;
  uint64_t r = t + u; if (r < t) r += EPS;
  if (r >= P) r -= P;
  return r;
}
__device__ __forceinline__ uint64_t mul(uint64_t a, uint64_t b) { return reduce128(a * b, __umul64hi(a, b)); }
__device__ __forceinline__ uint64_t add(uint64_t a, uint64_t b) { uint64_t r = a + b; if (r < a) r += EPS; if (r >= P) r -= P; return r; }
__device__ __forceinline__ uint64_t sub(uint64_t a, uint64_t b) { uint64_t r = a - b; if (a < b) r -= EPS; return r; }
}

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

constexpr int CH = 8;  // independent chains per lane

__global__ void k_glmul(uint64_t* out, int iters, uint64_t seed) {
  uint64_t a[CH], b = seed ^ (threadIdx.x * 0x9E3779B97F4A7C15ull);
  for (int c = 0; c < CH; ++c) a[c] = (seed + c * 77 + threadIdx.x) % gl::P;
  b %= gl::P;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int c = 0; c < CH; ++c) a[c] = gl::mul(a[c], b);
  }
  uint64_t s = 0;
  for (int c = 0; c < CH; ++c) s ^= a[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// butterfly: (x, y) -> (x + w*y, x - w*y)
__global__ void k_glbfly(uint64_t* out, int iters, uint64_t seed) {
  uint64_t x[CH], y[CH];
  uint64_t w = (seed ^ (threadIdx.x * 0x9E3779B97F4A7C15ull)) % gl::P;
  for (int c = 0; c < CH; ++c) { x[c] = (seed + c) % gl::P; y[c] = (seed * 3 + c + threadIdx.x) % gl::P; }
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      uint64_t t = gl::mul(y[c], w);
      uint64_t u = x[c];
      x[c] = gl::add(u, t);
      y[c] = gl::sub(u, t);
    }
  }
  uint64_t s = 0;
  for (int c = 0; c < CH; ++c) s ^= x[c] ^ y[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_f64fma(double* out, int iters, double seed) {
  double a[CH];
  double b = 1.0000001 + threadIdx.x * 1e-12, c0 = 1e-9;
  for (int c = 0; c < CH; ++c) a[c] = seed + c;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int c = 0; c < CH; ++c) a[c] = __fma_rn(a[c], b, c0);
  }
  double s = 0;
  for (int c = 0; c < CH; ++c) s += a[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_u32mul(uint32_t* out, int iters, uint32_t seed) {
  uint32_t a[CH], b = seed ^ threadIdx.x;
  for (int c = 0; c < CH; ++c) a[c] = seed + c * 7 + threadIdx.x;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int c = 0; c < CH; ++c) a[c] = __umulhi(a[c], b) ^ (a[c] * b);
  }
  uint32_t s = 0;
  for (int c = 0; c < CH; ++c) s ^= a[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_u64mad(uint64_t* out, int iters, uint64_t seed) {
  uint64_t a[CH];
  uint32_t b = (uint32_t)seed ^ threadIdx.x;
  for (int c = 0; c < CH; ++c) a[c] = seed + c * 7 + threadIdx.x;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int c = 0; c < CH; ++c) a[c] = (uint64_t)(uint32_t)a[c] * b + (a[c] >> 32);  // v_mad_u64_u32
  }
  uint64_t s = 0;
  for (int c = 0; c < CH; ++c) s ^= a[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main() {
  const int blocks = 256 * 8, threads = 256, iters = 4096;
  void* buf;
  CHK(hipMalloc(&buf, (size_t)blocks * threads * 8));
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0));
  CHK(hipEventCreate(&e1));
  const double ops = (double)blocks * threads * iters * CH;
  auto run = [&](const char* name, auto launch, double per) {
    launch();  // warm
    hipDeviceSynchronize();
    hipEventRecord(e0);
    for (int r = 0; r < 3; ++r) launch();
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    ms /= 3;
    printf("%-10s %8.3f ms  %8.2f Gop/s (op=%s)\n", name, ms, ops / (ms * 1e6) * per, "chain-step");
  };
  run("glmul", [&] { k_glmul<<<blocks, threads>>>((uint64_t*)buf, iters, 12345); }, 1);
  run("glbfly", [&] { k_glbfly<<<blocks, threads>>>((uint64_t*)buf, iters, 12345); }, 1);
  run("f64fma", [&] { k_f64fma<<<blocks, threads>>>((double*)buf, iters, 1.5); }, 1);
  run("u32mul", [&] { k_u32mul<<<blocks, threads>>>((uint32_t*)buf, iters, 12345); }, 1);
  run("u64mad", [&] { k_u64mad<<<blocks, threads>>>((uint64_t*)buf, iters, 12345); }, 1);
  CHK(hipGetLastError());
  return 0;
}
