// VALU issue-rate probe for gfx950: lane-ops/s of single 32-bit integer and
// f32 instructions with many waves per SIMD, to price the integer roofline of
// k_encrypt_linear (ChaCha20: v_add_u32, v_xor_b32, v_alignbit_b32; the u64
// MAC: v_mad_u64_u32, v_mul_lo_u32). Eight independent chains per lane, each
// instruction one inline-asm statement so nothing folds. Not part of the
// product. hipcc --offload-arch=gfx950 -O3 tools/valu_probe.hip -o tools/valu_probe
#include <hip/hip_runtime.h>
#include <cstdio>

#include "../fhe-icp_amd/csrc/prng.h"

#define CHK(x)                                                                   \
  do {                                                                           \
    hipError_t e = (x);                                                          \
    if (e != hipSuccess) {                                                       \
      printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__);                    \
      return 1;                                                                  \
    }                                                                            \
  } while (0)

constexpr int ITERS = 2048;

#define OP8(STMT) STMT(0) STMT(1) STMT(2) STMT(3) STMT(4) STMT(5) STMT(6) STMT(7)

template <int OP>
__global__ void __launch_bounds__(256) k_probe(unsigned* out, unsigned seed) {
  unsigned x[8], y = seed ^ threadIdx.x;
  float f[8], g = (float)(threadIdx.x & 7) * 1e-3f;
  unsigned long long m[8];
  double d[8], dg = 1.0 + 1e-9 * threadIdx.x, dh = 1e-3;
#pragma unroll
  for (int c = 0; c < 8; ++c) x[c] = seed * (c + 1) + threadIdx.x, f[c] = (float)c, m[c] = x[c], d[c] = c;
  for (int i = 0; i < ITERS; ++i) {
#define ADD(c) asm volatile("v_add_u32 %0, %0, %1" : "+v"(x[c]) : "v"(y));
#define XOR(c) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(x[c]) : "v"(y));
#define ALB(c) asm volatile("v_alignbit_b32 %0, %0, %0, 16" : "+v"(x[c]));
#define FAD(c) asm volatile("v_add_f32 %0, %0, %1" : "+v"(f[c]) : "v"(g));
#define MUL(c) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(x[c]) : "v"(y));
#define MAD(c) asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(m[c]) : "v"(x[c]), "v"(y) : "vcc");
#define AD3(c) asm volatile("v_add3_u32 %0, %0, %1, %1" : "+v"(x[c]) : "v"(y));
#define F64(c) asm volatile("v_fma_f64 %0, %1, %2, %0" : "+v"(d[c]) : "v"(dg), "v"(dh));
    if constexpr (OP == 0) { OP8(ADD) }
    if constexpr (OP == 1) { OP8(XOR) }
    if constexpr (OP == 2) { OP8(ALB) }
    if constexpr (OP == 3) { OP8(FAD) }
    if constexpr (OP == 4) { OP8(MUL) }
    if constexpr (OP == 5) { OP8(MAD) }
    if constexpr (OP == 6) { OP8(AD3) }
    if constexpr (OP == 7) { OP8(ADD) OP8(XOR) OP8(ALB) }  // ChaCha20's mix, 1:1:1
    if constexpr (OP == 10) { OP8(F64) }
    if constexpr (OP == 8 || OP == 9) {  // the product's ChaCha20 block (976 ops), 1 or 2 per step
      if ((i & 7) == 0) {
        fhei::ChaKey K;
#pragma unroll
        for (int q = 0; q < 8; ++q) K.w[q] = seed + q;
        uint32_t o[16], o2[16];
        fhei::chacha20_block(K, x[0], 7u, ((unsigned long long)i << 32) | threadIdx.x, o);
        if constexpr (OP == 9) fhei::chacha20_block(K, x[1], 8u, ((unsigned long long)i << 32) | threadIdx.x, o2);
#pragma unroll
        for (int q = 0; q < 8; ++q) x[q] ^= o[q] ^ o[q + 8];
        if constexpr (OP == 9) {
#pragma unroll
          for (int q = 0; q < 8; ++q) x[q] += o2[q] ^ o2[q + 8];
        }
      }
    }
  }
  unsigned r = 0;
#pragma unroll
  for (int c = 0; c < 8; ++c)
    r ^= x[c] ^ __float_as_uint(f[c]) ^ (unsigned)m[c] ^ (unsigned)(m[c] >> 32) ^ (unsigned)__double_as_longlong(d[c]);
  out[blockIdx.x * 256 + threadIdx.x] = r;
}

template <int OP>
static int run(const char* name, int per_iter, int blocks, unsigned* d) {
  hipEvent_t a, b;
  CHK(hipEventCreate(&a));
  CHK(hipEventCreate(&b));
  hipLaunchKernelGGL(k_probe<OP>, dim3(blocks), dim3(256), 0, 0, d, 7u);
  CHK(hipDeviceSynchronize());
  CHK(hipEventRecord(a));
  const int reps = 10;
  for (int i = 0; i < reps; ++i) hipLaunchKernelGGL(k_probe<OP>, dim3(blocks), dim3(256), 0, 0, d, 7u + i);
  CHK(hipEventRecord(b));
  CHK(hipEventSynchronize(b));
  float ms;
  CHK(hipEventElapsedTime(&ms, a, b));
  const double ops = (double)blocks * 256 * ITERS * per_iter * reps;  // lane-instructions
  printf("%-26s blocks %6d: %7.2f T lane-ops/s (%.3f ms per launch)\n", name, blocks, ops / (ms * 1e-3) / 1e12,
         ms / reps);
  return 0;
}

int main() {
  hipDeviceProp_t pr;
  CHK(hipGetDeviceProperties(&pr, 0));
  printf("%s, %d CUs, clock %d kHz\n", pr.gcnArchName, pr.multiProcessorCount, pr.clockRate);
  unsigned* d;
  const int maxb = pr.multiProcessorCount * 8 * 4;  // up to 8 waves per SIMD
  CHK(hipMalloc(&d, (size_t)maxb * 256 * 4));
  for (int wps : {1, 2, 4, 8}) {  // waves per SIMD (4 waves per block, one per SIMD)
    const int blocks = pr.multiProcessorCount * wps;
    printf("-- %d wave(s) per SIMD\n", wps);
    if (run<0>("v_add_u32", 8, blocks, d) || run<1>("v_xor_b32", 8, blocks, d) ||
        run<2>("v_alignbit_b32", 8, blocks, d) || run<3>("v_add_f32", 8, blocks, d) ||
        run<4>("v_mul_lo_u32", 8, blocks, d) || run<5>("v_mad_u64_u32", 8, blocks, d) ||
        run<6>("v_add3_u32", 8, blocks, d) || run<7>("add/xor/alignbit 1:1:1", 24, blocks, d) ||
        run<8>("chacha20 x1 (976/8 per it)", 122, blocks, d) || run<9>("chacha20 x2 (976/4 per it)", 244, blocks, d) ||
        run<10>("v_fma_f64", 8, blocks, d))
      return 1;
  }
  return 0;
}
