// VALU issue-rate probe for gfx950: lane-ops/s of single 32-bit integer and
// f32 instructions with many waves per SIMD, to price the integer roofline of
// k_encrypt_linear (ChaCha20: v_add_u32, v_xor_b32, v_alignbit_b32; the u64
// MAC: v_mad_u64_u32, v_mul_lo_u32). Eight independent chains per lane, each
// instruction one inline-asm statement so nothing folds. Not part of the
// product. hipcc --offload-arch=gfx950 -O3 tools/valu_probe.hip -o tools/valu_probe
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

constexpr int ITERS = 2048;

#define OP8(STMT) STMT(0) STMT(1) STMT(2) STMT(3) STMT(4) STMT(5) STMT(6) STMT(7)

template <int OP>
__global__ void __launch_bounds__(256) k_probe(unsigned* out, unsigned seed) {
  unsigned x[8], y = seed ^ threadIdx.x;
  float f[8], g = (float)(threadIdx.x & 7) * 1e-3f;
  unsigned long long m[8];
#pragma unroll
  for (int c = 0; c < 8; ++c) x[c] = seed * (c + 1) + threadIdx.x, f[c] = (float)c, m[c] = x[c];
  for (int i = 0; i < ITERS; ++i) {
#define ADD(c) asm volatile("v_add_u32 %0, %0, %1" : "+v"(x[c]) : "v"(y));
#define XOR(c) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(x[c]) : "v"(y));
#define ALB(c) asm volatile("v_alignbit_b32 %0, %0, %0, 16" : "+v"(x[c]));
#define FAD(c) asm volatile("v_add_f32 %0, %0, %1" : "+v"(f[c]) : "v"(g));
#define MUL(c) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(x[c]) : "v"(y));
#define MAD(c) asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(m[c]) : "v"(x[c]), "v"(y) : "vcc");
#define AD3(c) asm volatile("v_add3_u32 %0, %0, %1, %1" : "+v"(x[c]) : "v"(y));
    if constexpr (OP == 0) { OP8(ADD) }
    if constexpr (OP == 1) { OP8(XOR) }
    if constexpr (OP == 2) { OP8(ALB) }
    if constexpr (OP == 3) { OP8(FAD) }
    if constexpr (OP == 4) { OP8(MUL) }
    if constexpr (OP == 5) { OP8(MAD) }
    if constexpr (OP == 6) { OP8(AD3) }
    if constexpr (OP == 7) { OP8(ADD) OP8(XOR) OP8(ALB) }  // ChaCha20's mix, 1:1:1
  }
  unsigned r = 0;
#pragma unroll
  for (int c = 0; c < 8; ++c) r ^= x[c] ^ __float_as_uint(f[c]) ^ (unsigned)m[c] ^ (unsigned)(m[c] >> 32);
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
        run<6>("v_add3_u32", 8, blocks, d) || run<7>("add/xor/alignbit 1:1:1", 24, blocks, d))
      return 1;
  }
  return 0;
}
