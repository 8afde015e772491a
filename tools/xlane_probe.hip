// Cross-lane instruction probe for gfx950: issue cost of the lane exchanges
// the FFT transforms use (v_permlane32_swap, v_permlane16_swap, bank-masked
// v_mov_b32_dpp row shifts, v_cndmask_b32 with a quad_perm DPP source) against
// v_fma_f64 and v_mov_b32, at 1 and 3 waves per SIMD; eight independent
// chains per lane, one inline-asm statement per instruction. Not part of the
// product. hipcc --offload-arch=gfx950 -O3 tools/xlane_probe.hip -o tools/xlane_probe
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
#define OP8(STMT) STMT(0, 1) STMT(2, 3) STMT(4, 5) STMT(6, 7)

template <int OP>
__global__ void __launch_bounds__(1024) k_probe(unsigned* out, unsigned seed) {
  unsigned x[8];
  double d[8], dg = 1.0 + 1e-9 * threadIdx.x, dh = 1e-3;
#pragma unroll
  for (int c = 0; c < 8; ++c) x[c] = seed * (c + 1) + threadIdx.x, d[c] = c;
  for (int i = 0; i < ITERS; ++i) {
#define F64(a, b) asm volatile("v_fma_f64 %0, %2, %3, %0\n\tv_fma_f64 %1, %2, %3, %1" : "+v"(d[a]), "+v"(d[b]) : "v"(dg), "v"(dh));
#define MOV(a, b) asm volatile("v_mov_b32 %0, %1\n\tv_mov_b32 %1, %0" : "+v"(x[a]), "+v"(x[b]));
#define P32(a, b) asm volatile("v_permlane32_swap_b32 %0, %1" : "+v"(x[a]), "+v"(x[b]));
#define P16(a, b) asm volatile("v_permlane16_swap_b32 %0, %1" : "+v"(x[a]), "+v"(x[b]));
#define DPP(a, b) asm volatile("v_mov_b32_dpp %0, %1 row_shr:8 row_mask:0xf bank_mask:0xc\n\tv_mov_b32_dpp %1, %0 row_shl:8 row_mask:0xf bank_mask:0x3" : "+v"(x[a]), "+v"(x[b]));
#define CND(a, b) asm volatile("v_cndmask_b32_dpp %0, %1, %0, vcc quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\tv_cndmask_b32_dpp %1, %0, %1, vcc quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf" : "+v"(x[a]), "+v"(x[b]) :: "vcc");
    if constexpr (OP == 0) { OP8(F64) }
    if constexpr (OP == 1) { OP8(MOV) }
    if constexpr (OP == 2) { OP8(P32) OP8(P32) }
    if constexpr (OP == 3) { OP8(P16) OP8(P16) }
    if constexpr (OP == 4) { OP8(DPP) }
    if constexpr (OP == 5) { OP8(CND) }
  }
  unsigned s = 0;
#pragma unroll
  for (int c = 0; c < 8; ++c) s ^= x[c] ^ (unsigned)d[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int OP>
static int run(const char* name, int threads, unsigned* d, int insts_per_iter) {
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0));
  CHK(hipEventCreate(&e1));
  const int blocks = 256 * 4;
  for (int rep = 0; rep < 2; ++rep) {
    CHK(hipEventRecord(e0));
    hipLaunchKernelGGL((k_probe<OP>), dim3(blocks), dim3(threads), 0, 0, d, 1u + rep);
    CHK(hipEventRecord(e1));
    CHK(hipEventSynchronize(e1));
  }
  float ms;
  CHK(hipEventElapsedTime(&ms, e0, e1));
  const double waves_per_simd = threads / 64.0 / 4.0;
  const double insts = (double)blocks * threads / 64 * ITERS * insts_per_iter;  // wave-instructions
  // cycles per wave-instruction per SIMD at 2.4 GHz nominal
  const double cyc = ms * 1e-3 * 2.4e9 * 1024 / insts;
  printf("%-40s %4d thr (%.0f waves/SIMD) %8.3f ms  %.2f SIMD-cycles per wave-instruction (2.4 GHz)\n", name,
         threads, waves_per_simd, ms, cyc);
  return 0;
}

int main() {
  unsigned* d;
  CHK(hipMalloc(&d, sizeof(unsigned) * 256 * 4 * 1024));
  for (int thr : {256, 768}) {
    run<0>("v_fma_f64", thr, d, 8);
    run<1>("v_mov_b32", thr, d, 8);
    run<2>("v_permlane32_swap_b32", thr, d, 8);
    run<3>("v_permlane16_swap_b32", thr, d, 8);
    run<4>("v_mov_b32_dpp row_shr/shl:8 banks", thr, d, 8);
    run<5>("v_cndmask_b32_dpp quad_perm", thr, d, 8);
  }
  return 0;
}
