// Probe of the BERT GEMMs (fhe-icp_amd/csrc/bert.hip k_gemm3, bf16, and
// k_gemm2_f32, f32) at the embed bench's shapes (25.6k tokens, random
// operands): HIP-event time per launch and TFLOP/s.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 [-DFBERT_AB_NOEPI] tools/gemm_probe.hip -o gemm_probe
#include "../fhe-icp_amd/csrc/bert.hip"

#include <cstdio>
#include <vector>

int main() {
  using namespace fbert;
  const int M = 25600;
  const int shapes[4][3] = {{2304, 768, 0}, {768, 768, 2}, {3072, 768, 1}, {768, 3072, 2}};
  bf16 *A, *W;
  float *bias, *resid;
  void* out;
  hipMalloc(&A, (size_t)M * 3072 * 2);
  hipMalloc(&W, (size_t)3072 * 3072 * 2);
  hipMalloc(&bias, 3072 * 4);
  hipMalloc(&resid, (size_t)M * 3072 * 4);
  hipMalloc(&out, (size_t)M * 3072 * 4);
  {  // random bf16 in [-1, 1): exponent 0x3f00-0x3f7f (0.5-1) with random sign and mantissa
    std::vector<uint16_t> h((size_t)M * 3072);
    uint32_t x = 12345;
    for (auto& v : h) {
      x = x * 1664525u + 1013904223u;
      v = (uint16_t)(0x3e80 + ((x >> 9) & 0x7f) + (((x >> 20) & 1) << 15) + (((x >> 21) & 1) << 7));
    }
    hipMemcpy(A, h.data(), h.size() * 2, hipMemcpyHostToDevice);
    hipMemcpy(W, h.data(), (size_t)3072 * 3072 * 2, hipMemcpyHostToDevice);
  }
  hipMemset(bias, 0, 3072 * 4);
  hipMemset(resid, 0, (size_t)M * 3072 * 4);
  hipFuncSetAttribute((const void*)k_gemm3<0>, hipFuncAttributeMaxDynamicSharedMemorySize, G3_LDS);
  hipFuncSetAttribute((const void*)k_gemm3<1>, hipFuncAttributeMaxDynamicSharedMemorySize, G3_LDS);
  hipFuncSetAttribute((const void*)k_gemm3<2>, hipFuncAttributeMaxDynamicSharedMemorySize, G3_LDS);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (auto& sh : shapes) {
    const int N = sh[0], K = sh[1], epi = sh[2];
    auto run = [&]() {
      if (epi == 0) gemm3_launch<0>(A, W, bias, resid, out, M, N, K, 0);
      else if (epi == 1) gemm3_launch<1>(A, W, bias, resid, out, M, N, K, 0);
      else gemm3_launch<2>(A, W, bias, resid, out, M, N, K, 0);
    };
    run();
    hipEventRecord(e0, 0);
    for (int r = 0; r < 10; ++r) run();
    hipEventRecord(e1, 0);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    ms /= 10;
    printf("bf16 N=%d K=%d epi=%d: %.1f us, %.0f TF/s\n", N, K, epi, ms * 1e3, 2.0 * M * N * K / (ms * 1e-3) / 1e12);
  }
  // f32: the reference's arithmetic (EPI_F32 = QKV, EPI_GELU_F32 = FFN1, EPI_RESID_F32 = out / FFN2)
  float *Af, *Wf;
  hipMalloc(&Af, (size_t)M * 3072 * 4);
  hipMalloc(&Wf, (size_t)3072 * 3072 * 4);
  {
    std::vector<float> h((size_t)M * 3072);
    uint32_t x = 777;
    for (auto& v : h) {
      x = x * 1664525u + 1013904223u;
      v = (float)((int)(x >> 8) - (1 << 23)) / (float)(1 << 23);
    }
    hipMemcpy(Af, h.data(), h.size() * 4, hipMemcpyHostToDevice);
    hipMemcpy(Wf, h.data(), (size_t)3072 * 3072 * 4, hipMemcpyHostToDevice);
  }
  const int fshapes[4][3] = {{2304, 768, EPI_F32}, {768, 768, EPI_RESID_F32}, {3072, 768, EPI_GELU_F32},
                             {768, 3072, EPI_RESID_F32}};
  hipFuncSetAttribute((const void*)k_gemm2_f32<EPI_F32>, hipFuncAttributeMaxDynamicSharedMemorySize, F2_LDS);
  hipFuncSetAttribute((const void*)k_gemm2_f32<EPI_GELU_F32>, hipFuncAttributeMaxDynamicSharedMemorySize, F2_LDS);
  hipFuncSetAttribute((const void*)k_gemm2_f32<EPI_RESID_F32>, hipFuncAttributeMaxDynamicSharedMemorySize, F2_LDS);
  for (auto& sh : fshapes) {
    const int N = sh[0], K = sh[1], epi = sh[2];
    float* o = (float*)out;
    auto run = [&]() {
      if (epi == EPI_F32) gemm2_f32_launch<EPI_F32>(Af, Wf, bias, resid, o, M, N, K, 0);
      else if (epi == EPI_GELU_F32) gemm2_f32_launch<EPI_GELU_F32>(Af, Wf, bias, resid, o, M, N, K, 0);
      else gemm2_f32_launch<EPI_RESID_F32>(Af, Wf, bias, resid, o, M, N, K, 0);
    };
    run();
    hipEventRecord(e0, 0);
    for (int r = 0; r < 10; ++r) run();
    hipEventRecord(e1, 0);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    ms /= 10;
    printf("f32 k_gemm2_f32 N=%d K=%d epi=%d: %.1f us, %.1f TF/s\n", N, K, epi, ms * 1e3,
           2.0 * M * N * K / (ms * 1e-3) / 1e12);
  }
  return 0;
}
