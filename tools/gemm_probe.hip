// A/B probe of the BERT GEMM (fhe-icp_amd/csrc/bert.hip k_gemm) at the embed
// bench's shapes (25.6k tokens): HIP-event time per launch and TFLOP/s.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 [-DFBERT_AB_NOEPI|-DFBERT_AB_NOMFMA]
//        tools/gemm_probe.hip -o gemm_probe
#include "../fhe-icp_amd/csrc/bert.hip"

#include <cstdio>

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
  hipMemset(A, 0x3c, (size_t)M * 3072 * 2);  // bf16 ~1.1: finite, nonzero
  hipMemset(W, 0x3c, (size_t)3072 * 3072 * 2);
  hipMemset(bias, 0, 3072 * 4);
  hipMemset(resid, 0, (size_t)M * 3072 * 4);
  hipFuncSetAttribute((const void*)k_gemm<0, 256>, hipFuncAttributeMaxDynamicSharedMemorySize, gemm_lds<256>());
  hipFuncSetAttribute((const void*)k_gemm<1, 256>, hipFuncAttributeMaxDynamicSharedMemorySize, gemm_lds<256>());
  hipFuncSetAttribute((const void*)k_gemm<2, 128>, hipFuncAttributeMaxDynamicSharedMemorySize, gemm_lds<128>());
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (auto& sh : shapes) {
    const int N = sh[0], K = sh[1], epi = sh[2];
    auto run = [&]() {
      if (epi == 0) gemm_launch<0, 256>(A, W, bias, resid, out, M, N, K, 0);
      else if (epi == 1) gemm_launch<1, 256>(A, W, bias, resid, out, M, N, K, 0);
      else gemm_launch<2, 128>(A, W, bias, resid, out, M, N, K, 0);
    };
    run();
    hipEventRecord(e0, 0);
    for (int r = 0; r < 10; ++r) run();
    hipEventRecord(e1, 0);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    ms /= 10;
    printf("N=%d K=%d epi=%d: %.1f us, %.0f TF/s\n", N, K, epi, ms * 1e3, 2.0 * M * N * K / (ms * 1e-3) / 1e12);
  }
  return 0;
}
