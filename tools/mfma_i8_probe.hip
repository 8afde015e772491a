// Probe the A/B lane map of v_mfma_i32_16x16x64_i8 on gfx950 with exact
// integer data. Hypothesis (by analogy with the documented bf16 16x16x32
// map): lane l holds A[row l&15][k = 16*(l>>4) + j] and B[k = 16*(l>>4) + j]
// [col l&15] in byte j = 0..15; C/D: col = l&15, row = 4*(l>>4) + reg.
// Build: hipcc --offload-arch=gfx950 -O2 -o tools/mfma_i8_probe tools/mfma_i8_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>

typedef int v4i __attribute__((ext_vector_type(4)));

__global__ void probe(const int8_t* A, const int8_t* B, int* C) {
  const int l = threadIdx.x;
  v4i a, b;
  int8_t* pa = reinterpret_cast<int8_t*>(&a);
  int8_t* pb = reinterpret_cast<int8_t*>(&b);
  for (int j = 0; j < 16; ++j) {
    pa[j] = A[(l & 15) * 64 + 16 * (l >> 4) + j];   // A[16][64] row-major
    pb[j] = B[(16 * (l >> 4) + j) * 16 + (l & 15)]; // B[64][16] row-major
  }
  v4i c = {0, 0, 0, 0};
  c = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, c, 0, 0, 0);
  for (int r = 0; r < 4; ++r) C[(4 * (l >> 4) + r) * 16 + (l & 15)] = c[r];
}

int main() {
  int8_t hA[16 * 64], hB[64 * 16];
  srand(7);
  for (int i = 0; i < 16 * 64; ++i) hA[i] = (int8_t)(rand() % 256 - 128);
  for (int i = 0; i < 64 * 16; ++i) hB[i] = (int8_t)(rand() % 256 - 128);
  int8_t *dA, *dB;
  int* dC;
  hipMalloc(&dA, sizeof hA);
  hipMalloc(&dB, sizeof hB);
  hipMalloc(&dC, 16 * 16 * 4);
  hipMemcpy(dA, hA, sizeof hA, hipMemcpyHostToDevice);
  hipMemcpy(dB, hB, sizeof hB, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, dA, dB, dC);
  int hC[256];
  hipMemcpy(hC, dC, sizeof hC, hipMemcpyDeviceToHost);
  int bad = 0;
  for (int i = 0; i < 16; ++i)
    for (int j = 0; j < 16; ++j) {
      int s = 0;
      for (int k = 0; k < 64; ++k) s += hA[i * 64 + k] * hB[k * 16 + j];
      if (s != hC[i * 16 + j]) ++bad;
    }
  printf("mfma_i32_16x16x64_i8 lane-map hypothesis: %s (%d mismatches of 256)\n", bad ? "WRONG" : "OK", bad);
  return bad != 0;
}
