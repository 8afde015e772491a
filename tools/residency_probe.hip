// Residency probe for gfx950 (VERDICT r04 item 1's candidate): can two
// six-wave workgroups (two ciphertexts x three GLWE components) of a 3-wave-
// per-SIMD kernel (160-168 VGPRs) share a CU? Each workgroup holds LDS_KB of
// LDS (76 KB: the slots of two ciphertexts, a quarter psi table and the
// twiddles), spins SPIN_US, and records s_memrealtime at start and end plus
// the HW_ID of every wave; the host counts, per CU, how many workgroups ran at
// once. Compared with the 12-wave (four-ciphertext, one per CU) shape. Not part
// of the product. hipcc --offload-arch=gfx950 -O3 tools/residency_probe.hip -o tools/residency_probe
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <map>
#include <vector>

#define CHK(x)                                                                   \
  do {                                                                           \
    hipError_t e = (x);                                                          \
    if (e != hipSuccess) {                                                       \
      printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__);                    \
      return 1;                                                                  \
    }                                                                            \
  } while (0)

template <int NT, int LDS_BYTES>
__global__ void __launch_bounds__(NT, NT * (163840 / LDS_BYTES) / 256) k_res(unsigned long long* rec, int spin_ticks) {
  __shared__ char lds[LDS_BYTES];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  // keep ~160 VGPRs live so the allocation is 3 waves per SIMD (as the blind rotation)
  asm volatile("v_mov_b32 v159, 0" ::: "v159");
  lds[threadIdx.x] = (char)lane;
  __syncthreads();
  while ((long long)(__builtin_amdgcn_s_memrealtime() - t0) < spin_ticks) __builtin_amdgcn_s_sleep(1);
  unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
  if (lane == 0) {
    unsigned long long* r = rec + ((size_t)blockIdx.x * (NT / 64) + w) * 4;
    r[0] = t0;
    r[1] = t1;
    r[2] = (unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 4);    // HW_ID
    r[3] = (unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 20) + lds[threadIdx.x + 1];  // XCC_ID
  }
}

template <int NT, int LDS_BYTES>
static int run(const char* name, int blocks) {
  const int waves = NT / 64;
  std::vector<unsigned long long> h((size_t)blocks * waves * 4);
  unsigned long long* d;
  CHK(hipMalloc(&d, h.size() * 8));
  const int spin = 100 * 50;  // 50 us at 100 MHz
  hipLaunchKernelGGL((k_res<NT, LDS_BYTES>), dim3(blocks), dim3(NT), 0, 0, d, spin);
  CHK(hipDeviceSynchronize());
  CHK(hipMemcpy(h.data(), d, h.size() * 8, hipMemcpyDeviceToHost));
  CHK(hipFree(d));
  // per (XCC, SE, CU): the most workgroups whose [start, end) overlap
  std::map<unsigned, std::vector<std::pair<unsigned long long, unsigned long long>>> cu;
  std::map<unsigned, int> simd_waves;
  unsigned long long tmin = ~0ull, tmax = 0;
  for (int b = 0; b < blocks; ++b) {
    const unsigned long long* r = &h[(size_t)b * waves * 4];
    const unsigned hw = (unsigned)r[2], xcc = (unsigned)r[3] & 0xf;
    const unsigned key = (xcc << 16) | ((hw >> 8) & 0xff);  // SE, SH, CU
    cu[key].push_back({r[0], r[1]});
    tmin = std::min(tmin, r[0]);
    tmax = std::max(tmax, r[1]);
    for (int w = 0; w < waves; ++w) {
      const unsigned hw2 = (unsigned)h[((size_t)b * waves + w) * 4 + 2];
      simd_waves[(hw2 >> 4) & 3]++;
    }
  }
  int maxc = 0, cus2 = 0;
  for (auto& [k, v] : cu) {
    int best = 0;
    for (auto& a : v) {
      int c = 0;
      for (auto& b : v) c += (b.first <= a.first && a.first < b.second);
      best = std::max(best, c);
    }
    maxc = std::max(maxc, best);
    cus2 += best >= 2;
  }
  printf("%-48s blocks %4d  CUs used %3zu  max concurrent WGs per CU %d  CUs with >= 2 at once %3d  span %.1f us "
         "(one WG spins 50 us)\n",
         name, blocks, cu.size(), maxc, cus2, (tmax - tmin) / 100.0);
  return 0;
}

int main() {
  run<768, 153600>("12 waves (4 cts), 150 KB LDS", 256);
  run<384, 77824>("6 waves (2 cts), 76 KB LDS", 512);
  run<384, 77824>("6 waves (2 cts), 76 KB LDS, 2 rounds", 1024);
  run<192, 38912>("3 waves (1 ct), 38 KB LDS", 1024);
  return 0;
}
