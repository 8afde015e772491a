// libfheicp: MI355X-native TFHE engine for the encrypted pairwise compare of
// shipstone-labs/fhe-icp. C ABI in include/fhe_icp.h; design in DESIGN.md.
//
// One translation unit, so the whole engine is one gfx950 code object:
//   common.h          device helpers (modulus switch, gadget digits, test vectors)
//   k_client.h        keygen, encrypt / decrypt, seeded (stored) corpus kernels
//   k_server.h        leveled linear layer, key switch (VALU and i8 MFMA),
//                     quantisation, top-k
//   k_blind_rotate.h  blind rotation (external products over an f64 wave FFT):
//                     v4 (br_v4.h, the default hot kernel), v2/v3, v1
//   this file         context, launch selection, profiling, the C ABI
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <random>
#include <string>
#include <vector>

#include "../../include/fhe_icp.h"
#include "../../include/fhe_icp_dev.h"
#include "common.h"
#include "k_client.h"
#include "k_server.h"
#include "k_blind_rotate.h"

// ============================================================ host =========
struct ProfAcc {
  std::vector<std::pair<hipEvent_t, hipEvent_t>> ev;
  double ms = 0;
  int64_t launches = 0, items = 0;
  const char* kernel = nullptr;  // the last launched instantiation (rocprofv3's name)
};

struct fhe_ctx;
static void prof_begin(fhe_ctx* ctx, ProfAcc& a, hipStream_t st, hipEvent_t* e1);
static void prof_end(fhe_ctx* ctx, ProfAcc& a, hipStream_t st, hipEvent_t e1, int64_t items);

struct fhe_ctx {
  fhe_params p{};
  int device = -1;
  std::string err;
  bool keys = false;
  u64 *s_small = nullptr, *s_big = nullptr, *bsk = nullptr, *ksk = nullptr, *ksk_colsum = nullptr;
  c64 *bsk_fft = nullptr, *tw = nullptr, *twist = nullptr, *tw4 = nullptr;
  c64* bsk_fft_v2 = nullptr;  // v2-layout copy of the main BSK for the table bootstrap (made on first use)
  // bootstrapping keys of the other gadgets (g = 1..5: p.pbs_fast_*,
  // pbs_fast2_*, pbs_mid_*, pbs_mid2_*, pbs_mid0_*), coefficient domain and FFT form
  u64* bskf[5] = {nullptr, nullptr, nullptr, nullptr, nullptr};
  c64* bskf_fft[5] = {nullptr, nullptr, nullptr, nullptr, nullptr};
  // multi-bit blind rotation of the fast gadgets with pbs_fast*_group = 2
  // (DESIGN.md §4.5): their keys hold three GGSWs per pair of LWE
  // coefficients (messages in mb_msg); psi^x table, x < 2N (bank-swizzled)
  c64* psi = nullptr;
  u64* mb_msg = nullptr;
  int mb_dbg = 0;      // A/B builds: FHEICP_MB_DBG timing variants of the multi-bit kernel
  int v4s = 0;         // A/B builds: FHEICP_V4S=1, key-stationary v4s for the 32-bit kernels too
  // workspace
  void* ws = nullptr;
  size_t ws_bytes = 0;
  bool prof = false;
  ProfAcc prof_br, prof_brf[5], prof_ks;  // blind rotation on the main / fast / fast2 / mid / mid2 / mid0 gadget
  ProfAcc prof_enc;                       // the fused client encryption + leveled dot (k_encrypt_linear)
  int br_variant = 4;  // N=1024 blind rotation: 4 = a wave per GLWE component (k = 2, default), 2
                       // (two waves per ciphertext; forced by FHEICP_BR_VARIANT=2)
  // A/B builds only (FHEICP_AB, tools/build_variant.sh): other v4 shapes
  int v4_g = 4;        // v4 ciphertexts per workgroup (FHEICP_V4_G = 1, 2 or 4)
  int v4_fl = 0;       // v4 per-ciphertext LDS hand-offs instead of s_barrier (FHEICP_V4_FL=1)
  int v4_a64 = 0;      // v4: 64-bit accumulators even where 32 bits suffice (FHEICP_V4_A64=1)
  int v4_dbg = 0;      // timing experiments only (FHEICP_V4_DBG), wrong results
  // i8-MFMA key switch: key byte planes and a digit/body workspace
  int8_t* ksk8 = nullptr;
  void* ks_ws = nullptr;       // lane 0 (every caller stream)
  size_t ks_ws_bytes = 0;
  void* ks_ws1 = nullptr;      // lane 1: the second half of a pipelined compare
  size_t ks_ws1_bytes = 0;
  // two streams and their events for the pipelined sign extraction of
  // fhe_compare_batch (created on first use)
  hipStream_t lane_st[2] = {nullptr, nullptr};
  hipEvent_t lane_ev[3] = {nullptr, nullptr, nullptr};
  int ks_variant = 2;  // 2 = MFMA (i8 planes, any ks_level with kN % 64 == 0), 1 = VALU split-K
};

static std::mutex g_err_mu;
static std::string g_err;

static int fail(fhe_ctx* ctx, int code, const std::string& msg) {
  if (ctx) ctx->err = msg;
  std::lock_guard<std::mutex> lk(g_err_mu);
  g_err = msg;
  return code;
}
#define HIPCHK(ctx, x)                                                                          \
  do {                                                                                          \
    hipError_t e_ = (x);                                                                        \
    if (e_ != hipSuccess) return fail(ctx, FHE_E_DEVICE, std::string(#x ": ") + hipGetErrorString(e_)); \
  } while (0)

static int ilog2i(int x) {
  int r = 0;
  while ((1 << r) < x) ++r;
  return r;
}

static int validate(const fhe_params* p, std::string& why) {
  if (!p) { why = "null params"; return -1; }
  if (p->struct_size != FHE_PARAMS_SIZE) {
    why = "fhe_params.struct_size is " + std::to_string(p->struct_size) + ", this library's fhe_params has " +
          std::to_string(FHE_PARAMS_SIZE) + " bytes: the caller was built against another include/fhe_icp.h";
    return -1;
  }
  if (!(p->N == 256 || p->N == 512 || p->N == 1024 || p->N == 2048)) { why = "N must be 256/512/1024/2048"; return -1; }
  if (p->k < 1 || p->k > 2) { why = "k must be 1 or 2"; return -1; }
  if (p->N == 2048 && p->k != 1) { why = "N=2048 requires k=1"; return -1; }
  if (p->n < 1 || p->n > 4096) { why = "n out of range"; return -1; }
  if (p->pbs_level < 1 || p->pbs_level > 8 || p->pbs_base_log < 1 || p->pbs_level * p->pbs_base_log > 62) {
    why = "pbs decomposition out of range"; return -1;
  }
  if (p->ks_level < 1 || p->ks_level > 8 || p->ks_base_log < 1 || p->ks_base_log > 7 ||
      p->ks_level * p->ks_base_log + p->ks_level > 63) {
    why = "ks decomposition out of range (base_log <= 7 for int8 digits)"; return -1;
  }
  if (p->msg_bits < 2 || p->msg_bits > 40) { why = "msg_bits must be in [2, 40]"; return -1; }
  // the key switch's tie coins are input bits 62 - prec - j (j < ks_level),
  // fair only above the zero bits a shifted input brings in: the sign
  // extraction shifts by up to msg_bits - 1 (sign_rounds)
  if (p->ks_level * p->ks_base_log + p->ks_level + p->msg_bits > 64) {
    why = "ks_level * (ks_base_log + 1) + msg_bits must be <= 64 (key-switch tie coins above every shift)";
    return -1;
  }
  if (p->lwe_noise_bits < 0 || p->lwe_noise_bits > 60 || p->glwe_noise_bits < 0 || p->glwe_noise_bits > 60) {
    why = "noise bits out of range"; return -1;
  }
  if (p->sign_digit_bits != 0 && (p->sign_digit_bits < 3 || p->sign_digit_bits > 4)) {
    why = "sign_digit_bits must be 0 (auto), 3 or 4"; return -1;
  }
  if ((p->pbs_fast_base_log == 0) != (p->pbs_fast_level == 0) || p->pbs_fast_level < 0 || p->pbs_fast_level > 8 ||
      p->pbs_fast_base_log < 0 || p->pbs_fast_level * p->pbs_fast_base_log > 62) {
    why = "fast pbs decomposition out of range (0, 0 for none)"; return -1;
  }
  if ((p->pbs_fast2_base_log == 0) != (p->pbs_fast2_level == 0) || p->pbs_fast2_level < 0 ||
      p->pbs_fast2_level > 8 || p->pbs_fast2_base_log < 0 || p->pbs_fast2_level * p->pbs_fast2_base_log > 62 ||
      (p->pbs_fast2_level && !p->pbs_fast_level)) {
    why = "fast2 pbs decomposition out of range (0, 0 for none; needs a fast gadget)"; return -1;
  }
  if ((p->pbs_mid_base_log == 0) != (p->pbs_mid_level == 0) || p->pbs_mid_level < 0 || p->pbs_mid_level > 8 ||
      p->pbs_mid_base_log < 0 || p->pbs_mid_level * p->pbs_mid_base_log > 62 ||
      (p->pbs_mid_level && !p->pbs_fast_level)) {
    why = "mid pbs decomposition out of range (0, 0 for none; needs a fast gadget)"; return -1;
  }
  if ((p->pbs_mid2_base_log == 0) != (p->pbs_mid2_level == 0) || p->pbs_mid2_level < 0 ||
      p->pbs_mid2_level > 8 || p->pbs_mid2_base_log < 0 || p->pbs_mid2_level * p->pbs_mid2_base_log > 62 ||
      (p->pbs_mid2_level && !p->pbs_mid_level)) {
    why = "mid2 pbs decomposition out of range (0, 0 for none; needs the mid gadget)"; return -1;
  }
  if ((p->pbs_mid0_base_log == 0) != (p->pbs_mid0_level == 0) || p->pbs_mid0_level < 0 ||
      p->pbs_mid0_level > 8 || p->pbs_mid0_base_log < 0 || p->pbs_mid0_level * p->pbs_mid0_base_log > 62 ||
      (p->pbs_mid0_level && !p->pbs_mid_level)) {
    why = "mid0 pbs decomposition out of range (0, 0 for none; needs the mid gadget)"; return -1;
  }
  for (int g = 1; g <= 5; ++g) {
    const int grp = g == 1 ? p->pbs_fast_group : g == 2 ? p->pbs_fast2_group : g == 3 ? p->pbs_mid_group
                    : g == 4 ? p->pbs_mid2_group : p->pbs_mid0_group;
    const int L = g == 1 ? p->pbs_fast_level : g == 2 ? p->pbs_fast2_level : g == 3 ? p->pbs_mid_level
                  : g == 4 ? p->pbs_mid2_level : p->pbs_mid0_level;
    const int bl = g == 1 ? p->pbs_fast_base_log : g == 2 ? p->pbs_fast2_base_log
                   : g == 3 ? p->pbs_mid_base_log : g == 4 ? p->pbs_mid2_base_log : p->pbs_mid0_base_log;
    if (grp < 0 || grp > 2) {
      why = "pbs_fast_group / pbs_fast2_group / pbs_mid_group / pbs_mid2_group / pbs_mid0_group must be 0, 1 or 2";
      return -1;
    }
    // 32-bit accumulators when level <= 2 and level * base_log <= 31, else
    // 48-bit (k_blind_rotate_mb64), whose digits are read as 32-bit fields:
    // base_log <= 31 (a wider digit's f64 products are noise anyway)
    if (grp == 2 && L && !(p->N == 1024 && p->k == 2 && p->n <= 1023 && L <= 8 && bl <= 31)) {
      why = "multi-bit blind rotation (group 2) needs N = 1024, k = 2, n <= 1023, level <= 8, base_log <= 31";
      return -1;
    }
    // the 48-bit words keep bits 16-63: every digit field and the rounding
    // bit 2^(63 - L*beta) must lie there, so L * beta <= 47
    if (grp == 2 && L && !(L <= 2 && L * bl <= 31) && L * bl > 47) {
      why = "multi-bit blind rotation (group 2) on 48-bit accumulators needs level * base_log <= 47";
      return -1;
    }
  }
  return 0;
}

// The bootstrap gadgets of a parameter set: 0 main (pbs_base_log,
// pbs_level), 1 fast, 2 fast2, 3 mid, 4 mid2, 5 mid0 (0 levels: absent).
constexpr int NGAD = 6;
static int gadget_level(const fhe_params& p, int g) {
  switch (g) {
    case 0: return p.pbs_level;
    case 1: return p.pbs_fast_level;
    case 2: return p.pbs_fast2_level;
    case 3: return p.pbs_mid_level;
    case 4: return p.pbs_mid2_level;
    case 5: return p.pbs_mid0_level;
  }
  return 0;
}
static int gadget_base_log(const fhe_params& p, int g) {
  switch (g) {
    case 0: return p.pbs_base_log;
    case 1: return p.pbs_fast_base_log;
    case 2: return p.pbs_fast2_base_log;
    case 3: return p.pbs_mid_base_log;
    case 4: return p.pbs_mid2_base_log;
    case 5: return p.pbs_mid0_base_log;
  }
  return 0;
}
// grouping factor of gadget g's blind rotation (the main gadget is classic)
static int gadget_group(const fhe_params& p, int g) {
  const int v = g == 1 ? p.pbs_fast_group : g == 2 ? p.pbs_fast2_group : g == 3 ? p.pbs_mid_group
                : g == 4 ? p.pbs_mid2_group : g == 5 ? p.pbs_mid0_group : 1;
  return v == 2 ? 2 : 1;
}

static double tuniform_var(int b) { return (std::ldexp(1.0, 2 * b + 1) + 1.0) / 6.0; }

// Noise model, the same formulas as fheicp/params.py and
// oracle/tfhe_ref.c; variances relative to the 2^64 torus.
// Bootstrap output variance: key noise + gadget rounding + the f64 FFT's
// arithmetic error (C_FFT = 16 bounds the 11.6-13.8 measured on every kernel
// instance, tests/test_gpu_noise.py) + the 2^32 rounding of the 32-bit
// accumulators (L*beta <= 31), the last two key-weighted per step.
// The multi-bit rotation (group 2): 3x the key noise (three
// GGSWs per pair, each times X^a - 1), the same gadget rounding total, 3x the
// FFT error and half the 2^32 output roundings.
constexpr double C_FFT = 16.0;
static double pbs_var(const fhe_params& p, int beta, int L, int group = 1) {
  const double s2_bsk = tuniform_var(p.glwe_noise_bits) / std::ldexp(1.0, 128);
  const double B = std::ldexp(1.0, beta);
  const double rows = (double)L * (p.k + 1) * p.N;
  const double steps = p.n * (1 + p.k * p.N / 2.0);
  const double fft = C_FFT * rows * B * B / 144.0 * std::ldexp(1.0, -106);
  const double out32 = beta * L <= 31 ? std::ldexp(1.0, -64) / 12.0 : 0.0;
  const double km = group == 2 ? 3.0 : 1.0;
  const double arith = group == 2 ? 3.0 * fft + 0.5 * out32 : fft + out32;
  return km * p.n * rows * (B * B + 2) / 12.0 * s2_bsk + steps / (12.0 * std::pow(B, 2.0 * L)) + steps * arith;
}
// the key switch's KSK words are rounded to multiples of 2^R (k_server.h
// ks_round): R = 8 floor((lwe_noise_bits - 6) / 8), so the rounding's
// 2^R / sqrt(12) stays below 2^-7 of the KSK noise TUniform(lwe_noise_bits)
// and the i8 MFMA key switch runs on 8 - R / 8 byte planes (3 at the shipped
// lwe_noise_bits = 46; R at most 40). oracle/tfhe_ref.c ks_round_bits and
// params.ks_round_bits agree.
static int ks_round_bits(const fhe_params& p) {
  return p.lwe_noise_bits < 14 ? 0 : 8 * std::min((p.lwe_noise_bits - 6) / 8, 5);
}
// the MFMA key switch's column blocks per workgroup (k_keyswitch_mfma CB):
// three when the rounded key has at most 4 byte planes, and the 16-column
// blocks of the key planes padded to a multiple of it (zero columns)
static int ks_cb(const fhe_params& p) { return 8 - ks_round_bits(p) / 8 <= 4 ? 3 : 1; }
static int ks_nb(const fhe_params& p) {
  const int cb = ks_cb(p), nb = (p.n + 1 + KSM_NB_COLS - 1) / KSM_NB_COLS;
  return (nb + cb - 1) / cb * cb;
}
static double ks_var(const fhe_params& p) {
  const int R = ks_round_bits(p);
  const double s2_ksk = (tuniform_var(p.lwe_noise_bits) + (R ? std::ldexp(1.0, 2 * R) / 12.0 : 0.0)) /
                        std::ldexp(1.0, 128);
  const double Bk = std::ldexp(1.0, p.ks_base_log);
  return (double)p.k * p.N * p.ks_level * (Bk * Bk + 2) / 12.0 * s2_ksk +
         p.k * p.N / 2.0 * std::ldexp(1.0, -2 * p.ks_level * p.ks_base_log) / 12.0;
}
// modulus switch to 2N: one rounding per set key bit and the body (classic);
// the multi-bit rotation rounds the active subset's exponent from the exact
// sum (k_blind_rotate.h mb_rotate), one rounding per pair with a set bit
static double ms_var(const fhe_params& p, int group = 1) {
  const double per = group == 2 ? (p.n / 2) * 0.75 / 12.0 + (p.n % 2) * 0.5 / 12.0 + 1.0 / 12.0
                                : (p.n / 2.0 + 1) / 12.0;
  return per / ((2.0 * p.N) * (2.0 * p.N));
}

// Decision margin in sigmas of the worst round of a d-bit digit sign
// extraction on one gadget: the staircase round of the lowest digit, margin
// 2^-(d+1) of the torus, the preceding bootstrap's noise amplified by
// 2^(P-d), plus key switch and modulus switch noise.
static double digit_margin_sigmas(const fhe_params& p, int d) {
  const double v = pbs_var(p, p.pbs_base_log, p.pbs_level) * std::ldexp(1.0, 2 * (p.msg_bits - d)) + ks_var(p) +
                   ms_var(p);
  return std::ldexp(1.0, -(d + 1)) / std::sqrt(v);
}

// The bootstraps of fhe_sign_batch in order, as (shift, log2 margin): the
// round reads v << shift, and every earlier bootstrap output subtracted from
// v is amplified by 2^shift.
static int sign_rounds(int P, int d, int* shift, int* mlog) {
  int R = 0, b = 0;
  const int m = P - d;
  auto add = [&](int sh, int ml) { shift[R] = sh; mlog[R] = ml; ++R; };
  for (; b + d <= m; b += d) { add(P - b - d, -(d + 1)); add(P - b - d, -(d + 1)); }
  if (m - b >= 3) { const int c = m - b; add(P - b - c, -(c + 1)); add(P - b - c, -(c + 1)); b = m; }
  for (; b < m; ++b) add(P - b - 1, -2);
  add(0, -(d + 1));
  return R;
}
// worst margin (sigmas) over all R rounds when round r runs on gadget sched[r]
static double plan_worst(const fhe_params& p, int d, const int* sched) {
  int sh[64], ml[64];
  const int R = sign_rounds(p.msg_bits, d, sh, ml);
  double var[NGAD];
  for (int g = 0; g < NGAD; ++g)
    var[g] = gadget_level(p, g) ? pbs_var(p, gadget_base_log(p, g), gadget_level(p, g), gadget_group(p, g)) : 0.0;
  double fixed[NGAD];  // key switch + the modulus switch of each gadget's rotation
  for (int g = 0; g < NGAD; ++g) fixed[g] = ks_var(p) + ms_var(p, gadget_group(p, g));
  double acc = 0, worst = 1e300;
  for (int r = 0; r < R; ++r) {
    worst = std::min(worst, std::ldexp(1.0, ml[r]) / std::sqrt(acc * std::ldexp(1.0, 2 * sh[r]) + fixed[sched[r]]));
    acc += var[sched[r]];
  }
  // the last bootstrap's output is the sign ciphertext: decryptable at 1/4
  return std::min(worst, 0.25 / std::sqrt(var[sched[R - 1]]));
}
// The sign plan: digit width d and the gadget of every
// bootstrap (sched[0..R), returns R). Without a fast gadget: the
// single-gadget rule (d = 4 if its worst round keeps 9.2 sigma, else 3), all
// rounds on the main gadget. With fast gadgets: the widest d (or the forced
// one); then along the ladder main, mid0, mid, mid2, fast, fast2 (those present,
// noisier down the ladder) each gadget takes the fewest leading rounds for
// which the next gadget on all the remaining ones keeps every decision at 9.2
// sigma; the last one takes the rest.
static int sign_schedule(const fhe_params& p, int* d_out, int* sched) {
  int sh[64], ml[64];
  const int P = p.msg_bits;
  if (P < 4) {
    *d_out = 0;
    for (int r = 0; r < P; ++r) sched[r] = 0;
    return P;
  }
  auto all_main = [&](int d) {
    const int R = sign_rounds(P, d, sh, ml);
    for (int r = 0; r < R; ++r) sched[r] = 0;
    *d_out = d;
    return R;
  };
  if (!p.pbs_fast_level) {
    int d = 3;
    if (p.sign_digit_bits) d = std::min(p.sign_digit_bits, P);
    else if (digit_margin_sigmas(p, std::min(4, P)) >= 9.2) d = std::min(4, P);
    return all_main(d);
  }
  int lad[NGAD], m = 0;
  lad[m++] = 0;
  for (int g : {5, 3, 4, 1, 2})
    if (gadget_level(p, g)) lad[m++] = g;
  const int first = p.sign_digit_bits ? std::min(p.sign_digit_bits, P) : std::min(4, P);
  const int last = p.sign_digit_bits ? first : 3;
  for (int d = first; d >= last; --d) {
    const int R = sign_rounds(P, d, sh, ml);
    int start = 0;
    bool ok = true;
    for (int i = 0; i + 1 < m; ++i) {
      int c = start;
      for (; c <= R; ++c) {
        for (int r = start; r < R; ++r) sched[r] = r < c ? lad[i] : lad[i + 1];
        if (plan_worst(p, d, sched) >= 9.2) break;
      }
      if (c > R) {  // only when the main gadget alone cannot: a narrower d
        ok = false;
        break;
      }
      start = c;
    }
    if (ok) {
      *d_out = d;
      return R;
    }
  }
  return all_main(last);
}
// (d, j1, j2): digit width, the leading main-gadget rounds and the first
// fast2 round (R without one) of sign_schedule
static void sign_plan(const fhe_params& p, int* d_out, int* j1_out, int* j2_out) {
  int sched[64];
  const int R = sign_schedule(p, d_out, sched);
  int j1 = 0, j2 = R;
  while (j1 < R && sched[j1] == 0) ++j1;
  while (j2 > 0 && sched[j2 - 1] == 2) --j2;
  *j1_out = j1;
  *j2_out = j2;
}
static int sign_digits(const fhe_params& p) {
  int d, j1, j2;
  sign_plan(p, &d, &j1, &j2);
  return d;
}

extern "C" {

size_t fhe_bsk_words(const fhe_params* p) {
  return (size_t)p->n * (p->k + 1) * p->pbs_level * (p->k + 1) * p->N;
}
size_t fhe_ksk_words(const fhe_params* p) { return (size_t)p->k * p->N * p->ks_level * (p->n + 1); }
size_t fhe_big_lwe_words(const fhe_params* p) { return (size_t)p->k * p->N + 1; }
size_t fhe_small_lwe_words(const fhe_params* p) { return (size_t)p->n + 1; }

const char* fhe_last_error(const fhe_ctx* ctx) {
  if (ctx) return ctx->err.c_str();
  std::lock_guard<std::mutex> lk(g_err_mu);
  return g_err.c_str();
}

int fhe_get_params(const fhe_ctx* ctx, fhe_params* out) {
  if (!ctx || !out) return FHE_E_ARG;
  *out = ctx->p;
  return FHE_OK;
}

int fhe_ctx_create(const fhe_params* params, int device, fhe_ctx** out) {
  std::string why;
  if (!out) return fail(nullptr, FHE_E_ARG, "out is null");
  *out = nullptr;
  if (validate(params, why)) return fail(nullptr, FHE_E_ARG, why);
  fhe_ctx* ctx = new fhe_ctx();
  ctx->p = *params;
  ctx->device = device;
  if (const char* e = getenv("FHEICP_BR_VARIANT")) {
    const int v = atoi(e);
    ctx->br_variant = (v == 2 || v == 4) ? v : 4;
  }
#ifdef FHEICP_AB
  if (const char* e = getenv("FHEICP_V4_DBG")) ctx->v4_dbg = atoi(e);
  if (const char* e = getenv("FHEICP_V4_G")) {
    const int g = atoi(e);
    ctx->v4_g = (g == 1 || g == 2 || g == 4) ? g : 4;
  }
  if (const char* e = getenv("FHEICP_V4_FL")) ctx->v4_fl = atoi(e) != 0;
  if (const char* e = getenv("FHEICP_V4_A64")) ctx->v4_a64 = atoi(e) != 0;
  if (const char* e = getenv("FHEICP_MB_DBG")) ctx->mb_dbg = atoi(e);
  if (const char* e = getenv("FHEICP_V4S")) ctx->v4s = atoi(e);
#endif
  if (const char* e = getenv("FHEICP_KS_VARIANT")) ctx->ks_variant = atoi(e) == 1 ? 1 : 2;
  // the MFMA key switch: digits in i8, K = kN * ks_level level-major in
  // 64-blocks, |sum| <= K * 2^(beta-1) * 128 < 2^31 in the i32 accumulators
  if ((params->k * params->N) % 64 != 0 || params->ks_level * params->ks_base_log > 31 ||
      params->ks_base_log > 8 ||
      (double)params->k * params->N * params->ks_level * std::ldexp(1.0, params->ks_base_log - 1) * 128 >= 2147483648.0)
    ctx->ks_variant = 1;
  // v4 covers k = 2, n <= 1023 at N = 1024; otherwise the two-wave kernel
  // (measured: v4 wins at gadget levels <= 3, e.g. 21.6 vs 23.6 ms at P=21; from
  // level 4 its 64-bit accumulator spills and v2 is faster, 40.6 vs 53.0 ms at P=26)
  // (the choice is per gadget: variant_for)
  if (device >= 0) {
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device >= ndev) {
      delete ctx;
      return fail(nullptr, FHE_E_DEVICE, "no HIP device " + std::to_string(device));
    }
    if (hipSetDevice(device) != hipSuccess) {
      delete ctx;
      return fail(nullptr, FHE_E_DEVICE, "hipSetDevice failed");
    }
    const int N = params->N, M = N / 2;
    std::vector<c64> tw(M / 2), twist(M);
    for (int x = 0; x < M / 2; ++x) {
      const long double ang = 2.0L * 3.14159265358979323846264338327950288L * (long double)x / (long double)M;
      tw[x] = {(double)cosl(ang), (double)sinl(ang)};
    }
    for (int t = 0; t < M; ++t) {
      const long double ang = 3.14159265358979323846264338327950288L * (long double)t / (long double)N;
      twist[t] = {(double)cosl(ang), (double)sinl(ang)};
    }
    if (N == 1024) {  // v4 per-lane twiddles (br_v4.h), long double
      const long double PI = 3.14159265358979323846264338327950288L;
      std::vector<c64> t4(v4::NTW);
      for (int m = 0; m < 8; ++m)
        for (int lane = 0; lane < 64; ++lane) {
          const long double ang = PI * (long double)lane * (long double)(1 + 4 * m) / 1024.0L;
          t4[m * 64 + lane] = {(double)cosl(ang), (double)sinl(ang)};
        }
      for (int m = 1; m < 8; ++m)
        for (int L = 0; L < 8; ++L) {
          const long double ang = 2.0L * PI * (long double)(L * m) / 64.0L;
          t4[v4::NTA + (m - 1) * 8 + L] = {(double)cosl(ang), (double)sinl(ang)};
        }
      // psi^x - 1, psi = exp(i pi / N), x < 2N: the monomial factors of the multi-bit rotation
      std::vector<c64> ps(2 * N);
      for (int x = 0; x < 2 * N; ++x) {
        const long double ang = PI * (long double)x / (long double)N;
        // psi^x - 1, the factor the products take (cos - 1 = -2 sin^2),
        // bank-swizzled (k_blind_rotate_mb)
        const long double h = sinl(ang / 2);
        ps[mb::psi_pos(x)] = {(double)(-2.0L * h * h), (double)sinl(ang)};
      }
      if (hipMalloc(&ctx->tw4, sizeof(c64) * t4.size()) != hipSuccess ||
          hipMemcpy(ctx->tw4, t4.data(), sizeof(c64) * t4.size(), hipMemcpyHostToDevice) != hipSuccess ||
          hipMalloc(&ctx->psi, sizeof(c64) * ps.size()) != hipSuccess ||
          hipMemcpy(ctx->psi, ps.data(), sizeof(c64) * ps.size(), hipMemcpyHostToDevice) != hipSuccess) {
        fhe_ctx_destroy(ctx);
        return fail(nullptr, FHE_E_DEVICE, "twiddle upload failed");
      }
    }
    if (hipMalloc(&ctx->tw, sizeof(c64) * tw.size()) != hipSuccess ||
        hipMalloc(&ctx->twist, sizeof(c64) * twist.size()) != hipSuccess ||
        hipMemcpy(ctx->tw, tw.data(), sizeof(c64) * tw.size(), hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(ctx->twist, twist.data(), sizeof(c64) * twist.size(), hipMemcpyHostToDevice) != hipSuccess) {
      fhe_ctx_destroy(ctx);
      return fail(nullptr, FHE_E_DEVICE, "table upload failed");
    }
  }
  *out = ctx;
  return FHE_OK;
}

static void free_ev(ProfAcc& a) {
  for (auto& e : a.ev) {
    (void)hipEventDestroy(e.first);
    (void)hipEventDestroy(e.second);
  }
  a.ev.clear();
}

void fhe_ctx_destroy(fhe_ctx* ctx) {
  if (!ctx) return;
  if (ctx->device >= 0) {
    // teardown: nothing useful can be done about a failed free
    (void)hipSetDevice(ctx->device);
    for (void* ptr : {(void*)ctx->s_small, (void*)ctx->s_big, (void*)ctx->bsk, (void*)ctx->ksk,
                      (void*)ctx->ksk_colsum, (void*)ctx->bsk_fft, (void*)ctx->tw, (void*)ctx->twist, ctx->ws,
                      (void*)ctx->bskf[0], (void*)ctx->bskf[1], (void*)ctx->bskf_fft[0], (void*)ctx->bskf_fft[1],
                      (void*)ctx->bskf[2], (void*)ctx->bskf[3], (void*)ctx->bskf_fft[2], (void*)ctx->bskf_fft[3],
                      (void*)ctx->bskf[4], (void*)ctx->bskf_fft[4],
                      (void*)ctx->ksk8, (void*)ctx->ks_ws, (void*)ctx->ks_ws1, (void*)ctx->tw4, (void*)ctx->bsk_fft_v2,
                      (void*)ctx->psi, (void*)ctx->mb_msg})
      (void)hipFree(ptr);
    for (hipStream_t s : ctx->lane_st)
      if (s) (void)hipStreamDestroy(s);
    for (hipEvent_t e : ctx->lane_ev)
      if (e) (void)hipEventDestroy(e);
    free_ev(ctx->prof_br);
    for (auto& a : ctx->prof_brf) free_ev(a);
    free_ev(ctx->prof_ks);
    free_ev(ctx->prof_enc);
  }
  delete ctx;
}

int fhe_set_msg_bits(fhe_ctx* ctx, int32_t msg_bits) {
  if (!ctx) return fail(nullptr, FHE_E_ARG, "null ctx");
  fhe_params q = ctx->p;
  q.msg_bits = msg_bits;
  std::string why;
  if (validate(&q, why)) return fail(ctx, FHE_E_ARG, why);
  ctx->p = q;
  return FHE_OK;
}

static int need_device(fhe_ctx* ctx) {
  if (!ctx) return fail(nullptr, FHE_E_ARG, "null ctx");
  if (ctx->device < 0) return fail(ctx, FHE_E_DEVICE, "host-only context");
  if (hipSetDevice(ctx->device) != hipSuccess) return fail(ctx, FHE_E_DEVICE, "hipSetDevice failed");
  return FHE_OK;
}
static int need_keys(fhe_ctx* ctx) {
  int rc = need_device(ctx);
  if (rc) return rc;
  if (!ctx->keys) return fail(ctx, FHE_E_STATE, "no keys: call fhe_keygen or fhe_import_keys");
  return FHE_OK;
}

// blind-rotation kernel for a gadget: the requested variant (4 unless
// FHEICP_BR_VARIANT), falling back to v2 where v4 does not apply
// the v4 kernel keeps 32-bit accumulators for this gadget
// (the shipped 32-bit kernels exist for levels 1 and 2 only: a level-3
// gadget with L*beta <= 31, e.g. (10,3), runs on the 64-bit v4s<3> kernel,
// whose noise the model's 2^32 rounding term then over-counts)
static bool v4_a32(const fhe_ctx* ctx, const fhe_params& q) {
  return q.pbs_level <= 2 && q.pbs_level * q.pbs_base_log <= 31 && !ctx->v4_a64;
}

static int variant_for(const fhe_ctx* ctx, const fhe_params& q) {
  // v4 layout: the v4 kernels (32-bit accumulators, L <= 2) and the v4s
  // ones (64-bit accumulators, L <= 8)
  const int lmax = v4_a32(ctx, q) ? 2 : 8;
  if (ctx->br_variant == 4 &&
      !(q.k == 2 && q.n <= v4::NMAX && q.pbs_level <= lmax && (q.pbs_level == 1 || q.pbs_base_log <= 16)))
    return 2;
  return ctx->br_variant;
}
// the parameters seen through gadget g (1: pbs_fast_*, 2: pbs_fast2_*, 3:
// pbs_mid_*, 4: pbs_mid2_*, 5: pbs_mid0_*; same secret keys, other decomposition and
// bootstrapping key)
static int fast_level(const fhe_params& p, int g) { return g >= 1 && g < NGAD ? gadget_level(p, g) : 0; }
// fast gadget g runs the multi-bit blind rotation
static bool mb_for(const fhe_params& p, int g) { return g > 0 && fast_level(p, g) && gadget_group(p, g) == 2; }
static fhe_params fast_params(const fhe_params& p, int g) {
  fhe_params q = p;
  q.pbs_base_log = gadget_base_log(p, g);
  q.pbs_level = fast_level(p, g);
  return q;
}
// GGSWs of a fast gadget's key: one per LWE coefficient, or three per pair
static int fast_ggsws(const fhe_params& p, int g) { return mb_for(p, g) ? 3 * ((p.n + 1) / 2) : p.n; }
static size_t fast_bsk_words(const fhe_params& p, int g) {
  return (size_t)fast_ggsws(p, g) * (p.k + 1) * fast_level(p, g) * (p.k + 1) * p.N;
}
size_t fhe_fast_bsk_words(const fhe_params* p, int32_t which) {
  if (!p || which < 1 || which >= NGAD || !fast_level(*p, which)) return 0;
  return fast_bsk_words(*p, which);
}
// the other gadgets' keys under the ChaCha20 streams 9/10 (fast), 11/12
// (fast2), 17/18 (mid), 19/20 (mid2) and 25/26 (mid0); 13/14, 15/16, 21/22,
// 23/24 and 27/28 for those gadgets' multi-bit keys, whose GGSW messages
// k_mb_msgs derives
static const uint32_t kTagMask[NGAD] = {TAG_BSK_MASK, TAG_BSK2_MASK, TAG_BSK3_MASK, TAG_BSK4_MASK, TAG_BSK5_MASK,
                                        TAG_BSK6_MASK};
static const uint32_t kTagNoise[NGAD] = {TAG_BSK_NOISE, TAG_BSK2_NOISE, TAG_BSK3_NOISE, TAG_BSK4_NOISE, TAG_BSK5_NOISE,
                                         TAG_BSK6_NOISE};
static const uint32_t kTagMbMask[NGAD] = {0, TAG_MB2_MASK, TAG_MB3_MASK, TAG_MB4_MASK, TAG_MB5_MASK, TAG_MB6_MASK};
static const uint32_t kTagMbNoise[NGAD] = {0, TAG_MB2_NOISE, TAG_MB3_NOISE, TAG_MB4_NOISE, TAG_MB5_NOISE, TAG_MB6_NOISE};
static void keygen_fast_bsks(fhe_ctx* ctx, const ChaKey& K, hipStream_t st) {
  const fhe_params& p = ctx->p;
  const size_t shm = 8 * (size_t)p.N + p.N;
  for (int g = 1; g < NGAD; ++g) {
    if (!fast_level(p, g)) continue;
    const fhe_params q = fast_params(p, g);
    const bool mb = mb_for(p, g);
    if (mb) hipLaunchKernelGGL(k_mb_msgs, dim3((q.n + 255) / 256), dim3(256), 0, st, ctx->s_small, q.n, ctx->mb_msg);
    hipLaunchKernelGGL(k_keygen_bsk, dim3(fast_ggsws(p, g) * (q.k + 1) * q.pbs_level), dim3(256), shm, st, K, q.N,
                       q.k, q.pbs_level, q.pbs_base_log, q.glwe_noise_bits, mb ? ctx->mb_msg : ctx->s_small,
                       ctx->s_big, ctx->bskf[g - 1],
                       mb ? kTagMbMask[g] : kTagMask[g], mb ? kTagMbNoise[g] : kTagNoise[g]);
  }
}
static int alloc_keys(fhe_ctx* ctx) {
  const fhe_params& p = ctx->p;
  for (int g = 1; g < NGAD; ++g) {
    if (!fast_level(p, g) || ctx->bskf[g - 1]) continue;
    const fhe_params q = fast_params(p, g);
    HIPCHK(ctx, hipMalloc(&ctx->bskf[g - 1], 8 * fast_bsk_words(p, g)));
    HIPCHK(ctx, hipMalloc(&ctx->bskf_fft[g - 1], sizeof(c64) * fast_bsk_words(p, g) / 2));
    if (mb_for(p, g) && !ctx->mb_msg) HIPCHK(ctx, hipMalloc(&ctx->mb_msg, 8 * 3 * (size_t)((q.n + 1) / 2)));
  }
  if (ctx->s_small) return FHE_OK;
  HIPCHK(ctx, hipMalloc(&ctx->s_small, 8 * (size_t)p.n));
  HIPCHK(ctx, hipMalloc(&ctx->s_big, 8 * (size_t)p.k * p.N));
  HIPCHK(ctx, hipMalloc(&ctx->bsk, 8 * fhe_bsk_words(&p)));
  HIPCHK(ctx, hipMalloc(&ctx->ksk, 8 * fhe_ksk_words(&p)));
  HIPCHK(ctx, hipMalloc(&ctx->ksk_colsum, 8 * (size_t)(p.n + 1)));
  HIPCHK(ctx, hipMalloc(&ctx->bsk_fft, sizeof(c64) * fhe_bsk_words(&p) / 2));
  return FHE_OK;
}

static void bsk_to_fft(fhe_ctx* ctx, const fhe_params& p, const u64* bsk, c64* bsk_fft, hipStream_t st,
                       size_t words = 0) {
  const int npoly = (int)((words ? words : fhe_bsk_words(&p)) / p.N);
  switch (p.N) {
    case 256: hipLaunchKernelGGL(k_bsk_to_fft<7>, dim3(npoly), dim3(64), 0, st, bsk, npoly, ctx->tw, ctx->twist, bsk_fft); break;
    case 512: hipLaunchKernelGGL(k_bsk_to_fft<8>, dim3(npoly), dim3(64), 0, st, bsk, npoly, ctx->tw, ctx->twist, bsk_fft); break;
    case 1024:
      if (variant_for(ctx, p) == 4 || words)
        hipLaunchKernelGGL(k_bsk_to_fft_v4, dim3(std::min(npoly, 4096)), dim3(64), 0, st, bsk, npoly, ctx->tw4,
                           bsk_fft, 1.0 / 18446744073709551616.0 / (double)(p.N / 2), words && mb_xpose(p.pbs_level) ? 1 : 0);
      else
        hipLaunchKernelGGL(k_bsk_to_fft_mw<V2>, dim3(npoly), dim3(V2::NT), 0, st, bsk, npoly, ctx->tw, ctx->twist, bsk_fft);
      break;
    case 2048: hipLaunchKernelGGL(k_bsk_to_fft<10>, dim3(npoly), dim3(64), 0, st, bsk, npoly, ctx->tw, ctx->twist, bsk_fft); break;
  }
}
static int convert_bsk(fhe_ctx* ctx, hipStream_t st) {
  const fhe_params& p = ctx->p;
  if (ctx->bsk_fft_v2) {  // the table bootstrap's copy of the old key
    HIPCHK(ctx, hipDeviceSynchronize());
    HIPCHK(ctx, hipFree(ctx->bsk_fft_v2));
    ctx->bsk_fft_v2 = nullptr;
  }
  const int R = ks_round_bits(p);
  hipLaunchKernelGGL(k_ksk_colsum, dim3((p.n + 1 + 255) / 256), dim3(256), 0, st, ctx->ksk, p.k * p.N * p.ks_level,
                     p.n, R, ctx->ksk_colsum);
  if (ctx->ks_variant == 2) {
    const int K = p.k * p.N * p.ks_level, n1 = p.n + 1, NB = ks_nb(p);
    if (!ctx->ksk8) HIPCHK(ctx, hipMalloc(&ctx->ksk8, (size_t)K * NB * 16 * (8 - R / 8)));
    const int64_t tot = (int64_t)K * NB * 16;
    hipLaunchKernelGGL(k_ksk_to_i8, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, st, ctx->ksk, K, p.k * p.N,
                       p.ks_level, n1, NB, R, 8 - R / 8, ctx->ksk8);
  }
  bsk_to_fft(ctx, p, ctx->bsk, ctx->bsk_fft, st);
  for (int g = 1; g < NGAD; ++g)
    if (fast_level(p, g))
      bsk_to_fft(ctx, fast_params(p, g), ctx->bskf[g - 1], ctx->bskf_fft[g - 1], st,
                 mb_for(p, g) ? fast_bsk_words(p, g) : 0);
  HIPCHK(ctx, hipGetLastError());
  return FHE_OK;
}

int fhe_keygen_key(fhe_ctx* ctx, const uint32_t h_key[8], void* stream) {
  int rc = need_device(ctx);
  if (rc) return rc;
  if (!h_key) return fail(ctx, FHE_E_ARG, "null key");
  rc = alloc_keys(ctx);
  if (rc) return rc;
  const fhe_params& p = ctx->p;
  hipStream_t st = (hipStream_t)stream;
  ChaKey K;
  memcpy(K.w, h_key, 32);
  const int big = p.k * p.N;
  const int mx = std::max(p.n, big);
  hipLaunchKernelGGL(k_keygen_secrets, dim3((mx + 255) / 256), dim3(256), 0, st, K, p.n, big, ctx->s_small, ctx->s_big);
  const int rows_bsk = p.n * (p.k + 1) * p.pbs_level;
  const size_t shm = 8 * (size_t)p.N + p.N;
  hipLaunchKernelGGL(k_keygen_bsk, dim3(rows_bsk), dim3(256), shm, st, K, p.N, p.k, p.pbs_level, p.pbs_base_log,
                     p.glwe_noise_bits, ctx->s_small, ctx->s_big, ctx->bsk, (uint32_t)TAG_BSK_MASK,
                     (uint32_t)TAG_BSK_NOISE);
  keygen_fast_bsks(ctx, K, st);
  hipLaunchKernelGGL(k_keygen_ksk, dim3(big * p.ks_level), dim3(256), 0, st, K, p.n, p.ks_level, p.ks_base_log,
                     p.lwe_noise_bits, ctx->s_small, ctx->s_big, ctx->ksk);
  HIPCHK(ctx, hipGetLastError());
  rc = convert_bsk(ctx, st);
  if (rc) return rc;
  HIPCHK(ctx, hipStreamSynchronize(st));
  ctx->keys = true;
  return FHE_OK;
}

int fhe_keygen(fhe_ctx* ctx, uint64_t seed, void* stream) {
  ChaKey K = key_from_seed(seed);
  return fhe_keygen_key(ctx, K.w, stream);
}

int fhe_export_keys(fhe_ctx* ctx, uint64_t* h_s_small, uint64_t* h_s_big, uint64_t* h_bsk, uint64_t* h_ksk) {
  int rc = need_keys(ctx);
  if (rc) return rc;
  const fhe_params& p = ctx->p;
  HIPCHK(ctx, hipDeviceSynchronize());
  if (h_s_small) HIPCHK(ctx, hipMemcpy(h_s_small, ctx->s_small, 8 * (size_t)p.n, hipMemcpyDeviceToHost));
  if (h_s_big) HIPCHK(ctx, hipMemcpy(h_s_big, ctx->s_big, 8 * (size_t)p.k * p.N, hipMemcpyDeviceToHost));
  if (h_bsk) HIPCHK(ctx, hipMemcpy(h_bsk, ctx->bsk, 8 * fhe_bsk_words(&p), hipMemcpyDeviceToHost));
  if (h_ksk) HIPCHK(ctx, hipMemcpy(h_ksk, ctx->ksk, 8 * fhe_ksk_words(&p), hipMemcpyDeviceToHost));
  return FHE_OK;
}

int fhe_export_fast_bsk(fhe_ctx* ctx, int32_t which, uint64_t* h_bsk) {
  int rc = need_keys(ctx);
  if (rc) return rc;
  if (which < 1 || which >= NGAD)
    return fail(ctx, FHE_E_ARG, "which must be 1 (fast), 2 (fast2), 3 (mid), 4 (mid2) or 5 (mid0)");
  if (!fast_level(ctx->p, which)) return fail(ctx, FHE_E_STATE, "no such fast gadget in these parameters");
  if (!h_bsk) return fail(ctx, FHE_E_ARG, "null buffer");
  const fhe_params q = fast_params(ctx->p, which);
  HIPCHK(ctx, hipDeviceSynchronize());
  HIPCHK(ctx, hipMemcpy(h_bsk, ctx->bskf[which - 1], 8 * fast_bsk_words(ctx->p, which), hipMemcpyDeviceToHost));
  return FHE_OK;
}

int fhe_import_keys(fhe_ctx* ctx, const uint64_t* h_s_small, const uint64_t* h_s_big, const uint64_t* h_bsk,
                    const uint64_t* h_ksk) {
  int rc = need_device(ctx);
  if (rc) return rc;
  if (!h_s_small || !h_s_big || !h_bsk || !h_ksk) return fail(ctx, FHE_E_ARG, "all four key buffers are required");
  rc = alloc_keys(ctx);
  if (rc) return rc;
  const fhe_params& p = ctx->p;
  HIPCHK(ctx, hipMemcpy(ctx->s_small, h_s_small, 8 * (size_t)p.n, hipMemcpyHostToDevice));
  HIPCHK(ctx, hipMemcpy(ctx->s_big, h_s_big, 8 * (size_t)p.k * p.N, hipMemcpyHostToDevice));
  HIPCHK(ctx, hipMemcpy(ctx->bsk, h_bsk, 8 * fhe_bsk_words(&p), hipMemcpyHostToDevice));
  HIPCHK(ctx, hipMemcpy(ctx->ksk, h_ksk, 8 * fhe_ksk_words(&p), hipMemcpyHostToDevice));
  if (p.pbs_fast_level) {
    // the fast gadgets' keys are not part of the exported set: re-encrypt
    // them under the imported secrets with fresh randomness
    ChaKey K;
    std::random_device rd;
    for (int i = 0; i < 8; ++i) K.w[i] = rd();
    keygen_fast_bsks(ctx, K, nullptr);
    HIPCHK(ctx, hipGetLastError());
  }
  rc = convert_bsk(ctx, nullptr);
  if (rc) return rc;
  HIPCHK(ctx, hipDeviceSynchronize());
  ctx->keys = true;
  return FHE_OK;
}

// The encryption entry points take the stream key either as 32 bytes
// (fhe_*_key: the product, a fresh CSPRNG key per session) or as a 64-bit
// seed expanded by splitmix64 (reproducible tests and benches only).
static bool key_arg(const uint32_t* h_key, ChaKey& K) {
  if (!h_key) return false;
  memcpy(K.w, h_key, 32);
  return true;
}

static int encrypt_impl(fhe_ctx* ctx, const int64_t* d_msg, int64_t count, const ChaKey& K, uint64_t id0,
                        uint64_t* d_ct, void* stream) {
  int rc = need_keys(ctx);
  if (rc) return rc;
  if (count < 0 || (count > 0 && (!d_msg || !d_ct))) return fail(ctx, FHE_E_ARG, "bad encrypt arguments");
  if (count == 0) return FHE_OK;
  const fhe_params& p = ctx->p;
  hipLaunchKernelGGL(k_encrypt, dim3((unsigned)count), dim3(256), 0, (hipStream_t)stream, K, p.k * p.N, p.msg_bits,
                     p.glwe_noise_bits, ctx->s_big, d_msg, id0, d_ct);
  HIPCHK(ctx, hipGetLastError());
  return FHE_OK;
}
int fhe_encrypt_batch(fhe_ctx* ctx, const int64_t* d_msg, int64_t count, uint64_t seed, uint64_t id0,
                      uint64_t* d_ct, void* stream) {
  return encrypt_impl(ctx, d_msg, count, key_from_seed(seed), id0, d_ct, stream);
}
int fhe_encrypt_batch_key(fhe_ctx* ctx, const int64_t* d_msg, int64_t count, const uint32_t h_key[8], uint64_t id0,
                          uint64_t* d_ct, void* stream) {
  ChaKey K;
  if (!key_arg(h_key, K)) return fail(ctx, FHE_E_ARG, "null encryption key");
  return encrypt_impl(ctx, d_msg, count, K, id0, d_ct, stream);
}

// GLWEs per pair of the packed feature encoding (k_client.h)
static int packed_chunks(const fhe_params& p, int32_t D) { return (D + p.N - 1) / p.N; }

static int encrypt_packed_impl(fhe_ctx* ctx, const int64_t* d_qx, int64_t B, int32_t D, const ChaKey& K,
                               uint64_t id0, uint64_t* d_glwe, void* stream) {
  int rc = need_keys(ctx);
  if (rc) return rc;
  if (B < 0 || D <= 0 || (B > 0 && (!d_qx || !d_glwe))) return fail(ctx, FHE_E_ARG, "bad packed-encrypt arguments");
  if (B == 0) return FHE_OK;
  const fhe_params& p = ctx->p;
  const int G = packed_chunks(p, D);
  if (B * G > 0x7fffffffLL) return fail(ctx, FHE_E_ARG, "packed-encrypt batch too large: split the call");
  const size_t lds = (size_t)p.k * p.N * 9;
  hipLaunchKernelGGL(k_encrypt_packed, dim3((unsigned)(B * G)), dim3(256), lds, (hipStream_t)stream, K, p.N, p.k,
                     p.msg_bits, p.glwe_noise_bits, ctx->s_big, d_qx, (int)D, G, id0, d_glwe);
  HIPCHK(ctx, hipGetLastError());
  return FHE_OK;
}
int fhe_encrypt_packed_batch(fhe_ctx* ctx, const int64_t* d_qx, int64_t B, int32_t D, uint64_t seed, uint64_t id0,
                             uint64_t* d_glwe, void* stream) {
  return encrypt_packed_impl(ctx, d_qx, B, D, key_from_seed(seed), id0, d_glwe, stream);
}
int fhe_encrypt_packed_batch_key(fhe_ctx* ctx, const int64_t* d_qx, int64_t B, int32_t D, const uint32_t h_key[8],
                                 uint64_t id0, uint64_t* d_glwe, void* stream) {
  ChaKey K;
  if (!key_arg(h_key, K)) return fail(ctx, FHE_E_ARG, "null encryption key");
  return encrypt_packed_impl(ctx, d_qx, B, D, K, id0, d_glwe, stream);
}

int fhe_linear_packed_batch(fhe_ctx* ctx, const uint64_t* d_glwe, int64_t B, int32_t D, const int64_t* d_w,
                            int64_t cst, uint64_t* d_out, void* stream) {
  int rc = need_device(ctx);
  if (rc) return rc;
  if (B < 0 || D <= 0 || (B > 0 && (!d_glwe || !d_w || !d_out))) return fail(ctx, FHE_E_ARG, "bad packed-linear arguments");
  if (B == 0) return FHE_OK;
  if (B > 0x7fffffffLL) return fail(ctx, FHE_E_ARG, "packed-linear batch too large: split the call");
  const fhe_params& p = ctx->p;
  hipLaunchKernelGGL(k_linear_packed, dim3((unsigned)B), dim3(256), (size_t)p.k * p.N * 8, (hipStream_t)stream, p.N,
                     p.k, d_glwe, (int)D, packed_chunks(p, D), d_w, ((u64)cst) << (64 - p.msg_bits), d_out);
  HIPCHK(ctx, hipGetLastError());
  return FHE_OK;
}

static int encrypt_linear_impl(fhe_ctx* ctx, const int64_t* d_qx, int64_t B, int32_t D, const ChaKey& K,
                               uint64_t id0, const int64_t* d_w, int64_t cst, uint64_t* d_out, void* stream) {
  int rc = need_keys(ctx);
  if (rc) return rc;
  if (B < 0 || D <= 0 || (B > 0 && (!d_qx || !d_w || !d_out))) return fail(ctx, FHE_E_ARG, "bad encrypt-linear arguments");
  if (B == 0) return FHE_OK;
  const fhe_params& p = ctx->p;
  const int G = packed_chunks(p, D);
  if (B > 0x7fffffffLL || B * G > 0x7fffffffffffLL) return fail(ctx, FHE_E_ARG, "encrypt-linear batch too large: split the call");
  hipEvent_t e1;
  prof_begin(ctx, ctx->prof_enc, (hipStream_t)stream, &e1);
  ctx->prof_enc.kernel = "k_encrypt_linear";
  // the chunk's mask in its E form (k_client.h el_region): k * 2N * 9 / 8 words
  hipLaunchKernelGGL(k_encrypt_linear, dim3((unsigned)B), dim3(EL_THREADS), (size_t)p.k * el_region(p.N) * 8,
                     (hipStream_t)stream, K, p.N,
                     p.k, p.msg_bits, p.glwe_noise_bits, ctx->s_big, d_qx, (int)D, G, d_w,
                     ((u64)cst) << (64 - p.msg_bits), id0, d_out);
  prof_end(ctx, ctx->prof_enc, (hipStream_t)stream, e1, B);
  HIPCHK(ctx, hipGetLastError());
  return FHE_OK;
}
int fhe_encrypt_linear_batch(fhe_ctx* ctx, const int64_t* d_qx, int64_t B, int32_t D, uint64_t seed, uint64_t id0,
                             const int64_t* d_w, int64_t cst, uint64_t* d_out, void* stream) {
  return encrypt_linear_impl(ctx, d_qx, B, D, key_from_seed(seed), id0, d_w, cst, d_out, stream);
}
int fhe_encrypt_linear_batch_key(fhe_ctx* ctx, const int64_t* d_qx, int64_t B, int32_t D, const uint32_t h_key[8],
                                 uint64_t id0, const int64_t* d_w, int64_t cst, uint64_t* d_out, void* stream) {
  ChaKey K;
  if (!key_arg(h_key, K)) return fail(ctx, FHE_E_ARG, "null encryption key");
  return encrypt_linear_impl(ctx, d_qx, B, D, K, id0, d_w, cst, d_out, stream);
}

static int seeded_args(fhe_ctx* ctx, int64_t B, int32_t D, const void* a, const void* b, const void* c) {
  if (B < 0 || D <= 0 || (B > 0 && (!a || !b || !c))) return fail(ctx, FHE_E_ARG, "bad seeded-corpus arguments");
  if (B * (int64_t)D > 0x7fffffffLL) return fail(ctx, FHE_E_ARG, "seeded corpus batch too large (B*D >= 2^31)");
  return FHE_OK;
}

int fhe_encrypt_seeded_batch(fhe_ctx* ctx, const int64_t* d_msg, int64_t B, int32_t D, const uint32_t h_mask_key[8],
                             const uint32_t h_noise_key[8], const uint64_t* d_id0, uint64_t* d_body, void* stream) {
  int rc = need_keys(ctx);
  if (rc) return rc;
  if ((rc = seeded_args(ctx, B, D, d_msg, d_id0, d_body))) return rc;
  if (!h_mask_key || !h_noise_key) return fail(ctx, FHE_E_ARG, "seeded encryption needs both keys");
  if (B == 0) return FHE_OK;
  const fhe_params& p = ctx->p;
  ChaKey Km, Kn;
  for (int i = 0; i < 8; ++i) Km.w[i] = h_mask_key[i], Kn.w[i] = h_noise_key[i];
  hipLaunchKernelGGL(k_encrypt_seeded, dim3((unsigned)(B * D)), dim3(256), 0, (hipStream_t)stream, Km, Kn, p.k * p.N,
                     p.msg_bits, p.glwe_noise_bits, ctx->s_big, d_msg, d_id0, (int)D, d_body);
  HIPCHK(ctx, hipGetLastError());
  return FHE_OK;
}

int fhe_expand_seeded_batch(fhe_ctx* ctx, const uint64_t* d_body, const uint64_t* d_id0, int64_t B, int32_t D,
                            const uint32_t h_mask_key[8], uint64_t* d_ct, void* stream) {
  int rc = need_device(ctx);
  if (rc) return rc;
  if ((rc = seeded_args(ctx, B, D, d_body, d_id0, d_ct))) return rc;
  if (!h_mask_key) return fail(ctx, FHE_E_ARG, "missing mask key");
  if (B == 0) return FHE_OK;
  const fhe_params& p = ctx->p;
  ChaKey Km;
  for (int i = 0; i < 8; ++i) Km.w[i] = h_mask_key[i];
  hipLaunchKernelGGL(k_expand_seeded, dim3((unsigned)(B * D)), dim3(256), 0, (hipStream_t)stream, Km, p.k * p.N,
                     d_body, d_id0, (int)D, d_ct);
  HIPCHK(ctx, hipGetLastError());
  return FHE_OK;
}

int fhe_linear_seeded_batch(fhe_ctx* ctx, const uint64_t* d_body, const uint64_t* d_id0, int64_t B, int32_t D,
                            const uint32_t h_mask_key[8], const int64_t* d_w, int64_t cst, uint64_t* d_out,
                            void* stream) {
  int rc = need_device(ctx);
  if (rc) return rc;
  if ((rc = seeded_args(ctx, B, D, d_body, d_id0, d_out))) return rc;
  if (!h_mask_key || (B > 0 && !d_w)) return fail(ctx, FHE_E_ARG, "missing mask key or weights");
  if (B == 0) return FHE_OK;
  const fhe_params& p = ctx->p;
  ChaKey Km;
  for (int i = 0; i < 8; ++i) Km.w[i] = h_mask_key[i];
  hipLaunchKernelGGL(k_linear_seeded, dim3((unsigned)B), dim3(256), 0, (hipStream_t)stream, Km, p.k * p.N, d_body,
                     d_id0, (int)D, d_w, (u64)cst << (64 - p.msg_bits), d_out);
  HIPCHK(ctx, hipGetLastError());
  return FHE_OK;
}

static int decrypt_mode(fhe_ctx* ctx, const uint64_t* d_ct, int64_t count, int64_t* d_out, int mode, void* stream) {
  int rc = need_keys(ctx);
  if (rc) return rc;
  if (count < 0 || (count > 0 && (!d_ct || !d_out))) return fail(ctx, FHE_E_ARG, "bad decrypt arguments");
  if (count == 0) return FHE_OK;
  const fhe_params& p = ctx->p;
  hipLaunchKernelGGL(k_decrypt, dim3((unsigned)count), dim3(256), 0, (hipStream_t)stream, p.k * p.N, p.msg_bits,
                     mode, ctx->s_big, d_ct, d_out);
  HIPCHK(ctx, hipGetLastError());
  return FHE_OK;
}
int fhe_decrypt_batch(fhe_ctx* ctx, const uint64_t* d_ct, int64_t count, int64_t* d_out, void* stream) {
  return decrypt_mode(ctx, d_ct, count, d_out, 0, stream);
}
int fhe_decrypt_bits_batch(fhe_ctx* ctx, const uint64_t* d_ct, int64_t count, int64_t* d_out, void* stream) {
  return decrypt_mode(ctx, d_ct, count, d_out, 1, stream);
}
int fhe_phase_batch(fhe_ctx* ctx, const uint64_t* d_ct, int64_t count, uint64_t* d_out, void* stream) {
  return decrypt_mode(ctx, d_ct, count, (int64_t*)d_out, 2, stream);
}

int fhe_linear_batch(fhe_ctx* ctx, const uint64_t* d_ct, int64_t B, int32_t D, const int64_t* d_w, int64_t cst,
                     uint64_t* d_out, void* stream) {
  int rc = need_device(ctx);
  if (rc) return rc;
  if (B < 0 || D <= 0 || (B > 0 && (!d_ct || !d_w || !d_out))) return fail(ctx, FHE_E_ARG, "bad linear arguments");
  if (B == 0) return FHE_OK;
  if (B > 65535) return fail(ctx, FHE_E_ARG, "linear batch > 65535: split the call");
  const fhe_params& p = ctx->p;
  const int W = p.k * p.N + 1;
  hipLaunchKernelGGL(k_linear, dim3((W + 255) / 256, (unsigned)B), dim3(256), 0, (hipStream_t)stream, d_ct, D, W, d_w,
                     ((u64)cst) << (64 - p.msg_bits), d_out);
  HIPCHK(ctx, hipGetLastError());
  return FHE_OK;
}

static void prof_begin(fhe_ctx* ctx, ProfAcc& a, hipStream_t st, hipEvent_t* e1) {
  *e1 = nullptr;
  if (!ctx->prof) return;
  hipEvent_t e0;
  if (hipEventCreate(&e0) != hipSuccess) return;
  if (hipEventCreate(e1) != hipSuccess) {
    (void)hipEventDestroy(e0);
    *e1 = nullptr;
    return;
  }
  (void)hipEventRecord(e0, st);  // a failed record shows up in fhe_profile_read
  a.ev.push_back({e0, *e1});
}
static void prof_end(fhe_ctx* ctx, ProfAcc& a, hipStream_t st, hipEvent_t e1, int64_t items) {
  if (!ctx->prof || !e1) return;
  (void)hipEventRecord(e1, st);
  a.launches += 1;
  a.items += items;
}

// the MFMA key switch's digit + body workspace of lane 0 or 1, grown to
// `count` ciphertexts (a grow synchronises the device: callers that run two
// lanes reserve both before launching on either)
static int ks_reserve(fhe_ctx* ctx, int64_t count, int lane) {
  const fhe_params& p = ctx->p;
  const int K = p.k * p.N * p.ks_level;
  const size_t need = (size_t)((count + 15) / 16) * 16 * K + 8 * (size_t)count;
  void*& ws = lane ? ctx->ks_ws1 : ctx->ks_ws;
  size_t& have = lane ? ctx->ks_ws1_bytes : ctx->ks_ws_bytes;
  if (need <= have) return FHE_OK;
  if (ws) {
    HIPCHK(ctx, hipDeviceSynchronize());
    HIPCHK(ctx, hipFree(ws));
    ws = nullptr;
  }
  HIPCHK(ctx, hipMalloc(&ws, need));
  have = need;
  return FHE_OK;
}

static int keyswitch_lane(fhe_ctx* ctx, const uint64_t* d_big, int64_t count, int32_t shift, uint64_t add_body,
                          uint64_t* d_small, hipStream_t st, int lane) {
  const fhe_params& p = ctx->p;
  const int64_t tiles = (count + KS_TC - 1) / KS_TC;
  if (tiles > 65535) return fail(ctx, FHE_E_ARG, "keyswitch batch too large: split the call");
  if (ctx->ks_variant == 2) {
    const int K = p.k * p.N * p.ks_level, KB = K / 64, n1 = p.n + 1, NB = ks_nb(p), CB = ks_cb(p);
    const int64_t ncb = (count + 15) / 16;
    const size_t dbytes = (size_t)ncb * 16 * K;
    int rc = ks_reserve(ctx, count, lane);
    if (rc) return rc;
    if (ncb > 65535) return fail(ctx, FHE_E_ARG, "keyswitch batch too large: split the call");
    void* ws = lane ? ctx->ks_ws1 : ctx->ks_ws;
    uint32_t* D = (uint32_t*)ws;
    u64* body = (u64*)((char*)ws + dbytes);
    const int R = ks_round_bits(p);
    // K split over S workgroups when the (ciphertext block, column group)
    // grid alone would leave CUs idle: ~2 workgroups per CU (S = 3 at 1024
    // ciphertexts; 1, 2, 4-12 measured slower there, tools/ks_sweep.py)
    const int64_t ctb = (count + KSM_CTS - 1) / KSM_CTS, ktiles = ctb * (NB / CB);
    int S = (int)std::max<int64_t>(1, std::min<int64_t>(KB / KSM_RING, 512 / ktiles));
#ifdef FHEICP_KS_AB  // A/B builds only: the split forced (tools/build_variant.sh)
    if (const char* e = getenv("FHEICP_KS_S")) S = std::max(1, std::min(KB / KSM_RING, atoi(e)));
#endif
    const int kslice = (KB / KSM_RING + S - 1) / S * KSM_RING;
    S = (KB + kslice - 1) / kslice;
    hipEvent_t e1;
    prof_begin(ctx, ctx->prof_ks, st, &e1);
    // the digits kernel also zeroes the output the split's atomics add into
    hipLaunchKernelGGL(k_ks_digits, dim3((unsigned)(p.k * p.N / 64), (unsigned)ncb), dim3(256), 0, st, d_big, count,
                       p.k * p.N, p.ks_base_log, p.ks_level, shift, add_body, KB, D, body, S > 1 ? n1 : 0, d_small);
    const dim3 gks((unsigned)(ktiles * S));
#define KSM(Q, C)                                                                                                    \
  ctx->prof_ks.kernel = "k_keyswitch_mfma<" #Q ", " #C ">";                                                         \
  hipLaunchKernelGGL((k_keyswitch_mfma<Q, C>), gks, dim3(256), 0, st, (const v4i*)D, (const v4i*)ctx->ksk8, body,    \
                     count, n1, NB, KB, R, S, kslice, d_small)
    switch ((8 - R / 8) * 4 + CB) {
      case 3 * 4 + 3: KSM(3, 3); break;
      case 4 * 4 + 3: KSM(4, 3); break;
      case 5 * 4 + 1: KSM(5, 1); break;
      case 6 * 4 + 1: KSM(6, 1); break;
      case 7 * 4 + 1: KSM(7, 1); break;
      case 8 * 4 + 1: KSM(8, 1); break;
      default: return fail(ctx, FHE_E_ARG, "key-switch byte planes out of range");
    }
#undef KSM
    prof_end(ctx, ctx->prof_ks, st, e1, count);
    HIPCHK(ctx, hipGetLastError());
    return FHE_OK;
  }
  HIPCHK(ctx, hipMemsetAsync(d_small, 0, 8 * (size_t)count * (p.n + 1), st));
  hipEvent_t e1;
  prof_begin(ctx, ctx->prof_ks, st, &e1);
  ctx->prof_ks.kernel = "k_keyswitch";
  hipLaunchKernelGGL(k_keyswitch, dim3((p.n + 1 + 255) / 256, (unsigned)tiles, KS_SPLIT), dim3(256), 0, st, d_big,
                     count, p.k * p.N, p.n, p.ks_level, p.ks_base_log, shift, add_body, ctx->ksk, ctx->ksk_colsum,
                     ks_round_bits(p), d_small);
  prof_end(ctx, ctx->prof_ks, st, e1, count);
  HIPCHK(ctx, hipGetLastError());
  return FHE_OK;
}

// largest input shift whose key-switch tie coins (bits 62 - prec - j of the
// shifted input, j < ks_level) are all input bits, not the zeros shifted in
static int ks_max_shift(const fhe_params& p) { return 63 - p.ks_level * p.ks_base_log - p.ks_level; }
int fhe_keyswitch_batch(fhe_ctx* ctx, const uint64_t* d_big, int64_t count, int32_t shift, uint64_t add_body,
                        uint64_t* d_small, void* stream) {
  int rc = need_keys(ctx);
  if (rc) return rc;
  if (count < 0 || shift < 0 || shift > ks_max_shift(ctx->p) || (count > 0 && (!d_big || !d_small)))
    return fail(ctx, FHE_E_ARG, "bad keyswitch arguments (shift must be in [0, 63 - ks_level * (ks_base_log + 1)])");
  if (count == 0) return FHE_OK;
  return keyswitch_lane(ctx, d_big, count, shift, add_body, d_small, (hipStream_t)stream, 0);
}

#ifdef FHEICP_AB
// A/B-only v4 shapes (FHEICP_V4_G = 1 or 2 for the 32-bit-accumulator
// kernels, FHEICP_V4_FL per-ciphertext hand-offs, FHEICP_V4_DBG timing
// experiments); false when the shipped dispatch applies.
static bool launch_br_ab(fhe_ctx* ctx, const fhe_params& p, const uint64_t* d_small, int64_t count, const BrTv& tv, int mode, uint64_t* out,
                         uint64_t* ct_v, uint64_t* refreshed, uint64_t* sign, const c64* bsk_fft, hipStream_t st,
                         const char** name) {
  const bool a32 = v4_a32(ctx, p);
#define AB4(L, A32, D, GG, FLAGS)                                                                               do {                                                                                                            hipLaunchKernelGGL((k_blind_rotate_v4<L, A32, D, GG, FLAGS>), dim3((unsigned)((count + GG - 1) / GG)),                           dim3(v4::nthreads(GG)), 0, st, d_small, count, p.n, p.pbs_base_log, bsk_fft,                               ctx->tw4, tv, mode, out, ct_v, refreshed, sign);                                           *name = "k_blind_rotate_v4<" #L ", " #A32 ", " #D ", " #GG ", " #FLAGS ", 0>";                                    return true;                                                                                                } while (0)
#define AB4G(L, A32, D, GG)   do { if (ctx->v4_fl && GG > 1) AB4(L, A32, D, GG, true); else AB4(L, A32, D, GG, false); } while (0)
#define AB4D(D)   do { if (ctx->v4_g == 1) AB4G(2, true, D, 1); else if (ctx->v4_g == 2) AB4G(2, true, D, 2); else AB4G(2, true, D, 4); } while (0)
  if (ctx->v4_dbg && p.pbs_level == 2 && a32) {
    switch (ctx->v4_dbg) {
      case 1: AB4D(1); case 2: AB4D(2); case 4: AB4D(4); case 8: AB4D(8); case 16: AB4D(16);
      case 32: AB4D(32); case 6: AB4D(6); case 128: AB4D(128); default: AB4D(63);
    }
  }
  if (ctx->v4s && a32) {  // FHEICP_V4S=1: key-stationary products for the 32-bit kernels too
    if (p.pbs_level == 1)
      hipLaunchKernelGGL((k_blind_rotate_v4s<1, true>), dim3((unsigned)((count + 3) / 4)), dim3(v4::nthreads(4)), 0,
                         st, d_small, count, p.n, p.pbs_base_log, bsk_fft, ctx->tw4, tv, mode, out, ct_v, refreshed, sign);
    else
      hipLaunchKernelGGL((k_blind_rotate_v4s<2, true>), dim3((unsigned)((count + 3) / 4)), dim3(v4::nthreads(4)), 0,
                         st, d_small, count, p.n, p.pbs_base_log, bsk_fft, ctx->tw4, tv, mode, out, ct_v, refreshed, sign);
    *name = "k_blind_rotate_v4s<A32>";
    return true;
  }
  // shapes other than the shipped ones; the 64-bit v4 kernels (v4s ships)
  if (!(ctx->v4_g == 1 || ctx->v4_fl || ctx->v4_g == 2)) return false;
  const int G = ctx->v4_g;
  switch (p.pbs_level) {
    case 1:
      if (a32) { if (G == 1) AB4G(1, true, 0, 1); else if (G == 2) AB4G(1, true, 0, 2); else AB4G(1, true, 0, 4); }
      else { if (G == 1) AB4G(1, false, 0, 1); else if (G == 2) AB4G(1, false, 0, 2); else AB4G(1, false, 0, 4); }
      break;
    case 2:
      if (a32) { if (G == 1) AB4G(2, true, 0, 1); else if (G == 2) AB4G(2, true, 0, 2); else AB4G(2, true, 0, 4); }
      else { if (G == 1) AB4G(2, false, 0, 1); else if (G == 2) AB4G(2, false, 0, 2); else AB4G(2, false, 0, 4); }
      break;
    case 3:
      if (G == 1) AB4G(3, false, 0, 1); else if (G == 2) AB4G(3, false, 0, 2); else AB4G(3, false, 0, 4);
      break;
  }
#undef AB4
#undef AB4G
#undef AB4D
  return false;
}
#endif

// gad = 1 / 2: the fast / fast2 gadget and its key (fhe_params.pbs_fast*_*),
// else the main one. The launched instantiation's name (as rocprofv3 prints
// it) is recorded in the profile bucket (fhe_profile_kernel_name).
static int launch_br(fhe_ctx* ctx, const uint64_t* d_small, int64_t count, BrTv tv, int mode, uint64_t* out,
                     uint64_t* ct_v, uint64_t* refreshed, uint64_t* sign, hipStream_t st, int gad = 0) {
  const bool fast = gad > 0 && fast_level(ctx->p, gad);
  const fhe_params p = fast ? fast_params(ctx->p, gad) : ctx->p;
  const c64* bsk_fft = fast ? ctx->bskf_fft[gad - 1] : ctx->bsk_fft;
  const int var = variant_for(ctx, p);
  hipEvent_t e1;
  ProfAcc& prof = fast ? ctx->prof_brf[gad - 1] : ctx->prof_br;
  prof_begin(ctx, prof, st, &e1);
  const char* name = nullptr;
  const dim3 g((unsigned)count), b(64);
#define BR(LOGM, K)                                                                                           \
  do {                                                                                                        \
    hipLaunchKernelGGL((k_blind_rotate<LOGM, K>), g, b, 0, st, d_small, p.n, p.pbs_level, p.pbs_base_log,    \
                       bsk_fft, ctx->tw, ctx->twist, tv, mode, out, ct_v, refreshed, sign);                  \
    name = "k_blind_rotate<" #LOGM ", " #K ", BrTv>";                                                         \
  } while (0)
#define BRV(V, K, W)                                                                                          \
  do {                                                                                                        \
    hipLaunchKernelGGL((k_blind_rotate_mw<V, K, W>), g, dim3(V::NT), 0, st, d_small, p.n, p.pbs_level,        \
                       p.pbs_base_log, bsk_fft, ctx->tw, ctx->twist, tv, mode, out, ct_v, refreshed, sign);   \
    name = "k_blind_rotate_mw<fhei::" #V ", " #K ", " #W ", BrTv>";                                           \
  } while (0)
#define BR4F(L, A32, D, GG, FLAGS, B)                                                                         \
  do {                                                                                                        \
    hipLaunchKernelGGL((k_blind_rotate_v4<L, A32, D, GG, FLAGS, B>), dim3((unsigned)((count + GG - 1) / GG)), \
                       dim3(v4::nthreads(GG)), 0, st, d_small, count, p.n, p.pbs_base_log, bsk_fft, ctx->tw4, \
                       tv, mode, out, ct_v, refreshed, sign);                                                 \
    name = "k_blind_rotate_v4<" #L ", " #A32 ", " #D ", " #GG ", " #FLAGS ", " #B ">";                         \
  } while (0)
  // The shipped N = 1024, k = 2 instances: the multi-bit kernels for fast
  // gadgets with pbs_fast*_group = 2; v4 at 4 ciphertexts per workgroup (3
  // waves per SIMD, <= 168 VGPRs) for the 32-bit accumulators; v4s for the
  // 64-bit ones. Other shapes are A/B builds (FHEICP_AB).
  bool done = false;
#ifdef FHEICP_AB
  if (p.N == 1024 && p.k == 2 && var == 4) done = launch_br_ab(ctx, p, d_small, count, tv, mode, out, ct_v, refreshed, sign,
                                                               bsk_fft, st, &name);
#endif
  if (done) {
  } else if (fast && mb_for(ctx->p, gad)) {
    // multi-bit rotation, key-stationary products (k_blind_rotate_mb)
    const dim3 gm((unsigned)((count + 3) / 4)), bm(v4::nthreads(4));
#define MBD(L, D, B)                                                                                            \
  hipLaunchKernelGGL((k_blind_rotate_mb<L, D, B>), gm, bm, 0, st, d_small, count, p.n, p.pbs_base_log, bsk_fft, \
                     ctx->tw4, ctx->psi, tv, mode, out, ct_v, refreshed, sign)
#ifdef FHEICP_AB
    if (ctx->mb_dbg) {
      const int w = ctx->mb_dbg >> 8;
      if (ctx->mb_dbg == 2) { if (p.pbs_level == 1) MBD(1, 2, 0); else MBD(2, 2, 0); }
      else if (ctx->mb_dbg == 16) { if (p.pbs_level == 1) MBD(1, 16, 0); else MBD(2, 16, 0); }
      else if (ctx->mb_dbg == 32) { if (p.pbs_level == 1) MBD(1, 32, 0); else MBD(2, 32, 0); }
      else if (ctx->mb_dbg == 48) { if (p.pbs_level == 1) MBD(1, 48, 0); else MBD(2, 48, 0); }
      else if (ctx->mb_dbg == 64) { if (p.pbs_level == 1) MBD(1, 64, 0); else MBD(2, 64, 0); }
      else if (ctx->mb_dbg == 18) { if (p.pbs_level == 1) MBD(1, 18, 0); else MBD(2, 18, 0); }
      else if (ctx->mb_dbg == 130) { if (p.pbs_level == 1) MBD(1, 130, 0); else MBD(2, 130, 0); }
      else if (w == 0) { if (p.pbs_level == 1) MBD(1, 128, 0); else MBD(2, 128, 0); }
      else if (w == 1) { if (p.pbs_level == 1) MBD(1, 128 + 256, 0); else MBD(2, 128 + 256, 0); }
      else { if (p.pbs_level == 1) MBD(1, 128 + 512, 0); else MBD(2, 128 + 512, 0); }
      name = "k_blind_rotate_mb<DBG>";
    } else
#endif
    // wide (48-bit) accumulators (L * beta > 31 or L > 2): the deep gadgets
    if (!(p.pbs_level <= 2 && p.pbs_level * p.pbs_base_log <= 31)) {
#define MB64(L)                                                                                                  \
  hipLaunchKernelGGL((k_blind_rotate_mb64<L, 0>), gm, bm, 0, st, d_small, count, p.n, p.pbs_base_log, bsk_fft,   \
                     ctx->tw4, ctx->psi, tv, mode, out, ct_v, refreshed, sign);                                 \
  name = "k_blind_rotate_mb64<" #L ", 0, BrTv>"
      switch (p.pbs_level) {
        case 1: MB64(1); break;
        case 2: MB64(2); break;
        case 3: MB64(3); break;
        case 4: MB64(4); break;
        case 5: MB64(5); break;
        case 6: MB64(6); break;
        case 7: MB64(7); break;
        case 8: MB64(8); break;
        default: return fail(ctx, FHE_E_ARG, "multi-bit blind rotation: pbs_level > 8");
      }
#undef MB64
    } else
    // the shipped fast gadgets (23,1) and (15,2) with their base log fixed
    if (p.pbs_level == 1 && p.pbs_base_log == 23) {
      MBD(1, 0, 23);
      name = "k_blind_rotate_mb<1, 0, 23, BrTv>";
    } else if (p.pbs_level == 1) {
      MBD(1, 0, 0);
      name = "k_blind_rotate_mb<1, 0, 0, BrTv>";
    } else if (p.pbs_base_log == 15) {
      MBD(2, 0, 15);
      name = "k_blind_rotate_mb<2, 0, 15, BrTv>";
    } else {
      MBD(2, 0, 0);
      name = "k_blind_rotate_mb<2, 0, 0, BrTv>";
    }
#undef MBD
  } else if (p.N == 1024 && p.k == 2 && var == 4 && !v4_a32(ctx, p)) {
    // 64-bit accumulators: the key-stationary v4s kernels, 4 ciphertexts per
    // workgroup (15.9 vs 20.7 ms per 1024 at (12,3) for v4 at 2 per workgroup)
#define BR4S(L, B)                                                                                            \
  do {                                                                                                        \
    hipLaunchKernelGGL((k_blind_rotate_v4s<L, false, 0, B>), dim3((unsigned)((count + 3) / 4)),              \
                       dim3(v4::nthreads(4)), 0, st, d_small, count, p.n, p.pbs_base_log, bsk_fft, ctx->tw4,  \
                       tv, mode, out, ct_v, refreshed, sign);                                                 \
    name = "k_blind_rotate_v4s<" #L ", false, 0, " #B ">";                                                     \
  } while (0)
    // run-time base log: fixing (12, 3)'s at compile time made the compiler
    // emit 144 more f64 instructions per step and a 56-byte spill
    switch (p.pbs_level) {
      case 1: BR4S(1, 0); break;
      case 2: BR4S(2, 0); break;
      case 3: BR4S(3, 0); break;
      // the deep gadgets (C5's main and mid ones): 1.5-1.6x faster than v2,
      // e.g. (6,7) 29.5 vs 46.7 ms and (8,5) 23.0 vs 35.1 ms per 1024
      case 4: BR4S(4, 0); break;
      case 5: BR4S(5, 0); break;
      case 6: BR4S(6, 0); break;
      case 7: BR4S(7, 0); break;
      case 8: BR4S(8, 0); break;
      default: return fail(ctx, FHE_E_ARG, "v4s blind rotation: pbs_level > 8");
    }
#undef BR4S
  } else if (p.N == 1024 && p.k == 2 && var == 4) {
    switch (p.pbs_level) {
      // (23, 1) and (15, 2), the classic gadgets of the parameter table, with
      // their base log fixed; others on the run-time instances
      case 1:
        if (p.pbs_base_log == 23) BR4F(1, true, 0, 4, false, 23);
        else BR4F(1, true, 0, 4, false, 0);
        break;
      case 2:
        if (p.pbs_base_log == 15) BR4F(2, true, 0, 4, false, 15);
        else BR4F(2, true, 0, 4, false, 0);
        break;
      default: return fail(ctx, FHE_E_ARG, "v4 blind rotation: 32-bit accumulators need pbs_level <= 2");
    }
  } else if (p.N == 256 && p.k == 1) BR(7, 1);
  else if (p.N == 256 && p.k == 2) BR(7, 2);
  else if (p.N == 512 && p.k == 1) BR(8, 1);
  else if (p.N == 512 && p.k == 2) BR(8, 2);
  else if (p.N == 1024 && p.k == 1) BRV(V2, 1, 2);
  else if (p.N == 1024 && p.k == 2) BRV(V2, 2, 2);
  else if (p.N == 2048 && p.k == 1) BR(10, 1);
  else return fail(ctx, FHE_E_ARG, "unsupported (N, k)");
#undef BR
#undef BR4F
#undef BRV
  prof.kernel = name;
  prof_end(ctx, prof, st, e1, count);
  HIPCHK(ctx, hipGetLastError());
  return FHE_OK;
}

int fhe_pbs_batch(fhe_ctx* ctx, const uint64_t* d_small, int64_t count, uint64_t tv, uint64_t* d_out, void* stream) {
  int rc = need_keys(ctx);
  if (rc) return rc;
  if (count < 0 || (count > 0 && (!d_small || !d_out))) return fail(ctx, FHE_E_ARG, "bad pbs arguments");
  if (count == 0) return FHE_OK;
  return launch_br(ctx, d_small, count, BrTv{tv, 0, 0}, 0, d_out, nullptr, nullptr, nullptr, (hipStream_t)stream);
}

int fhe_pbs_gadget_batch(fhe_ctx* ctx, const uint64_t* d_small, int64_t count, int32_t gadget, uint64_t tv,
                         uint64_t* d_out, void* stream) {
  int rc = need_keys(ctx);
  if (rc) return rc;
  if (count < 0 || gadget < 0 || gadget >= NGAD || (count > 0 && (!d_small || !d_out)))
    return fail(ctx, FHE_E_ARG, "bad pbs-gadget arguments");
  if (gadget > 0 && !fast_level(ctx->p, gadget)) return fail(ctx, FHE_E_STATE, "no such fast gadget in these parameters");
  if (count == 0) return FHE_OK;
  return launch_br(ctx, d_small, count, BrTv{tv, 0, 0}, 0, d_out, nullptr, nullptr, nullptr, (hipStream_t)stream,
                   gadget);
}

static int log2i(int x) {
  int l = 0;
  while ((1 << l) < x) ++l;
  return l;
}

int fhe_pbs_lut_batch(fhe_ctx* ctx, const uint64_t* d_small, int64_t count, uint64_t base, uint64_t step,
                      int32_t log_slots, uint64_t* d_out, void* stream) {
  int rc = need_keys(ctx);
  if (rc) return rc;
  const int logN = log2i(ctx->p.N);
  if (count < 0 || (count > 0 && (!d_small || !d_out)) || log_slots < 0 || log_slots > logN)
    return fail(ctx, FHE_E_ARG, "bad pbs-lut arguments");
  if (count == 0) return FHE_OK;
  return launch_br(ctx, d_small, count, BrTv{base, step, logN - log_slots}, 0, d_out, nullptr, nullptr, nullptr,
                   (hipStream_t)stream);
}

// The gadget fhe_pbs_table_batch runs on: the most precise (smallest
// bootstrap variance) multi-bit gadget of the set, whose rotation is the
// shipped k_blind_rotate_mb / _mb64 family (e.g. (15,2) at P = 16, (5,8) at
// P = 26); 0 (the classic main gadget, v2 / v1 kernels) when the set has none.
static int table_gadget(const fhe_params& p) {
  int best = 0;
  double v = 0;
  for (int g = 1; g < NGAD; ++g) {
    if (!mb_for(p, g)) continue;
    const double vg = pbs_var(p, gadget_base_log(p, g), gadget_level(p, g), 2);
    if (!best || vg < v) best = g, v = vg;
  }
  return best;
}

// The table bootstrap on a multi-bit gadget: the sign extraction's kernels
// (k_blind_rotate_mb: 32-bit accumulators, (23,1) and (15,2) with their base
// log fixed as there; k_blind_rotate_mb64: 48-bit, levels 2-8) instantiated
// for the table test vector (BrTvLut), with that gadget's multi-bit key.
static int launch_br_table_mb(fhe_ctx* ctx, const uint64_t* d_small, int64_t count, const BrTvLut& tv, uint64_t* out,
                              hipStream_t st, int gad) {
  const fhe_params q = fast_params(ctx->p, gad);
  const c64* bsk = ctx->bskf_fft[gad - 1];
  ProfAcc& prof = ctx->prof_brf[gad - 1];
  hipEvent_t e1;
  prof_begin(ctx, prof, st, &e1);
  const char* name = nullptr;
  const dim3 gm((unsigned)((count + 3) / 4)), bm(v4::nthreads(4));
#define MBT(L, B)                                                                                                  \
  do {                                                                                                             \
    hipLaunchKernelGGL((k_blind_rotate_mb<L, 0, B, BrTvLut>), gm, bm, 0, st, d_small, count, q.n, q.pbs_base_log,   \
                       bsk, ctx->tw4, ctx->psi, tv, 0, out, nullptr, nullptr, nullptr);                            \
    name = "k_blind_rotate_mb<" #L ", 0, " #B ", BrTvLut>";                                                        \
  } while (0)
#define MB64T(L)                                                                                                   \
  do {                                                                                                             \
    hipLaunchKernelGGL((k_blind_rotate_mb64<L, 0, BrTvLut>), gm, bm, 0, st, d_small, count, q.n, q.pbs_base_log,    \
                       bsk, ctx->tw4, ctx->psi, tv, 0, out, nullptr, nullptr, nullptr);                            \
    name = "k_blind_rotate_mb64<" #L ", 0, BrTvLut>";                                                              \
  } while (0)
  if (q.pbs_level <= 2 && q.pbs_level * q.pbs_base_log <= 31) {
    if (q.pbs_level == 1) {
      if (q.pbs_base_log == 23) MBT(1, 23);
      else MBT(1, 0);
    } else {
      if (q.pbs_base_log == 15) MBT(2, 15);
      else MBT(2, 0);
    }
  } else {
    switch (q.pbs_level) {
      case 2: MB64T(2); break;
      case 3: MB64T(3); break;
      case 4: MB64T(4); break;
      case 5: MB64T(5); break;
      case 6: MB64T(6); break;
      case 7: MB64T(7); break;
      case 8: MB64T(8); break;
      default: return fail(ctx, FHE_E_ARG, "table bootstrap: no multi-bit kernel for this gadget level");
    }
  }
#undef MBT
#undef MB64T
  prof.kernel = name;
  prof_end(ctx, prof, st, e1, count);
  HIPCHK(ctx, hipGetLastError());
  return FHE_OK;
}

// The table bootstrap on the classic main gadget (parameter sets without a
// multi-bit gadget): the v2 kernel at N = 1024 (v1 otherwise), instantiated
// for the wide test-vector argument (BrTvLut); the compare's hot kernels keep
// the three-word one.
static int launch_br_table(fhe_ctx* ctx, const uint64_t* d_small, int64_t count, const BrTvLut& tv, uint64_t* out,
                           hipStream_t st) {
  const fhe_params& p = ctx->p;
  hipEvent_t e1;
  prof_begin(ctx, ctx->prof_br, st, &e1);
  const char* name = nullptr;
  const dim3 g((unsigned)count), b(64);
#define BRT(LOGM, K)                                                                                          \
  do {                                                                                                        \
    hipLaunchKernelGGL((k_blind_rotate<LOGM, K, BrTvLut>), g, b, 0, st, d_small, p.n, p.pbs_level,            \
                       p.pbs_base_log, ctx->bsk_fft, ctx->tw, ctx->twist, tv, 0, out, nullptr, nullptr, nullptr); \
    name = "k_blind_rotate<" #LOGM ", " #K ", BrTvLut>";                                                      \
  } while (0)
  if (p.N == 1024 && variant_for(ctx, p) == 4) {
    // the BSK is in the v4 FFT layout: build a v2-layout copy once
    if (!ctx->bsk_fft_v2) {
      HIPCHK(ctx, hipMalloc(&ctx->bsk_fft_v2, sizeof(c64) * fhe_bsk_words(&p) / 2));
      const int npoly = (int)(fhe_bsk_words(&p) / p.N);
      hipLaunchKernelGGL(k_bsk_to_fft_mw<V2>, dim3(npoly), dim3(V2::NT), 0, st, ctx->bsk, npoly, ctx->tw, ctx->twist,
                         ctx->bsk_fft_v2);
      // once per key: a later table bootstrap on another stream must not
      // read the copy before this conversion has finished
      HIPCHK(ctx, hipGetLastError());
      HIPCHK(ctx, hipStreamSynchronize(st));
    }
  }
  const c64* bsk = (p.N == 1024 && ctx->bsk_fft_v2) ? ctx->bsk_fft_v2 : ctx->bsk_fft;
  if (p.N == 1024) {
    if (p.k == 1) {
      hipLaunchKernelGGL((k_blind_rotate_mw<V2, 1, 2, BrTvLut>), g, dim3(V2::NT), 0, st, d_small, p.n, p.pbs_level,
                         p.pbs_base_log, bsk, ctx->tw, ctx->twist, tv, 0, out, nullptr, nullptr, nullptr);
      name = "k_blind_rotate_mw<fhei::V2, 1, 2, BrTvLut>";
    } else {
      hipLaunchKernelGGL((k_blind_rotate_mw<V2, 2, 2, BrTvLut>), g, dim3(V2::NT), 0, st, d_small, p.n, p.pbs_level,
                         p.pbs_base_log, bsk, ctx->tw, ctx->twist, tv, 0, out, nullptr, nullptr, nullptr);
      name = "k_blind_rotate_mw<fhei::V2, 2, 2, BrTvLut>";
    }
  } else if (p.N == 256 && p.k == 1) BRT(7, 1);
  else if (p.N == 256 && p.k == 2) BRT(7, 2);
  else if (p.N == 512 && p.k == 1) BRT(8, 1);
  else if (p.N == 512 && p.k == 2) BRT(8, 2);
  else if (p.N == 2048 && p.k == 1) BRT(10, 1);
  else return fail(ctx, FHE_E_ARG, "unsupported (N, k)");
#undef BRT
  ctx->prof_br.kernel = name;
  prof_end(ctx, ctx->prof_br, st, e1, count);
  HIPCHK(ctx, hipGetLastError());
  return FHE_OK;
}

int fhe_pbs_table_gadget_batch(fhe_ctx* ctx, const uint64_t* d_small, int64_t count, int32_t gadget,
                               const int64_t* d_lut, int32_t lut_bits, uint64_t* d_out, void* stream) {
  int rc = need_keys(ctx);
  if (rc) return rc;
  const int logN = log2i(ctx->p.N);
  if (count < 0 || lut_bits < 0 || lut_bits > logN - 1 || !d_lut || (count > 0 && (!d_small || !d_out)))
    return fail(ctx, FHE_E_ARG, "bad pbs-table arguments (0 <= lut_bits <= log2(N) - 1)");
  if (gadget < 0 || gadget >= NGAD || (gadget > 0 && !mb_for(ctx->p, gadget)))
    return fail(ctx, FHE_E_ARG, "pbs-table gadget must be 0 (the classic main gadget) or a multi-bit gadget of "
                                "these parameters");
  if (count == 0) return FHE_OK;
  BrTvLut tv{0, 0, 0, logN - lut_bits, 1 << lut_bits, d_lut, 1ull << (64 - ctx->p.msg_bits)};
  if (gadget > 0) return launch_br_table_mb(ctx, d_small, count, tv, d_out, (hipStream_t)stream, gadget);
  return launch_br_table(ctx, d_small, count, tv, d_out, (hipStream_t)stream);
}

int fhe_pbs_table_batch(fhe_ctx* ctx, const uint64_t* d_small, int64_t count, const int64_t* d_lut, int32_t lut_bits,
                        uint64_t* d_out, void* stream) {
  if (!ctx) return fail(nullptr, FHE_E_ARG, "null ctx");
  return fhe_pbs_table_gadget_batch(ctx, d_small, count, table_gadget(ctx->p), d_lut, lut_bits, d_out, stream);
}

int fhe_pbs_table_gadget(const fhe_params* params) {
  std::string why;
  if (validate(params, why)) return FHE_E_ARG;
  return table_gadget(*params);
}

static int ensure_ws(fhe_ctx* ctx, size_t bytes) {
  if (bytes <= ctx->ws_bytes) return FHE_OK;
  if (ctx->ws) {
    HIPCHK(ctx, hipDeviceSynchronize());
    HIPCHK(ctx, hipFree(ctx->ws));
    ctx->ws = nullptr;
    ctx->ws_bytes = 0;
  }
  HIPCHK(ctx, hipMalloc(&ctx->ws, bytes));
  ctx->ws_bytes = bytes;
  return FHE_OK;
}

// bit extraction driver; `small` is caller-provided scratch (count x (n+1))
static int bit_extract(fhe_ctx* ctx, uint64_t* d_ct_v, int64_t count, uint64_t* d_ref, uint64_t* d_sign,
                       uint64_t* small, hipStream_t st) {
  const fhe_params& p = ctx->p;
  const int P = p.msg_bits;
  HIPCHK(ctx, hipMemsetAsync(d_ref, 0, 8 * (size_t)count * fhe_big_lwe_words(&p), st));
  for (int i = 0; i < P; ++i) {
    int rc = fhe_keyswitch_batch(ctx, d_ct_v, count, P - 1 - i, 1ull << 62, small, st);
    if (rc) return rc;
    rc = launch_br(ctx, small, count, BrTv{1ull << (63 - P + i), 0, 0}, 1, nullptr, d_ct_v, d_ref,
                   (i == P - 1) ? d_sign : nullptr, st);
    if (rc) return rc;
  }
  return FHE_OK;
}

// Sign of the msg_bits-bit value v in d_ct_v (consumed) with d-bit digits
// (DESIGN.md §3.4): the low m = P - d bits are cleared LSB-first, each full
// digit [b, b+c) by two bootstraps (its top bit by a sign bootstrap; then,
// with a zero padding bit, its c-1 low bits by a 2^(c-1)-slot staircase LUT),
// a leftover of 1-2 bits by single-bit rounds; the sign of the top d bits is
// the sign of v.
int fhe_sign_digit_bits(const fhe_params* params) {
  std::string why;
  if (validate(params, why)) return -1;
  return sign_digits(*params);
}

int fhe_sign_pbs_count(const fhe_params* params) {
  std::string why;
  if (validate(params, why)) return -1;
  const int P = params->msg_bits, d = sign_digits(*params);
  if (P < 4) return P;
  const int m = P - d, r = m % d;
  return 2 * (m / d) + (r >= 3 ? 2 : r) + 1;
}

int fhe_sign_precise_rounds(const fhe_params* params) {
  std::string why;
  if (validate(params, why)) return -1;
  int d, j1, j2;
  sign_plan(*params, &d, &j1, &j2);
  return j1;
}

int fhe_sign_schedule(const fhe_params* params, int32_t* gadgets, int32_t cap) {
  std::string why;
  if (validate(params, why)) return FHE_E_ARG;
  int d, sched[64];
  const int R = sign_schedule(*params, &d, sched);
  for (int r = 0; r < R && r < cap; ++r)
    if (gadgets) gadgets[r] = sched[r];
  return R;
}

int fhe_sign_plan(const fhe_params* params, int32_t* digit_bits, int32_t* main_rounds, int32_t* fast_end) {
  std::string why;
  if (validate(params, why)) return FHE_E_ARG;
  int d, j1, j2;
  sign_plan(*params, &d, &j1, &j2);
  if (digit_bits) *digit_bits = d;
  if (main_rounds) *main_rounds = j1;
  if (fast_end) *fast_end = j2;
  return FHE_OK;
}

// Trace of a sign extraction (fhe_sign_trace_batch, measurement only): an
// explicit gadget per round instead of sign_schedule's, a stop after the
// first `rounds` bootstraps, and the rotation exponent of every round's input
// (k_ms_phase) into phase[round * count + c].
struct SignTrace {
  const int* sched = nullptr;
  int rounds = 0;
  uint32_t* phase = nullptr;
};

static int sign_extract(fhe_ctx* ctx, uint64_t* d_ct_v, int64_t count, uint64_t* d_sign, uint64_t* small,
                        hipStream_t st, int lane = 0, const SignTrace* tr = nullptr) {
  const fhe_params& p = ctx->p;
  const int P = p.msg_bits, logN = log2i(p.N);
  int rc;
  int d = 0, sched[64];
  if (P < 4) {
    for (int r = 0; r < P; ++r) sched[r] = 0;
  } else {
    sign_schedule(p, &d, sched);
  }
  if (tr && tr->sched) {
    int dd, tmp[64];
    const int R = P < 4 ? P : sign_schedule(p, &dd, tmp);
    for (int r = 0; r < R; ++r) sched[r] = tr->sched[r];
  }
  int round = 0;  // bootstraps issued so far; round r runs on gadget sched[r]
  // one round: key switch of v << shift, centred by `add`, then the bootstrap
  auto step = [&](int shift, uint64_t add, BrTv tv, int mode, uint64_t* sign) -> int {
    if (tr && tr->rounds && round >= tr->rounds) return FHE_OK;
    int r = keyswitch_lane(ctx, d_ct_v, count, shift, add, small, st, lane);
    if (r) return r;
    if (tr && tr->phase) {
      hipLaunchKernelGGL(k_ms_phase, dim3((unsigned)count), dim3(64), 0, st, p.n, logN + 1,
                         gadget_group(p, sched[round]), ctx->s_small, small, count,
                         tr->phase + (size_t)round * count);
      HIPCHK(ctx, hipGetLastError());
    }
    return launch_br(ctx, small, count, tv, mode, nullptr, d_ct_v, nullptr, sign, st, sched[round++]);
  };
  if (P < 4) {
    for (int i = 0; i < P; ++i)
      if ((rc = step(P - 1 - i, 1ull << 62, BrTv{1ull << (63 - P + i), 0, 0}, 1, (i == P - 1) ? d_sign : nullptr)))
        return rc;
    return FHE_OK;
  }
  const int m = P - d;
  // one c-bit digit at bit b: the pair of rounds on v << (P-b-c) centred by 2^(63-c)
  auto digit = [&](int b, int c) -> int {
    int r;
    // digit MSB (bit b+c-1): sign bootstrap, ct_v -= [bit] * 2^(b+c-1) * Delta
    if ((r = step(P - b - c, 1ull << (63 - c), BrTv{1ull << (62 - P + b + c), 0, 0}, 1, nullptr))) return r;
    // bits [b, b+c-1): top bit is now 0 -> 2^(c-1)-slot staircase, output D' * 2^b * Delta
    return step(P - b - c, 1ull << (63 - c), BrTv{0, 1ull << (64 - P + b), logN - (c - 1)}, 2, nullptr);
  };
  int b = 0;
  for (; b + d <= m; b += d)
    if ((rc = digit(b, d))) return rc;
  if (m - b >= 3) {
    if ((rc = digit(b, m - b))) return rc;
    b = m;
  }
  for (; b < m; ++b)
    if ((rc = step(P - b - 1, 1ull << 62, BrTv{1ull << (63 - P + b), 0, 0}, 1, nullptr))) return rc;
  // sign = MSB of the top digit [P-d, P)
  return step(0, 1ull << (63 - d), BrTv{1ull << 62, 0, 0}, 1, d_sign);
}

// The sign extraction of a large batch (>= PIPE_MIN ciphertexts) in two
// halves on two streams: each half runs its key switches and bootstraps in
// order, and the GPU overlaps one half's key switches and kernel tails with
// the other half's bootstraps. Below PIPE_MIN (one or two waves of
// workgroups) it stays on the caller's stream, so single-launch timings keep
// their meaning. FHEICP_PIPE=0 turns it off (A/B runs).
constexpr int64_t PIPE_MIN = 2048;
static int sign_extract_batch(fhe_ctx* ctx, uint64_t* d_ct_v, int64_t count, uint64_t* d_sign, uint64_t* small,
                              hipStream_t st) {
  static const bool off = [] {
    const char* e = getenv("FHEICP_PIPE");
    return e && atoi(e) == 0;
  }();
  static const int64_t pipe_min = [] {  // FHEICP_PIPE_MIN: A/B runs of the threshold
    const char* e = getenv("FHEICP_PIPE_MIN");
    return e ? (int64_t)std::max(8, atoi(e)) : PIPE_MIN;
  }();
  if (count < pipe_min || off) return sign_extract(ctx, d_ct_v, count, d_sign, small, st, 0);
  const fhe_params& p = ctx->p;
  const size_t Wb = fhe_big_lwe_words(&p), Ws = fhe_small_lwe_words(&p);
  // the first half a whole number of 1024-ciphertext waves (256 four-ciphertext
  // workgroups, one per CU) nearest count / 2, so only the second half ends on
  // a partial wave: at 12,500 (a C4 shard) 6144 + 6356 runs 13 rounds of
  // workgroups where 6252 + 6248 ran 14 (6.1 waves each)
  const int64_t c0 = count < 2048 ? ((count / 2) + 3) & ~(int64_t)3
                                  : std::min(std::max((int64_t)1024, 1024 * ((count + 1024) / 2048)), count - 4),
                c1 = count - c0;
  for (int l = 0; l < 2; ++l)
    if (!ctx->lane_st[l]) HIPCHK(ctx, hipStreamCreateWithFlags(&ctx->lane_st[l], hipStreamNonBlocking));
  for (int l = 0; l < 3; ++l)
    if (!ctx->lane_ev[l]) HIPCHK(ctx, hipEventCreateWithFlags(&ctx->lane_ev[l], hipEventDisableTiming));
  // the MFMA key switch's per-lane workspaces (the VALU variant needs none)
  int rc = ctx->ks_variant == 2 ? ks_reserve(ctx, c0, 0) : FHE_OK;
  if (!rc && ctx->ks_variant == 2) rc = ks_reserve(ctx, c1, 1);
  if (rc) return rc;
  HIPCHK(ctx, hipEventRecord(ctx->lane_ev[0], st));
  for (int l = 0; l < 2; ++l) HIPCHK(ctx, hipStreamWaitEvent(ctx->lane_st[l], ctx->lane_ev[0], 0));
  rc = sign_extract(ctx, d_ct_v, c0, d_sign, small, ctx->lane_st[0], 0);
  if (!rc)
    rc = sign_extract(ctx, d_ct_v + (size_t)c0 * Wb, c1, d_sign + (size_t)c0 * Wb, small + (size_t)c0 * Ws,
                      ctx->lane_st[1], 1);
  // the caller's stream waits for both halves (also on an error, so nothing
  // queued on it can overtake work already launched on the lanes)
  for (int l = 0; l < 2; ++l) {
    HIPCHK(ctx, hipEventRecord(ctx->lane_ev[1 + l], ctx->lane_st[l]));
    HIPCHK(ctx, hipStreamWaitEvent(st, ctx->lane_ev[1 + l], 0));
  }
  return rc;
}

int fhe_sign_batch(fhe_ctx* ctx, uint64_t* d_ct_v, int64_t count, uint64_t* d_sign, void* stream) {
  int rc = need_keys(ctx);
  if (rc) return rc;
  if (count < 0 || (count > 0 && (!d_ct_v || !d_sign))) return fail(ctx, FHE_E_ARG, "bad sign arguments");
  if (count == 0) return FHE_OK;
  rc = ensure_ws(ctx, 8 * (size_t)count * fhe_small_lwe_words(&ctx->p));
  if (rc) return rc;
  return sign_extract_batch(ctx, d_ct_v, count, d_sign, (uint64_t*)ctx->ws, (hipStream_t)stream);
}

int fhe_sign_trace_batch(fhe_ctx* ctx, uint64_t* d_ct_v, int64_t count, const int32_t* h_sched, int32_t rounds,
                         uint64_t* d_sign, uint32_t* d_phase, void* stream) {
  int rc = need_keys(ctx);
  if (rc) return rc;
  const fhe_params& p = ctx->p;
  int d, tmp[64];
  const int R = p.msg_bits < 4 ? p.msg_bits : sign_schedule(p, &d, tmp);
  if (count < 0 || rounds < 0 || rounds > R || (count > 0 && !d_ct_v) ||
      (count > 0 && (rounds == 0 || rounds == R) && !d_sign))
    return fail(ctx, FHE_E_ARG, "bad sign-trace arguments (0 <= rounds <= the plan's bootstraps; d_sign when the "
                                "last round runs)");
  int sched[64];
  if (h_sched) {
    for (int r = 0; r < R; ++r) {
      const int g = h_sched[r];
      if (g < 0 || g >= NGAD || (g > 0 && !fast_level(p, g)))
        return fail(ctx, FHE_E_ARG, "sign-trace schedule names a gadget these parameters do not have");
      sched[r] = g;
    }
  }
  if (count == 0) return FHE_OK;
  rc = ensure_ws(ctx, 8 * (size_t)count * fhe_small_lwe_words(&p));
  if (rc) return rc;
  SignTrace tr;
  tr.sched = h_sched ? sched : nullptr;
  tr.rounds = rounds;
  tr.phase = d_phase;
  return sign_extract(ctx, d_ct_v, count, d_sign, (uint64_t*)ctx->ws, (hipStream_t)stream, 0, &tr);
}

int fhe_bit_extract_batch(fhe_ctx* ctx, uint64_t* d_ct_v, int64_t count, uint64_t* d_refreshed, uint64_t* d_sign,
                          void* stream) {
  int rc = need_keys(ctx);
  if (rc) return rc;
  if (count < 0 || (count > 0 && (!d_ct_v || !d_refreshed || !d_sign)))
    return fail(ctx, FHE_E_ARG, "bad bit-extract arguments");
  if (count == 0) return FHE_OK;
  rc = ensure_ws(ctx, 8 * (size_t)count * fhe_small_lwe_words(&ctx->p));
  if (rc) return rc;
  return bit_extract(ctx, d_ct_v, count, d_refreshed, d_sign, (uint64_t*)ctx->ws, (hipStream_t)stream);
}

static int compare_impl(fhe_ctx* ctx, const int64_t* d_qx, int64_t B, int32_t D, const int64_t* d_w, int64_t cst,
                        int64_t T, const ChaKey& K, uint64_t id0, int64_t* d_acc, int64_t* d_below, void* stream) {
  int rc = need_keys(ctx);
  if (rc) return rc;
  if (B < 0 || D <= 0 || (B > 0 && (!d_qx || !d_w || !d_acc || !d_below)))
    return fail(ctx, FHE_E_ARG, "bad compare arguments");
  if (B == 0) return FHE_OK;
  const fhe_params& p = ctx->p;
  hipStream_t st = (hipStream_t)stream;
  const size_t Wb = fhe_big_lwe_words(&p), Ws = fhe_small_lwe_words(&p);
  // workspace: ct_v (B big) | sign (B big) | small (B) | v (B); the B x D
  // input ciphertexts are never materialised (k_encrypt_linear)
  const size_t bytes = 8 * (2 * (size_t)B * Wb + (size_t)B * Ws + (size_t)B);
  rc = ensure_ws(ctx, bytes);
  if (rc) return rc;
  u64* ctv = (u64*)ctx->ws;
  u64* sgn = ctv + (size_t)B * Wb;
  u64* small = sgn + (size_t)B * Wb;
  int64_t* v = (int64_t*)(small + (size_t)B * Ws);
  rc = encrypt_linear_impl(ctx, d_qx, B, D, K, id0, d_w, cst - T, ctv, stream);
  if (rc) return rc;
  // The score comes from the leveled accumulator ciphertext (noise ~2^20,
  // as in the reference's leveled Concrete circuit); the PBS chain then
  // computes the encrypted threshold bit [acc < T] exactly.
  rc = fhe_decrypt_batch(ctx, ctv, B, v, stream);
  if (rc) return rc;
  rc = sign_extract_batch(ctx, ctv, B, sgn, small, st);
  if (rc) return rc;
  rc = fhe_decrypt_bits_batch(ctx, sgn, B, d_below, stream);
  if (rc) return rc;
  hipLaunchKernelGGL(k_add_scalar, dim3((unsigned)((B + 255) / 256)), dim3(256), 0, st, v, B, T, d_acc);
  HIPCHK(ctx, hipGetLastError());
  return FHE_OK;
}
int fhe_compare_batch(fhe_ctx* ctx, const int64_t* d_qx, int64_t B, int32_t D, const int64_t* d_w, int64_t cst,
                      int64_t T, uint64_t enc_seed, uint64_t id0, int64_t* d_acc, int64_t* d_below, void* stream) {
  return compare_impl(ctx, d_qx, B, D, d_w, cst, T, key_from_seed(enc_seed), id0, d_acc, d_below, stream);
}
int fhe_compare_batch_key(fhe_ctx* ctx, const int64_t* d_qx, int64_t B, int32_t D, const int64_t* d_w, int64_t cst,
                          int64_t T, const uint32_t h_enc_key[8], uint64_t id0, int64_t* d_acc, int64_t* d_below,
                          void* stream) {
  ChaKey K;
  if (!key_arg(h_enc_key, K)) return fail(ctx, FHE_E_ARG, "null encryption key");
  return compare_impl(ctx, d_qx, B, D, d_w, cst, T, K, id0, d_acc, d_below, stream);
}

// The reference's own encrypted predict (fhe_similarity.py:142-160): the
// leveled circuit only. No key switch and no bootstrap; T only centres the
// accumulator in the msg_bits-bit encoding (acc - T must fit it).
static int score_impl(fhe_ctx* ctx, const int64_t* d_qx, int64_t B, int32_t D, const int64_t* d_w, int64_t cst,
                      int64_t T, const ChaKey& K, uint64_t id0, int64_t* d_acc, void* stream) {
  int rc = need_keys(ctx);
  if (rc) return rc;
  if (B < 0 || D <= 0 || (B > 0 && (!d_qx || !d_w || !d_acc))) return fail(ctx, FHE_E_ARG, "bad score arguments");
  if (B == 0) return FHE_OK;
  const fhe_params& p = ctx->p;
  hipStream_t st = (hipStream_t)stream;
  const size_t Wb = fhe_big_lwe_words(&p);
  // workspace: ct_v (B big) | v (B)
  rc = ensure_ws(ctx, 8 * ((size_t)B * Wb + (size_t)B));
  if (rc) return rc;
  u64* ctv = (u64*)ctx->ws;
  int64_t* v = (int64_t*)(ctv + (size_t)B * Wb);
  rc = encrypt_linear_impl(ctx, d_qx, B, D, K, id0, d_w, cst - T, ctv, stream);
  if (rc) return rc;
  rc = fhe_decrypt_batch(ctx, ctv, B, v, stream);
  if (rc) return rc;
  hipLaunchKernelGGL(k_add_scalar, dim3((unsigned)((B + 255) / 256)), dim3(256), 0, st, v, B, T, d_acc);
  HIPCHK(ctx, hipGetLastError());
  return FHE_OK;
}
int fhe_score_batch(fhe_ctx* ctx, const int64_t* d_qx, int64_t B, int32_t D, const int64_t* d_w, int64_t cst,
                    int64_t T, uint64_t enc_seed, uint64_t id0, int64_t* d_acc, void* stream) {
  return score_impl(ctx, d_qx, B, D, d_w, cst, T, key_from_seed(enc_seed), id0, d_acc, stream);
}
int fhe_score_batch_key(fhe_ctx* ctx, const int64_t* d_qx, int64_t B, int32_t D, const int64_t* d_w, int64_t cst,
                        int64_t T, const uint32_t h_enc_key[8], uint64_t id0, int64_t* d_acc, void* stream) {
  ChaKey K;
  if (!key_arg(h_enc_key, K)) return fail(ctx, FHE_E_ARG, "null encryption key");
  return score_impl(ctx, d_qx, B, D, d_w, cst, T, K, id0, d_acc, stream);
}

int fhe_compare_seeded_batch(fhe_ctx* ctx, const uint64_t* d_body, const uint64_t* d_id0, int64_t B, int32_t D,
                             const uint32_t h_mask_key[8], const int64_t* d_w, int64_t cst, int64_t T,
                             int64_t* d_acc, int64_t* d_below, void* stream) {
  int rc = need_keys(ctx);
  if (rc) return rc;
  if ((rc = seeded_args(ctx, B, D, d_body, d_id0, d_w))) return rc;
  if (!h_mask_key || (B > 0 && (!d_acc || !d_below))) return fail(ctx, FHE_E_ARG, "bad seeded compare arguments");
  if (B == 0) return FHE_OK;
  const fhe_params& p = ctx->p;
  hipStream_t st = (hipStream_t)stream;
  const size_t Wb = fhe_big_lwe_words(&p), Ws = fhe_small_lwe_words(&p);
  // workspace: ct_v (B big) | sign (B big) | small (B) | v (B)
  rc = ensure_ws(ctx, 8 * (2 * (size_t)B * Wb + (size_t)B * Ws + (size_t)B));
  if (rc) return rc;
  u64* ctv = (u64*)ctx->ws;
  u64* sgn = ctv + (size_t)B * Wb;
  u64* small = sgn + (size_t)B * Wb;
  int64_t* v = (int64_t*)(small + (size_t)B * Ws);
  rc = fhe_linear_seeded_batch(ctx, d_body, d_id0, B, D, h_mask_key, d_w, cst - T, ctv, stream);
  if (rc) return rc;
  rc = fhe_decrypt_batch(ctx, ctv, B, v, stream);
  if (rc) return rc;
  rc = sign_extract_batch(ctx, ctv, B, sgn, small, st);
  if (rc) return rc;
  rc = fhe_decrypt_bits_batch(ctx, sgn, B, d_below, stream);
  if (rc) return rc;
  hipLaunchKernelGGL(k_add_scalar, dim3((unsigned)((B + 255) / 256)), dim3(256), 0, st, v, B, T, d_acc);
  HIPCHK(ctx, hipGetLastError());
  return FHE_OK;
}

int fhe_threshold_batch(fhe_ctx* ctx, const uint64_t* d_ct_acc, int64_t count, int64_t T, uint64_t* d_bit,
                        void* stream) {
  int rc = need_keys(ctx);
  if (rc) return rc;
  if (count < 0 || (count > 0 && (!d_ct_acc || !d_bit))) return fail(ctx, FHE_E_ARG, "bad threshold arguments");
  if (count == 0) return FHE_OK;
  const fhe_params& p = ctx->p;
  hipStream_t st = (hipStream_t)stream;
  const size_t Wb = fhe_big_lwe_words(&p), Ws = fhe_small_lwe_words(&p);
  // workspace: v = acc - T (B big, consumed by the extraction) | small (B)
  rc = ensure_ws(ctx, 8 * ((size_t)count * Wb + (size_t)count * Ws));
  if (rc) return rc;
  u64* ctv = (u64*)ctx->ws;
  u64* small = ctv + (size_t)count * Wb;
  const int64_t words = count * (int64_t)Wb;
  hipLaunchKernelGGL(k_lwe_affine, dim3((unsigned)((words + 255) / 256)), dim3(256), 0, st, d_ct_acc, count, (int)Wb,
                     (u64)1, (u64)0 - ((u64)T << (64 - p.msg_bits)), ctv);
  HIPCHK(ctx, hipGetLastError());
  rc = sign_extract_batch(ctx, ctv, count, d_bit, small, st);
  if (rc) return rc;
  // [acc >= T] = 1 - [v < 0]: negate the sign ciphertext and add 2^63 to its body
  hipLaunchKernelGGL(k_lwe_affine, dim3((unsigned)((words + 255) / 256)), dim3(256), 0, st, d_bit, count, (int)Wb,
                     (u64)0 - 1, 1ull << 63, d_bit);
  HIPCHK(ctx, hipGetLastError());
  return FHE_OK;
}

void fhe_key_from_seed(uint64_t seed, uint32_t h_key_out[8]) {
  const ChaKey K = key_from_seed(seed);
  for (int i = 0; i < 8; ++i) h_key_out[i] = K.w[i];
}

int fhe_quantize_pairs(fhe_ctx* ctx, const void* d_query, int32_t query_is_f64, const void* d_docs,
                       int32_t docs_is_f64, int64_t B, int32_t D, double scale, int64_t zero_point, int64_t qmin,
                       int64_t qmax, int64_t* d_qx, void* stream) {
  int rc = need_device(ctx);
  if (rc) return rc;
  if (B < 0 || D <= 0 || (B > 0 && (!d_docs || !d_qx)) || !(scale > 0) || qmin > qmax)
    return fail(ctx, FHE_E_ARG, "bad quantize arguments");
  if (B == 0) return FHE_OK;
  const int64_t total = B * D;
  const dim3 g((unsigned)((total + 255) / 256)), b(256);
  hipStream_t st = (hipStream_t)stream;
  const double z = (double)zero_point, lo = (double)qmin, hi = (double)qmax;
#define QLAUNCH(QT, DT) \
  hipLaunchKernelGGL((k_pair_quantize<QT, DT>), g, b, 0, st, (const QT*)d_query, (const DT*)d_docs, B, D, scale, z, lo, hi, d_qx)
  if (query_is_f64 && docs_is_f64) QLAUNCH(double, double);
  else if (query_is_f64) QLAUNCH(double, float);
  else if (docs_is_f64) QLAUNCH(float, double);
  else QLAUNCH(float, float);
#undef QLAUNCH
  HIPCHK(ctx, hipGetLastError());
  return FHE_OK;
}

int fhe_pca_transform(fhe_ctx* ctx, const float* d_x, int64_t B, int32_t K, const float* d_mean,
                      const float* d_components, int32_t D, float* d_out, void* stream) {
  int rc = need_device(ctx);
  if (rc) return rc;
  if (B < 0 || K <= 0 || K > 1024 || D <= 0 || (B > 0 && (!d_x || !d_mean || !d_components || !d_out)))
    return fail(ctx, FHE_E_ARG, "bad pca arguments (1 <= K <= 1024, D >= 1)");
  if (B == 0) return FHE_OK;
  if (B > 0x7fffffffLL) return fail(ctx, FHE_E_ARG, "pca batch too large: split the call");
  hipLaunchKernelGGL(k_pca_transform, dim3((unsigned)B), dim3(256), 0, (hipStream_t)stream, d_x, (int)K, d_mean,
                     d_components, (int)D, d_out);
  HIPCHK(ctx, hipGetLastError());
  return FHE_OK;
}

int fhe_dequantize(fhe_ctx* ctx, const int64_t* d_acc, int64_t B, double out_scale, double* d_score, void* stream) {
  int rc = need_device(ctx);
  if (rc) return rc;
  if (B < 0 || (B > 0 && (!d_acc || !d_score))) return fail(ctx, FHE_E_ARG, "bad dequantize arguments");
  if (B == 0) return FHE_OK;
  hipLaunchKernelGGL(k_dequantize, dim3((unsigned)((B + 255) / 256)), dim3(256), 0, (hipStream_t)stream, d_acc, B,
                     out_scale, d_score);
  HIPCHK(ctx, hipGetLastError());
  return FHE_OK;
}

int fhe_topk(fhe_ctx* ctx, const int64_t* d_acc, const int64_t* d_below, int64_t B, int64_t base_idx, int32_t k,
             int64_t* d_out_acc, int64_t* d_out_idx, void* stream) {
  int rc = need_device(ctx);
  if (rc) return rc;
  if (B < 0 || k < 0 || (k > 0 && (!d_out_acc || !d_out_idx)) || (B > 0 && !d_acc))
    return fail(ctx, FHE_E_ARG, "bad topk arguments");
  if (k == 0) return FHE_OK;
  hipLaunchKernelGGL(k_topk, dim3(1), dim3(1024), 0, (hipStream_t)stream, d_acc, d_below, B, base_idx, k, d_out_acc,
                     d_out_idx);
  HIPCHK(ctx, hipGetLastError());
  return FHE_OK;
}

int fhe_dev_alloc(fhe_ctx* ctx, size_t bytes, void** d_out) {
  int rc = need_device(ctx);
  if (rc) return rc;
  if (!d_out) return fail(ctx, FHE_E_ARG, "null output pointer");
  *d_out = nullptr;
  if (bytes == 0) return FHE_OK;
  if (hipMalloc(d_out, bytes) != hipSuccess) {
    *d_out = nullptr;
    return fail(ctx, FHE_E_NOMEM, "hipMalloc failed");
  }
  return FHE_OK;
}

int fhe_dev_free(fhe_ctx* ctx, void* d_ptr) {
  int rc = need_device(ctx);
  if (rc) return rc;
  if (d_ptr) HIPCHK(ctx, hipFree(d_ptr));
  return FHE_OK;
}

int fhe_memcpy_h2d(fhe_ctx* ctx, void* d_dst, const void* h_src, size_t bytes, void* stream) {
  int rc = need_device(ctx);
  if (rc) return rc;
  if (bytes == 0) return FHE_OK;
  if (!d_dst || !h_src) return fail(ctx, FHE_E_ARG, "null copy pointer");
  HIPCHK(ctx, hipMemcpyAsync(d_dst, h_src, bytes, hipMemcpyHostToDevice, (hipStream_t)stream));
  return FHE_OK;
}

int fhe_memcpy_d2h(fhe_ctx* ctx, void* h_dst, const void* d_src, size_t bytes, void* stream) {
  int rc = need_device(ctx);
  if (rc) return rc;
  if (bytes == 0) return FHE_OK;
  if (!h_dst || !d_src) return fail(ctx, FHE_E_ARG, "null copy pointer");
  HIPCHK(ctx, hipMemcpyAsync(h_dst, d_src, bytes, hipMemcpyDeviceToHost, (hipStream_t)stream));
  HIPCHK(ctx, hipStreamSynchronize((hipStream_t)stream));
  return FHE_OK;
}

int fhe_stream_sync(fhe_ctx* ctx, void* stream) {
  int rc = need_device(ctx);
  if (rc) return rc;
  HIPCHK(ctx, hipStreamSynchronize((hipStream_t)stream));
  return FHE_OK;
}

int fhe_debug_v4_stamps(fhe_ctx* ctx, uint64_t* h_out) {
  int rc = need_device(ctx);
  if (rc) return rc;
  if (!h_out) return fail(ctx, FHE_E_ARG, "null output");
#ifndef FHEICP_AB
  return fail(ctx, FHE_E_STATE, "phase stamps need an A/B build (FHEICP_AB, tools/build_variant.sh)");
#endif
  HIPCHK(ctx, hipDeviceSynchronize());
  HIPCHK(ctx, hipMemcpyFromSymbol(h_out, HIP_SYMBOL(g_v4_stamps), sizeof(unsigned long long) * 64));
  HIPCHK(ctx, hipMemcpyFromSymbol(h_out + 64, HIP_SYMBOL(g_v4_span), sizeof(unsigned long long) * 2048 * 3));
  return FHE_OK;
}

int fhe_debug_el_stamps(fhe_ctx* ctx, uint64_t* h_out) {
  int rc = need_device(ctx);
  if (rc) return rc;
  if (!h_out) return fail(ctx, FHE_E_ARG, "null output");
#ifndef FHEICP_AB
  return fail(ctx, FHE_E_STATE, "phase stamps need an A/B build (FHEICP_AB, tools/build_variant.sh)");
#else
  HIPCHK(ctx, hipDeviceSynchronize());
  HIPCHK(ctx, hipMemcpyFromSymbol(h_out, HIP_SYMBOL(g_el_stamps), sizeof(unsigned long long) * 1024 * 4 * 10));
  return FHE_OK;
#endif
}

// FHEICP_SRC_SHA: sha256 (first 16 hex digits) of the sources the library was
// compiled from, passed by __graft_entry__.build_lib (tests/test_abi.py checks
// it against the tree, so a stale binary cannot pass for the current one)
#ifndef FHEICP_SRC_SHA
#define FHEICP_SRC_SHA "unknown"
#endif
const char* fhe_build_info(void) {
#ifdef FHEICP_AB
  return "libfheicp gfx950 ab=1 src=" FHEICP_SRC_SHA;
#else
  return "libfheicp gfx950 ab=0 src=" FHEICP_SRC_SHA;
#endif
}

static ProfAcc* prof_bucket(fhe_ctx* ctx, const char* kernel) {
  if (!strcmp(kernel, "blind_rotate") || !strcmp(kernel, "blind_rotate_main")) return &ctx->prof_br;
  if (!strcmp(kernel, "blind_rotate_fast")) return &ctx->prof_brf[0];
  if (!strcmp(kernel, "blind_rotate_fast2")) return &ctx->prof_brf[1];
  if (!strcmp(kernel, "blind_rotate_mid")) return &ctx->prof_brf[2];
  if (!strcmp(kernel, "blind_rotate_mid2")) return &ctx->prof_brf[3];
  if (!strcmp(kernel, "blind_rotate_mid0")) return &ctx->prof_brf[4];
  if (!strcmp(kernel, "keyswitch")) return &ctx->prof_ks;
  if (!strcmp(kernel, "encrypt_linear")) return &ctx->prof_enc;
  return nullptr;
}

int fhe_profile_kernel_name(fhe_ctx* ctx, const char* kernel, char* h_buf, size_t len) {
  if (!ctx) return fail(nullptr, FHE_E_ARG, "null ctx");
  if (!kernel || !h_buf || len == 0) return fail(ctx, FHE_E_ARG, "null kernel name or buffer");
  ProfAcc* a = prof_bucket(ctx, kernel);
  if (!a) return fail(ctx, FHE_E_ARG, "unknown kernel name");
  const char* nm = a->kernel ? a->kernel : "";
  snprintf(h_buf, len, "%s", nm);
  return FHE_OK;
}

int fhe_profile_enable(fhe_ctx* ctx, int enable) {
  if (!ctx) return fail(nullptr, FHE_E_ARG, "null ctx");
  ctx->prof = enable != 0;
  return FHE_OK;
}

int fhe_profile_read(fhe_ctx* ctx, const char* kernel, double* total_ms, int64_t* launches, int64_t* items) {
  int rc = need_device(ctx);
  if (rc) return rc;
  if (!kernel) return fail(ctx, FHE_E_ARG, "null kernel name");
  std::vector<ProfAcc*> acc;
  if (!strcmp(kernel, "blind_rotate"))
    acc = {&ctx->prof_br, &ctx->prof_brf[0], &ctx->prof_brf[1], &ctx->prof_brf[2], &ctx->prof_brf[3], &ctx->prof_brf[4]};
  else if (ProfAcc* a = prof_bucket(ctx, kernel)) acc = {a};
  else return fail(ctx, FHE_E_ARG, "unknown kernel name");
  double ms = 0;
  int64_t nl = 0, it = 0;
  for (ProfAcc* a : acc) {
    for (auto& e : a->ev) {
      HIPCHK(ctx, hipEventSynchronize(e.second));
      float x = 0;
      HIPCHK(ctx, hipEventElapsedTime(&x, e.first, e.second));
      ms += x;
    }
    nl += a->launches;
    it += a->items;
    free_ev(*a);
    a->launches = 0;
    a->items = 0;
  }
  if (total_ms) *total_ms = ms;
  if (launches) *launches = nl;
  if (items) *items = it;
  return FHE_OK;
}

}  // extern "C"
