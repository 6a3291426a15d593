// Token GEMM planner and C-ABI entry points (kernel: gemm_tok.h).
#include <stdlib.h>

#include "gemm_tok.h"

namespace msu_tok {
namespace {

// Stage depth: the largest instantiated one dividing K.  Chunk width: the widest
// instantiated multiple of 32 dividing N whose W image fits in LDS next to a 3-deep ring
// (else a 2-deep one when that halves the chunk count).
TokPlan tok_plan(long M, int N, int K, int epi = EPI_PLAIN) {
  TokPlan p;
  static const int kcs[] = {96, 128, 48};
  for (int kc : kcs)
    if (K % kc == 0) { p.kc = kc; break; }
  if (!p.kc) return p;
  static const int ncs[] = {384, 288, 256, 192, 128, 96, 64};
  int best[2] = {0, 0};
  for (int i = 0; i < 2; ++i) {
    const int nst = 3 - i;
    for (int nc : ncs) {
      if (N % nc) continue;
      if (epi != EPI_PLAIN && nc > 192) continue;  // GELU epilogue registers
      if (plan_lds(p.kc, nc, nst, K) > LDS_MAX) continue;
      best[i] = nc;
      break;
    }
  }
  int nst = 3;
  if (best[1] >= 2 * best[0]) nst = 2;
  p.nc = best[3 - nst];
  if (!p.nc) { nst = 2; p.nc = best[1]; }
  if (!p.nc) return p;
  p.nst = nst;
  p.lds = plan_lds(p.kc, p.nc, nst, K);
  // eight waves with 2-deep rings when the W chunk leaves room (8 vs 4 waves measured equal
  // within noise on two boxes, r02c: kept)
  if (plan_lds(p.kc, p.nc, 2, K, 8) <= LDS_MAX) {
    p.nst = 2;
    p.nw = 8;
    p.lds = plan_lds(p.kc, p.nc, 2, K, 8);
  }
  p.nchunk = N / p.nc;
  const int per_cu = (p.nw == 4 && 2 * p.lds <= LDS_MAX) ? 2 : 1;
  int groups = (256 * per_cu) / (8 * p.nchunk);
  if (groups < 1) groups = 1;
  const long ntiles = (M + RT - 1) / RT;
  const long max_groups = (ntiles + 8L * p.nw - 1) / (8L * p.nw);  // every wave gets a tile
  if (groups > max_groups) groups = (int)(max_groups < 1 ? 1 : max_groups);
  p.grid = 8 * p.nchunk * groups;
  return p;
}

}  // namespace
}  // namespace msu_tok

using namespace msu_tok;

extern "C" {

// 1 if the token GEMM covers (M, N, K); otherwise the caller uses a library GEMM.
int msu_tok_gemm_supported(long M, int N, int K) {
  if (M <= 0 || N % 32 || K % 16) return 0;
  return tok_plan(M, N, K).nc ? 1 : 0;
}

// Same for a given epilogue (the GELU epilogues cap the chunk width at 192 columns).
int msu_tok_gemm_supported_epi(long M, int N, int K, int epi) {
  if (M <= 0 || N % 32 || K % 16 || epi < 0 || epi > 2) return 0;
  return tok_plan(M, N, K, epi).nc ? 1 : 0;
}

// Y[M][N] = epi(A . W^T + bias), bf16 in / out.  epi 0: plain (+ bias); 1: Y = H and
// Y2 = GELU(H) (needs bias); 2: Y = (A . W^T) * GELU'(H) (no bias).  A2 != null: columns
// [K1, K) of A come from A2 ([M][K - K1]; needs bias).
int msu_tok_gemm(int dtype, const void* A, const void* A2, int K1, const void* W, const float* bias, void* Y,
                 void* Y2, const void* H, long M, int N, int K, int epi, void* stream) {
  if (!msu_is16(dtype)) return -3;
  if (M < 0 || N % 32 || K % 16) return -2;
  if (M == 0) return 0;
  if (A2 != nullptr && (K1 <= 0 || K1 >= K || K1 % 8)) return -2;
  if (epi == EPI_GELU_DUAL && (Y2 == nullptr || bias == nullptr || A2 != nullptr)) return -3;
  if (epi == EPI_GELU_GRAD && (H == nullptr || bias != nullptr || A2 != nullptr)) return -3;
  if (epi == EPI_PLAIN && A2 != nullptr && bias == nullptr) return -3;
  if (epi < 0 || epi > 2) return -3;
  const TokPlan p = tok_plan(M, N, K, epi);
  if (!p.nc) return -3;
  TokArgs a;
  a.A = (const bf16_t*)A;
  a.A2 = (const bf16_t*)A2;
  a.K1 = A2 ? K1 : K;
  a.W = (const bf16_t*)W;
  a.bias = bias;
  a.Y = (bf16_t*)Y;
  a.Y2 = (bf16_t*)Y2;
  a.H = (const bf16_t*)H;
  a.M = M;
  a.N = N;
  a.K = K;
  a.nchunk = p.nchunk;
  a.rgroups = p.grid / p.nchunk;
  hipStream_t st = (hipStream_t)stream;
  const bool has_bias = bias != nullptr, concat = A2 != nullptr;
  int rc = -3;
  switch (p.kc) {
    case 96: rc = dispatch_k96(dtype, p, a, epi, has_bias, concat, st); break;
    case 128: rc = dispatch_k128(dtype, p, a, epi, has_bias, concat, st); break;
    case 48: rc = dispatch_k48(dtype, p, a, epi, has_bias, concat, st); break;
  }
  if (rc) return rc;
  return MSU_CHECK_LAUNCH();
}

// Plan introspection for tests / benchmarks: out6 = {kc, nc, nst, nchunk, grid, lds bytes}.
int msu_tok_gemm_plan(long M, int N, int K, long* out6) {
  const TokPlan p = tok_plan(M, N, K);
  out6[0] = p.kc; out6[1] = p.nc; out6[2] = p.nst * 100 + p.nw; out6[3] = p.nchunk; out6[4] = p.grid;
  out6[5] = (long)p.lds;
  return p.nc ? 0 : -3;
}

}  // extern "C"
