// Refine-conv weight-gradient entry points (kernels: conv3x3.h).
#include "conv3x3.h"

extern "C" {

long msu_conv3x3_wgrad_workspace(int nchunk, int Cin, int Cout, int dtype, int unused) {
  (void)dtype; (void)unused;
  const int CinP = (Cin + 31) / 32 * 32;
  // chunk partials [nchunk][3][Cout][3][CinP] + bias partials [nchunk][Cout] + their sum
  return (long)(nchunk + 1) * 3 * Cout * 3 * CinP + (long)nchunk * Cout;
}

// dW [Cout][Cin][3][3] f32 and db [Cout] f32 (db may be null), overwritten or (accumulate != 0)
// added to.  in_mode as in fwd.
int msu_conv3x3_wgrad2(int dtype, int in_mode, const void* X, const void* dY, float* dW, float* db,
                       float* workspace, int nchunk, int B, int H, int W, int Cin, int Cout, int accumulate,
                       void* stream) {
  if (Cout % 16 || Cin % 8 || Cout > 128 || Cin > 128 || nchunk < 1) return -2;
  const ConvGeom g = make_geom(B, H, W, Cin, Cout, msu_is16(dtype) ? 2 : 4);
  hipStream_t st = (hipStream_t)stream;
  float* part = workspace;
  float* dbpart = workspace + (long)nchunk * 3 * Cout * 3 * g.CinP;
  int rc = -3;
#define MSU_WG(T, D2S, GL) rc = wgrad_nt<T, D2S, GL>(g, X, dY, part, dbpart, nchunk, st)
  if (msu_is16(dtype) && Cin == 96 && Cout == 96) {
    const bf16_t* x = (const bf16_t*)X; const bf16_t* d = (const bf16_t*)dY;
    MSU_DISPATCH16(dtype, T,
      switch (in_mode & 3) {
        case 0: rc = launch_wgrad_v2<T, false, false>(g, x, d, part, dbpart, nchunk, st); break;
        case 1: rc = launch_wgrad_v2<T, false, true>(g, x, d, part, dbpart, nchunk, st); break;
        case 2: rc = launch_wgrad_v2<T, true, false>(g, x, d, part, dbpart, nchunk, st); break;
        case 3: rc = launch_wgrad_v2<T, true, true>(g, x, d, part, dbpart, nchunk, st); break;
      });
  } else if (msu_is16(dtype)) {
    MSU_DISPATCH16(dtype, T,
      switch (in_mode & 3) {
        case 0: MSU_WG(T, false, false); break;
        case 1: MSU_WG(T, false, true); break;
        case 2: MSU_WG(T, true, false); break;
        case 3: MSU_WG(T, true, true); break;
      });
  } else {
    switch (in_mode & 3) {
      case 0: MSU_WG(float, false, false); break;
      case 1: MSU_WG(float, false, true); break;
      case 2: MSU_WG(float, true, false); break;
      case 3: MSU_WG(float, true, true); break;
    }
  }
#undef MSU_WG
  if (rc) return rc;
  // deterministic chunk sums (one launch for the weight slab and the bias), then the
  // [dy][co][dx][ci] -> [co][ci][dy][dx] permutation
  const long slab = 3L * Cout * 3 * g.CinP;
  float* sum = dbpart + (long)nchunk * Cout;
  const ColSeg segs[2] = {{part, slab, slab, sum}, {dbpart, Cout, Cout, db}};
  // (the slab sum is workspace, always overwritten; db and the permuted dW accumulate)
  colsum_multi(segs, db ? 2 : 1, nchunk, 0, st, accumulate ? 2 : 0);
  const long n = (long)Cout * Cin * 9;
  hipLaunchKernelGGL(wgrad_permute_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, sum, Cout, Cin,
                     g.CinP, dW, accumulate);
  return MSU_CHECK_LAUNCH();
}

int msu_conv3x3_wgrad(int dtype, int in_mode, const void* X, const void* dY, float* dW, float* db,
                      float* workspace, void* unused, int nchunk, int B, int H, int W, int Cin,
                      int Cout, void* stream) {
  (void)unused;
  return msu_conv3x3_wgrad2(dtype, in_mode, X, dY, dW, db, workspace, nchunk, B, H, W, Cin, Cout, 0, stream);
}

}  // extern "C"
