// Refine-conv forward and backward-data entry points (kernels: conv3x3.h).
#include "conv3x3.h"

extern "C" {

// in_mode bit 0: GELU on the loaded input, bit 1: input is the pre-d2s [B,H/4,W/4,16*Cin]
// tensor.  Wt: [9][Cout][CinP] (CinP = roundup(Cin, 32), zero padded), dtype of X.
// Y2 (may be null, only without GELU on load): GELU(Y) written by the same epilogue.
int msu_conv3x3_fwd2(int dtype, int in_mode, const void* X, const void* Wt, const float* bias,
                     void* Y, void* Y2, int B, int H, int W, int Cin, int Cout, void* stream) {
  if (Cout % 16 || Cin % 8 || Cout > 128 || Cin > 128) return -2;
  if ((in_mode & 2) && (H % 4 || W % 4)) return -2;
  if (Y2 && (in_mode & 1)) return -2;
  const ConvGeom g = make_geom(B, H, W, Cin, Cout, msu_is16(dtype) ? 2 : 4);
  hipStream_t st = (hipStream_t)stream;
  if (bias == nullptr) return -2;
#define MSU_FWD(T, D2S, GL, DU) return conv_nt<T, D2S, GL, false, false, true, DU>(g, X, Wt, bias, nullptr, Y, Y2, st)
#define MSU_FWD_ALL(T)                              \
  switch ((in_mode & 3) | (Y2 ? 4 : 0)) {           \
    case 0: MSU_FWD(T, false, false, false);        \
    case 1: MSU_FWD(T, false, true, false);         \
    case 2: MSU_FWD(T, true, false, false);         \
    case 3: MSU_FWD(T, true, true, false);          \
    case 4: MSU_FWD(T, false, false, true);         \
    case 6: MSU_FWD(T, true, false, true);          \
  }
  if (dtype == MSU_BF16) {
    MSU_FWD_ALL(bf16_t)
  } else if (dtype == MSU_F16) {
    MSU_FWD_ALL(f16_t)
  } else {
    MSU_FWD_ALL(float)
  }
#undef MSU_FWD_ALL
#undef MSU_FWD
  return -3;
}

int msu_conv3x3_fwd(int dtype, int in_mode, const void* X, const void* Wt, const float* bias,
                    void* Y, int B, int H, int W, int Cin, int Cout, void* stream) {
  return msu_conv3x3_fwd2(dtype, in_mode, X, Wt, bias, Y, nullptr, B, H, W, Cin, Cout, stream);
}

// dX = (conv(dY, Wflip) * GELU'(S)) scattered through the input map.  Wflip: [9][Cin][CoutP]
// with Wflip[t][ci][co] = W[co][ci][8-t].  out_mode bit 0: multiply by GELU'(S), bit 1:
// dX / S live in the pre-d2s layout.  Here the GEMM input channels are Cout (of the
// forward conv) and the GEMM outputs are Cin.
int msu_conv3x3_dgrad(int dtype, int out_mode, const void* dY, const void* Wflip, const void* S,
                      void* dX, int B, int H, int W, int Cin, int Cout, void* stream) {
  if (Cout % 16 || Cin % 16 || Cout > 128 || Cin > 128) return -2;
  if ((out_mode & 2) && (H % 4 || W % 4)) return -2;
  const ConvGeom g = make_geom(B, H, W, Cout, Cin, msu_is16(dtype) ? 2 : 4);
  hipStream_t st = (hipStream_t)stream;
#define MSU_DG(T, D2S, GG) return conv_nt<T, false, false, D2S, GG, false>(g, dY, Wflip, nullptr, S, dX, nullptr, st)
  if (dtype == MSU_BF16) {
    switch (out_mode & 3) {
      case 1: MSU_DG(bf16_t, false, true);
      case 3: MSU_DG(bf16_t, true, true);
    }
  } else if (dtype == MSU_F16) {
    switch (out_mode & 3) {
      case 1: MSU_DG(f16_t, false, true);
      case 3: MSU_DG(f16_t, true, true);
    }
  } else {
    switch (out_mode & 3) {
      case 1: MSU_DG(float, false, true);
      case 3: MSU_DG(float, true, true);
    }
  }
#undef MSU_DG
  return -3;
}

// bit 0: the refine-conv kernel's tile queue (g_conv_dyn); returns the previous mode
int msu_conv_mode(int mode) {
  const int prev = g_conv_dyn;
  g_conv_dyn = mode & 1;
  return prev;
}

}  // extern "C"
