// 3x3 / stride 1 / pad 1 convolution of the full-resolution decoder head, NHWC, as an
// implicit GEMM on MFMA with an LDS halo tile.  Replaces FinalPatchExpand_X4_V2's
// refine1 / refine2 (network/model_parts.py:447-448, :468-471) together with the ops
// around them:
//   * depth-to-space 4x4 of the expand output (model_parts.py:464-465) is folded into the
//     input addressing (IN_D2S) -- the d2s tensor and the NHWC->NCHW permute never exist;
//   * GELU of the conv input (model_parts.py:460, :469) is applied on load (IN_GELU), so
//     only pre-activations are stored;
//   * bias add in the epilogue; backward-data multiplies by GELU'(pre-activation) in the
//     epilogue and scatters through the same d2s map (OUT_D2S / OUT_GGRAD).
// fwd and dgrad share one kernel (dgrad = conv with spatially flipped, ci<->co swapped
// weights).  wgrad reads both operands k-strided from natural [pixel][channel] LDS images
// with ds_read_b64_tr_b16 (bf16) and writes deterministic per-block partials.
#include "common.h"
#include "mfma_frag.h"

namespace {

constexpr int TW = 16;  // output tile width (pixels) = one MFMA M tile

struct ConvGeom {
  int B, H, W;
  int Cin, CinP;   // GEMM input channels, padded to a multiple of 32
  int Cout;        // GEMM output channels (multiple of 16)
  int PS;          // LDS pixel stride (elements) of the input image
  int PSW;         // LDS row stride of the weight tile (fwd/dgrad)
  int PSD;         // LDS pixel stride of the dY tile (wgrad)
};

// element offset of channel 0 of pixel (b, y, x) of the logical [B,H,W,C] image
template <bool D2S>
MSU_DEV long pix_off(int b, int y, int x, int H, int W, int C) {
  if constexpr (D2S) {
    const int h4 = H >> 2, w4 = W >> 2;
    return (((long)b * h4 + (y >> 2)) * w4 + (x >> 2)) * (16L * C) + (long)(((y & 3) * 4 + (x & 3)) * C);
  } else {
    return (((long)b * H + y) * W + x) * (long)C;
  }
}

// Stage rows [y_first, y_first + nrows) x cols [x0 - 1, x0 + TW + 1) of the transformed
// input image (GELU optional) into LDS sX[(row * (TW+2) + col) * PS + c]; zero outside.
template <typename T, bool D2S, bool GELU>
MSU_DEV void stage_halo(const T* X, T* sX, int b, int y_first, int nrows, int x0, const ConvGeom& g,
                        int tid, int nthreads) {
  const int cpp = g.CinP / 8;  // 8-element chunks per pixel
  const int total = nrows * (TW + 2) * cpp;
  for (int i = tid; i < total; i += nthreads) {
    const int pix = i / cpp, ch = i - pix * cpp;
    const int row = pix / (TW + 2), col = pix - row * (TW + 2);
    const int y = y_first + row, x = x0 - 1 + col;
    float v[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = 0.f;
    if (y >= 0 && y < g.H && x >= 0 && x < g.W && ch * 8 < g.Cin) {
      const T* p = X + pix_off<D2S>(b, y, x, g.H, g.W, g.Cin) + ch * 8;
      float a[4], c[4];
      Vec4<T>::load(p, a);
      Vec4<T>::load(p + 4, c);
#pragma unroll
      for (int e = 0; e < 4; ++e) { v[e] = a[e]; v[4 + e] = c[e]; }
      if constexpr (GELU) {
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = gelu_f(v[e]);
      }
    }
    T* d = sX + pix * g.PS + ch * 8;
    float lo[4] = {v[0], v[1], v[2], v[3]}, hi[4] = {v[4], v[5], v[6], v[7]};
    Vec4<T>::store(d, lo);
    Vec4<T>::store(d + 4, hi);
  }
}

// acc += A(16 x 32) B(32 x 16) with both operands k-contiguous in LDS.
template <typename T> struct KC;
template <> struct KC<bf16_t> {
  static MSU_DEV void mma(f32x4& acc, const bf16_t* A, int lda, const bf16_t* B, int ldb, int lane) {
    const bf16x8 a = *reinterpret_cast<const bf16x8*>(A + (lane & 15) * lda + 8 * (lane >> 4));
    const bf16x8 b = *reinterpret_cast<const bf16x8*>(B + (lane & 15) * ldb + 8 * (lane >> 4));
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc, 0, 0, 0);
  }
  static MSU_DEV bf16x8 fragA(const bf16_t* A, int lda, int lane) {
    return *reinterpret_cast<const bf16x8*>(A + (lane & 15) * lda + 8 * (lane >> 4));
  }
};
template <> struct KC<float> {
  static MSU_DEV void mma(f32x4& acc, const float* A, int lda, const float* B, int ldb, int lane) {
    const float* pa = A + (lane & 15) * lda + (lane >> 4);
    const float* pb = B + (lane & 15) * ldb + (lane >> 4);
#pragma unroll
    for (int s = 0; s < 8; ++s) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(pa[4 * s], pb[4 * s], acc, 0, 0, 0);
  }
};

// ------------------------------------------------------------------ fwd / dgrad kernel
// Y[pixel][co] = sum_{tap, ci} Xt[pixel + off(tap)][ci] * Wt[tap][co][ci] (+ bias[co])
//               (* GELU'(S[pixel][co]) when OUT_GGRAD), Xt = GELU?(map(X)).
// Block = NWAVES waves = TH x 16 output pixels x all Cout; wave w owns MT image rows.
template <typename T, int NT, int TH, int MT, bool DB, bool IN_D2S, bool IN_GELU, bool OUT_D2S,
          bool OUT_GGRAD, bool BIAS>
__global__ void __launch_bounds__(64 * (TH / MT)) conv3x3_kernel(const T* __restrict__ X,
                                                                 const T* __restrict__ Wt,
                                                                 const float* __restrict__ bias,
                                                                 const T* __restrict__ S,
                                                                 T* __restrict__ Y, ConvGeom g) {
  constexpr int NWAVES = TH / MT;
  constexpr int NTHR = 64 * NWAVES;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  T* sX = reinterpret_cast<T*>(smem_raw);
  T* sW0 = sX + (TH + 2) * (TW + 2) * g.PS;
  T* sW1 = sW0 + g.Cout * g.PSW;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int tiles_x = (g.W + TW - 1) / TW, tiles_y = (g.H + TH - 1) / TH;
  const long ntiles = (long)g.B * tiles_x * tiles_y;
  const long tile = xcd_remap(blockIdx.x, gridDim.x);
  if (tile >= ntiles) return;
  const int b = (int)(tile / ((long)tiles_x * tiles_y));
  const int trem = (int)(tile - (long)b * tiles_x * tiles_y);
  const int y0 = (trem / tiles_x) * TH, x0 = (trem % tiles_x) * TW;

  stage_halo<T, IN_D2S, IN_GELU>(X, sX, b, y0 - 1, TH + 2, x0, g, tid, NTHR);
  // weight tile of tap t: Wt[t] is [Cout][CinP] contiguous -> sW[co * PSW + ci]
  const int wchunks = g.Cout * (g.CinP / 8);
  auto load_w = [&](int t, T* dst) {
    const T* src = Wt + (long)t * g.Cout * g.CinP;
    for (int i = tid; i < wchunks; i += NTHR) {
      const int co = i / (g.CinP / 8), ch = i - co * (g.CinP / 8);
      *reinterpret_cast<uint4*>(dst + co * g.PSW + ch * 8) =
          *reinterpret_cast<const uint4*>(src + (long)co * g.CinP + ch * 8);
    }
  };
  static_assert(sizeof(T) == 2 || !DB, "double-buffered weights only for bf16");
  if constexpr (sizeof(T) == 2) {
    load_w(0, sW0);
  } else {
    // f32: 8-element chunks are 32 bytes
    const float* src = reinterpret_cast<const float*>(Wt);
    for (int i = tid; i < g.Cout * g.CinP; i += NTHR) {
      const int co = i / g.CinP, ci = i - co * g.CinP;
      reinterpret_cast<float*>(sW0)[co * g.PSW + ci] = src[i];
    }
  }
  __syncthreads();

  f32x4 acc[MT][NT];
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int n = 0; n < NT; ++n) acc[m][n] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nks = g.CinP / 32;
  for (int tap = 0; tap < 9; ++tap) {
    const int dy = tap / 3, dx = tap - (tap / 3) * 3;
    T* sW = (DB && (tap & 1)) ? sW1 : sW0;
    if constexpr (DB) {
      if (tap + 1 < 9) load_w(tap + 1, (tap & 1) ? sW0 : sW1);
    }
    for (int ks = 0; ks < nks; ++ks) {
#pragma unroll
      for (int m = 0; m < MT; ++m) {
        const int hrow = wave * MT + m + dy;  // halo row
        const T* A = sX + (hrow * (TW + 2) + dx) * g.PS + ks * 32;
#pragma unroll
        for (int n = 0; n < NT; ++n)
          KC<T>::mma(acc[m][n], A, g.PS, sW + n * 16 * g.PSW + ks * 32, g.PSW, lane);
      }
    }
    __syncthreads();
    if constexpr (!DB) {
      if (tap + 1 < 9) {
        if constexpr (sizeof(T) == 2) {
          load_w(tap + 1, sW0);
        } else {
          const float* src = reinterpret_cast<const float*>(Wt) + (long)(tap + 1) * g.Cout * g.CinP;
          for (int i = tid; i < g.Cout * g.CinP; i += NTHR) {
            const int co = i / g.CinP, ci = i - co * g.CinP;
            reinterpret_cast<float*>(sW0)[co * g.PSW + ci] = src[i];
          }
        }
        __syncthreads();
      }
    }
  }

  // epilogue: lane holds pixel x0 + (lane>>4)*4 + r of row y0 + wave*MT + m, channel n*16 + (lane&15)
#pragma unroll
  for (int m = 0; m < MT; ++m) {
    const int y = y0 + wave * MT + m;
    if (y >= g.H) continue;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int x = x0 + (lane >> 4) * 4 + r;
      if (x >= g.W) continue;
      const long base = pix_off<OUT_D2S>(b, y, x, g.H, g.W, g.Cout);
#pragma unroll
      for (int n = 0; n < NT; ++n) {
        const int co = n * 16 + (lane & 15);
        float v = acc[m][n][r];
        if constexpr (BIAS) v += bias[co];
        if constexpr (OUT_GGRAD) v *= gelu_grad_f(to_f32(S[base + co]));
        Y[base + co] = from_f32<T>(v);
      }
    }
  }
}

// ------------------------------------------------------------------ wgrad kernel
// dW[dy][co][dx][ci] partial per block: sum over the block's pixel tiles of
//   DY[pixel][co] * Xt[pixel + (dy-1, dx-1)][ci];  one block = one dy, NT waves (one per
//   co tile), each wave 3 * CinP/16 n-tiles.  dbias partial from the dy == 0 blocks.

template <typename T, int NT, int NTI, int TH, bool IN_D2S, bool IN_GELU>
__global__ void __launch_bounds__(64 * NT) conv3x3_wgrad_kernel(const T* __restrict__ X,
                                                                const T* __restrict__ DY,
                                                                float* __restrict__ part,
                                                                float* __restrict__ dbpart,
                                                                ConvGeom g, int nchunk) {
  // NT = Cout/16 (waves), NTI = CinP/16 (ci tiles per dx)
  constexpr int NTHR = 64 * NT;
  constexpr int NPIX = TH * TW;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  T* sX = reinterpret_cast<T*>(smem_raw);         // [TH][TW+2][PS]
  T* sD = sX + TH * (TW + 2) * g.PS;              // [NPIX][PSD]   (PSD = Cout + pad)
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int w = xcd_remap(blockIdx.x, gridDim.x);
  const int dy = w % 3, chunk = w / 3;
  const int tiles_x = (g.W + TW - 1) / TW, tiles_y = (g.H + TH - 1) / TH;
  const long ntiles = (long)g.B * tiles_x * tiles_y;

  f32x4 acc[3][NTI];
#pragma unroll
  for (int d = 0; d < 3; ++d)
#pragma unroll
    for (int n = 0; n < NTI; ++n) acc[d][n] = f32x4{0.f, 0.f, 0.f, 0.f};
  float dbacc = 0.f;

  for (long tile = chunk; tile < ntiles; tile += nchunk) {
    const int b = (int)(tile / ((long)tiles_x * tiles_y));
    const int trem = (int)(tile - (long)b * tiles_x * tiles_y);
    const int y0 = (trem / tiles_x) * TH, x0 = (trem % tiles_x) * TW;
    __syncthreads();
    stage_halo<T, IN_D2S, IN_GELU>(X, sX, b, y0 + dy - 1, TH, x0, g, tid, NTHR);
    // dY tile [NPIX][Cout]: rows outside the image are zero
    {
      const int cpp = g.Cout / 8;
      for (int i = tid; i < NPIX * cpp; i += NTHR) {
        const int pix = i / cpp, ch = i - pix * cpp;
        const int y = y0 + pix / TW, x = x0 + pix % TW;
        float v[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = 0.f;
        if (y < g.H && x < g.W) {
          const T* p = DY + (((long)b * g.H + y) * g.W + x) * g.Cout + ch * 8;
          float a[4], c[4];
          Vec4<T>::load(p, a);
          Vec4<T>::load(p + 4, c);
#pragma unroll
          for (int e = 0; e < 4; ++e) { v[e] = a[e]; v[4 + e] = c[e]; }
        }
        float lo[4] = {v[0], v[1], v[2], v[3]}, hi[4] = {v[4], v[5], v[6], v[7]};
        Vec4<T>::store(sD + pix * g.PSD + ch * 8, lo);
        Vec4<T>::store(sD + pix * g.PSD + ch * 8 + 4, hi);
      }
    }
    __syncthreads();
    if (dy == 0 && tid < g.Cout) {
      for (int p = 0; p < NPIX; ++p) dbacc += to_f32(sD[p * g.PSD + tid]);
    }
    auto rowA = [&](int k) { return sD + k * g.PSD; };
#pragma unroll
    for (int ks = 0; ks < NPIX / 32; ++ks) {
#pragma unroll
      for (int d = 0; d < 3; ++d) {
        auto rowB = [&](int k) { return sX + ((k / TW) * (TW + 2) + (k % TW) + d) * g.PS; };
#pragma unroll
        for (int n = 0; n < NTI; ++n)
          TR<T>::mma(acc[d][n], rowA, wave * 16, rowB, n * 16, ks * 32, lane);
      }
    }
  }
  // partial [blk][dy][co][dx][ci]   (co = wave*16 + row, ci = n*16 + (lane&15))
  float* out = part + ((long)chunk * 3 + dy) * (long)g.Cout * 3 * g.CinP;
#pragma unroll
  for (int d = 0; d < 3; ++d)
#pragma unroll
    for (int n = 0; n < NTI; ++n)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int co = wave * 16 + (lane >> 4) * 4 + r;
        const int ci = n * 16 + (lane & 15);
        out[((long)co * 3 + d) * g.CinP + ci] = acc[d][n][r];
      }
  if (dy == 0 && tid < g.Cout) dbpart[(long)chunk * g.Cout + tid] = dbacc;
}

// sum partials -> dW[co][ci][3][3] (torch Conv2d layout) and db[co]
__global__ void __launch_bounds__(256) wgrad_reduce_kernel(const float* part, const float* dbpart,
                                                           int nchunk, int Cout, int Cin, int CinP,
                                                           float* dW, float* db) {
  const long n = (long)Cout * Cin * 9;
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i < n) {
    const int co = (int)(i / (Cin * 9));
    const int rem = (int)(i - (long)co * Cin * 9);
    const int ci = rem / 9, tap = rem % 9, dy = tap / 3, dx = tap % 3;
    const long slab = (long)Cout * 3 * CinP;
    float s = 0.f;
    for (int c = 0; c < nchunk; ++c)
      s += part[((long)c * 3 + dy) * slab + ((long)co * 3 + dx) * CinP + ci];
    dW[i] = s;
  }
  if (db && i < Cout) {
    float s = 0.f;
    for (int c = 0; c < nchunk; ++c) s += dbpart[(long)c * Cout + i];
    db[i] = s;
  }
}

// ------------------------------------------------------------------ host dispatch
ConvGeom make_geom(int B, int H, int W, int Cin, int Cout, int elem_bytes) {
  ConvGeom g;
  g.B = B; g.H = H; g.W = W; g.Cin = Cin; g.Cout = Cout;
  g.CinP = (Cin + 31) / 32 * 32;
  const int pad = elem_bytes == 2 ? 8 : 4;
  g.PS = g.CinP + pad;
  g.PSW = g.CinP + pad;
  g.PSD = Cout + pad;
  return g;
}

template <typename T, int NT, bool IN_D2S, bool IN_GELU, bool OUT_D2S, bool OUT_GGRAD, bool BIAS>
int launch_conv(const ConvGeom& g, const T* X, const T* Wt, const float* bias, const T* S, T* Y,
                hipStream_t st) {
  constexpr bool BF = sizeof(T) == 2;
  constexpr int TH = BF ? 16 : 4;
  constexpr int MT = BF ? 2 : 1;
  constexpr int NW = TH / MT;
  const size_t lds = sizeof(T) * ((size_t)(TH + 2) * (TW + 2) * g.PS + (size_t)(BF ? 2 : 1) * g.Cout * g.PSW);
  if (lds > 160 * 1024) return -4;
  auto kern = conv3x3_kernel<T, NT, TH, MT, BF, IN_D2S, IN_GELU, OUT_D2S, OUT_GGRAD, BIAS>;
  static bool attr_set = false;
  if (!attr_set) {
    hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr_set = true;
  }
  const long ntiles = (long)g.B * ((g.W + TW - 1) / TW) * ((g.H + TH - 1) / TH);
  if (ntiles == 0) return 0;
  hipLaunchKernelGGL(kern, dim3((unsigned)ntiles), dim3(64 * NW), lds, st, X, Wt, bias, S, Y, g);
  return MSU_CHECK_LAUNCH();
}

template <typename T, bool IN_D2S, bool IN_GELU, bool OUT_D2S, bool OUT_GGRAD, bool BIAS>
int conv_nt(const ConvGeom& g, const void* X, const void* Wt, const float* bias, const void* S,
            void* Y, hipStream_t st) {
  const T* x = (const T*)X; const T* w = (const T*)Wt; const T* s = (const T*)S; T* y = (T*)Y;
  switch (g.Cout / 16) {
    case 1: return launch_conv<T, 1, IN_D2S, IN_GELU, OUT_D2S, OUT_GGRAD, BIAS>(g, x, w, bias, s, y, st);
    case 2: return launch_conv<T, 2, IN_D2S, IN_GELU, OUT_D2S, OUT_GGRAD, BIAS>(g, x, w, bias, s, y, st);
    case 4: return launch_conv<T, 4, IN_D2S, IN_GELU, OUT_D2S, OUT_GGRAD, BIAS>(g, x, w, bias, s, y, st);
    case 6: return launch_conv<T, 6, IN_D2S, IN_GELU, OUT_D2S, OUT_GGRAD, BIAS>(g, x, w, bias, s, y, st);
    case 8: return launch_conv<T, 8, IN_D2S, IN_GELU, OUT_D2S, OUT_GGRAD, BIAS>(g, x, w, bias, s, y, st);
  }
  return -2;
}

template <typename T, int NT, bool IN_D2S, bool IN_GELU>
int launch_wgrad_nti(const ConvGeom& g, const T* X, const T* DY, float* part, float* dbpart,
                     int nchunk, hipStream_t st) {
  constexpr int TH = 8;
  const size_t lds = sizeof(T) * ((size_t)TH * (TW + 2) * g.PS + (size_t)TH * TW * g.PSD);
  if (lds > 160 * 1024) return -4;
  auto go = [&](auto kern) {
    hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    hipLaunchKernelGGL(kern, dim3((unsigned)(nchunk * 3)), dim3(64 * NT), lds, st, X, DY, part, dbpart, g, nchunk);
    return MSU_CHECK_LAUNCH();
  };
  switch (g.CinP / 16) {
    case 2: return go(conv3x3_wgrad_kernel<T, NT, 2, TH, IN_D2S, IN_GELU>);
    case 4: return go(conv3x3_wgrad_kernel<T, NT, 4, TH, IN_D2S, IN_GELU>);
    case 6: return go(conv3x3_wgrad_kernel<T, NT, 6, TH, IN_D2S, IN_GELU>);
    case 8: return go(conv3x3_wgrad_kernel<T, NT, 8, TH, IN_D2S, IN_GELU>);
  }
  return -2;
}

template <typename T, bool IN_D2S, bool IN_GELU>
int wgrad_nt(const ConvGeom& g, const void* X, const void* DY, float* part, float* dbpart,
             int nchunk, hipStream_t st) {
  const T* x = (const T*)X; const T* d = (const T*)DY;
  switch (g.Cout / 16) {
    case 1: return launch_wgrad_nti<T, 1, IN_D2S, IN_GELU>(g, x, d, part, dbpart, nchunk, st);
    case 2: return launch_wgrad_nti<T, 2, IN_D2S, IN_GELU>(g, x, d, part, dbpart, nchunk, st);
    case 4: return launch_wgrad_nti<T, 4, IN_D2S, IN_GELU>(g, x, d, part, dbpart, nchunk, st);
    case 6: return launch_wgrad_nti<T, 6, IN_D2S, IN_GELU>(g, x, d, part, dbpart, nchunk, st);
    case 8: return launch_wgrad_nti<T, 8, IN_D2S, IN_GELU>(g, x, d, part, dbpart, nchunk, st);
  }
  return -2;
}

}  // namespace

extern "C" {

// in_mode bit 0: GELU on the loaded input, bit 1: input is the pre-d2s [B,H/4,W/4,16*Cin]
// tensor.  Wt: [9][Cout][CinP] (CinP = roundup(Cin, 32), zero padded), dtype of X.
int msu_conv3x3_fwd(int dtype, int in_mode, const void* X, const void* Wt, const float* bias,
                    void* Y, int B, int H, int W, int Cin, int Cout, void* stream) {
  if (Cout % 16 || Cin % 8 || Cout > 128 || Cin > 128) return -2;
  if ((in_mode & 2) && (H % 4 || W % 4)) return -2;
  const ConvGeom g = make_geom(B, H, W, Cin, Cout, dtype == MSU_BF16 ? 2 : 4);
  hipStream_t st = (hipStream_t)stream;
  if (bias == nullptr) return -2;
#define MSU_FWD(T, D2S, GL) return conv_nt<T, D2S, GL, false, false, true>(g, X, Wt, bias, nullptr, Y, st)
  // instantiated modes: GELU on load (the refine convs' inputs are always GELU outputs)
  if (dtype == MSU_BF16) {
    switch (in_mode & 3) {
      case 1: MSU_FWD(bf16_t, false, true);
      case 3: MSU_FWD(bf16_t, true, true);
    }
  } else {
    switch (in_mode & 3) {
      case 1: MSU_FWD(float, false, true);
      case 3: MSU_FWD(float, true, true);
    }
  }
#undef MSU_FWD
  return -3;
}

// dX = (conv(dY, Wflip) * GELU'(S)) scattered through the input map.  Wflip: [9][Cin][CoutP]
// with Wflip[t][ci][co] = W[co][ci][8-t].  out_mode bit 0: multiply by GELU'(S), bit 1:
// dX / S live in the pre-d2s layout.  Here the GEMM input channels are Cout (of the
// forward conv) and the GEMM outputs are Cin.
int msu_conv3x3_dgrad(int dtype, int out_mode, const void* dY, const void* Wflip, const void* S,
                      void* dX, int B, int H, int W, int Cin, int Cout, void* stream) {
  if (Cout % 16 || Cin % 16 || Cout > 128 || Cin > 128) return -2;
  if ((out_mode & 2) && (H % 4 || W % 4)) return -2;
  const ConvGeom g = make_geom(B, H, W, Cout, Cin, dtype == MSU_BF16 ? 2 : 4);
  hipStream_t st = (hipStream_t)stream;
#define MSU_DG(T, D2S, GG) return conv_nt<T, false, false, D2S, GG, false>(g, dY, Wflip, nullptr, S, dX, st)
  if (dtype == MSU_BF16) {
    switch (out_mode & 3) {
      case 1: MSU_DG(bf16_t, false, true);
      case 3: MSU_DG(bf16_t, true, true);
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

long msu_conv3x3_wgrad_workspace(int nchunk, int Cin, int Cout, int dtype, int unused) {
  (void)dtype; (void)unused;
  const int CinP = (Cin + 31) / 32 * 32;
  return (long)nchunk * 3 * Cout * 3 * CinP + (long)nchunk * Cout;
}

// dW [Cout][Cin][3][3] f32 and db [Cout] f32 (db may be null).  in_mode as in fwd.
int msu_conv3x3_wgrad(int dtype, int in_mode, const void* X, const void* dY, float* dW, float* db,
                      float* workspace, void* unused, int nchunk, int B, int H, int W, int Cin,
                      int Cout, void* stream) {
  (void)unused;
  if (Cout % 16 || Cin % 8 || Cout > 128 || Cin > 128 || nchunk < 1) return -2;
  const ConvGeom g = make_geom(B, H, W, Cin, Cout, dtype == MSU_BF16 ? 2 : 4);
  hipStream_t st = (hipStream_t)stream;
  float* part = workspace;
  float* dbpart = workspace + (long)nchunk * 3 * Cout * 3 * g.CinP;
  int rc = -3;
#define MSU_WG(T, D2S, GL) rc = wgrad_nt<T, D2S, GL>(g, X, dY, part, dbpart, nchunk, st)
  if (dtype == MSU_BF16) {
    switch (in_mode & 3) {
      case 1: MSU_WG(bf16_t, false, true); break;
      case 3: MSU_WG(bf16_t, true, true); break;
    }
  } else {
    switch (in_mode & 3) {
      case 1: MSU_WG(float, false, true); break;
      case 3: MSU_WG(float, true, true); break;
    }
  }
#undef MSU_WG
  if (rc) return rc;
  const long n = (long)Cout * Cin * 9;
  hipLaunchKernelGGL(wgrad_reduce_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, part,
                     dbpart, nchunk, Cout, Cin, g.CinP, dW, db);
  return MSU_CHECK_LAUNCH();
}

}  // extern "C"
