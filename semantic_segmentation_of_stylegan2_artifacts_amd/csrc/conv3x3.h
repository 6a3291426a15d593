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
#pragma once
#include <cstdlib>
#include <utility>

#include "common.h"
#include "mfma_frag.h"
#include "reduce.h"

// MSU_EXP: ablation bits for timing experiments only (tools/build_exp.sh); 0 in every real build
#ifndef MSU_EXP
#define MSU_EXP 0
#endif

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

// 32-bit variant (tensors below 2^31 elements; checked on the host)
template <bool D2S>
MSU_DEV int pix_off32(int b, int y, int x, int H, int W, int C) {
  if constexpr (D2S) {
    const int h4 = H >> 2, w4 = W >> 2;
    return ((b * h4 + (y >> 2)) * w4 + (x >> 2)) * (16 * C) + ((y & 3) * 4 + (x & 3)) * C;
  } else {
    return ((b * H + y) * W + x) * C;
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
template <typename T> struct KC16 {
  static MSU_DEV void mma(f32x4& acc, const T* A, int lda, const T* B, int ldb, int lane) {
    const bf16x8 a = *reinterpret_cast<const bf16x8*>(A + (lane & 15) * lda + 8 * (lane >> 4));
    const bf16x8 b = *reinterpret_cast<const bf16x8*>(B + (lane & 15) * ldb + 8 * (lane >> 4));
    acc = Fmt16<T>::mma16(a, b, acc);
  }
};
template <> struct KC<bf16_t> : KC16<bf16_t> {};
template <> struct KC<f16_t> : KC16<f16_t> {};
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
//               (* GELU'(S[pixel][co]) when OUT_GGRAD), Xt = GELU?(map(X));
// DUAL: Y2 = GELU(Y) as well (the following conv then loads it without converting).
// Block = NWAVES waves = TH x 16 output pixels x all Cout; wave w owns MT image rows.
template <typename T, int NT, int TH, int MT, bool DB, bool IN_D2S, bool IN_GELU, bool OUT_D2S,
          bool OUT_GGRAD, bool BIAS, bool DUAL>
__global__ void __launch_bounds__(64 * (TH / MT)) conv3x3_kernel(const T* __restrict__ X,
                                                                 const T* __restrict__ Wt,
                                                                 const float* __restrict__ bias,
                                                                 const T* __restrict__ S,
                                                                 T* __restrict__ Y, T* __restrict__ Y2,
                                                                 ConvGeom g) {
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
        // DUAL: also GELU of the stored (rounded) value -- the next conv's input
        if constexpr (DUAL) Y2[base + co] = from_f32<T>(gelu_f(to_f32(from_f32<T>(v))));
      }
    }
  }
}

// ------------------------------------------------------------------ 16-bit fwd / dgrad, v2
// Persistent implicit GEMM on v_mfma_f32_32x32x16_{bf16,f16} (raw 16-bit storage; T = format) (Cout = 32*NCT, CinP = 16*KS).  One
// workgroup of NW waves per CU loops over output tiles of NW*MT rows x 32 pixels x all
// Cout; wave w owns MT image rows.  D[co][pixel] = W_tap[co][ci] * X[ci][pixel]: the weight
// fragment is the A operand, so each lane ends with 4 consecutive output channels of one
// pixel (8-B stores).  Everything is register staged:
//   * weights: a ring of three register sets; W(tap+1) is written to the other LDS buffer
//     while tap runs (WDB: one barrier per tap; else between two barriers after the tap),
//     its global load issued three taps earlier;
//   * halo of the next tile: loaded after tap 0, GELU-converted in registers a third per
//     tap (waves of the lower half at taps 2-4, the upper half at 5-7: on each SIMD one wave
//     converts while its partner issues MFMAs), stored to LDS after tap 8;
//   * dgrad: the pre-activation S of the tile's outputs is prefetched at tap 5 for the
//     GELU' epilogue.
// Index math of the halo chunks goes through opaque() so it is recomputed per tile instead
// of pinning registers for the whole persistent loop.
template <typename T> MSU_DEV void unpack8(const u32x4& q, float (&v)[8]) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    v[2 * i] = Fmt16<T>::lo(q[i]);
    v[2 * i + 1] = Fmt16<T>::hi(q[i]);
  }
}
template <typename T> MSU_DEV u32x4 gelu8(const u32x4& q) {
  float v[8];
  unpack8<T>(q, v);
  return u32x4{pack2<T>(gelu_fast(v[0]), gelu_fast(v[1])), pack2<T>(gelu_fast(v[2]), gelu_fast(v[3])),
               pack2<T>(gelu_fast(v[4]), gelu_fast(v[5])), pack2<T>(gelu_fast(v[6]), gelu_fast(v[7]))};
}

template <int I> using IC = std::integral_constant<int, I>;
template <typename F, int... Is>
MSU_DEV void static_for(F&& f, std::integer_sequence<int, Is...>) {
  (f(IC<Is>{}), ...);
}

template <typename T, int NCT, int KS, int NW, int MT, bool WDB, bool IN_D2S, bool IN_GELU, bool OUT_D2S,
          bool OUT_GGRAD, bool BIAS, bool DUAL>
__global__ void __launch_bounds__(64 * NW) conv3x3_v2_kernel(const bf16_t* __restrict__ X,
                                                         const bf16_t* __restrict__ Wt,
                                                         const float* __restrict__ bias,
                                                         const bf16_t* __restrict__ S,
                                                         bf16_t* __restrict__ Y, bf16_t* __restrict__ Y2,
                                                         ConvGeom g, int ntiles) {
  constexpr int TH = NW * MT, TWV = 32;
  constexpr int CinP = KS * 16, Cout = NCT * 32;
  constexpr int PS = CinP + 8;           // LDS pixel / weight-row stride: conflict-free b128 reads
  constexpr int CPP = CinP / 8;          // 16-B chunks per pixel
  constexpr int HWD = TWV + 2;           // halo width
  constexpr int HPIX = (TH + 2) * HWD;
  constexpr int HCH = HPIX * CPP;
  constexpr int NTHR = 64 * NW;
  constexpr int NHC = (HCH + NTHR - 1) / NTHR;
  constexpr int WCH = Cout * CPP;
  constexpr int NWC = (WCH + NTHR - 1) / NTHR;
  constexpr int WIMG = Cout * PS;        // elements of one LDS weight image

  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  bf16_t* sX = reinterpret_cast<bf16_t*>(smem_raw);
  bf16_t* sW = sX + HPIX * PS;           // [WDB ? 2 : 1][Cout][PS]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int tiles_x = (g.W + TWV - 1) / TWV, tiles_y = (g.H + TH - 1) / TH;
  const int per_img = tiles_x * tiles_y;

  u32x4 hr[NHC];
  u32x4 w0[NWC], w1[NWC], w2[NWC];       // weight register ring (sets picked at compile time)
  u32x4 sp[OUT_GGRAD ? MT : 1][OUT_GGRAD ? NCT : 1][2];

  auto coords = [&](int tile, int& b, int& y0, int& x0) {
    b = tile / per_img;
    const int r = tile - b * per_img;
    y0 = (r / tiles_x) * TH;
    x0 = (r - (r / tiles_x) * tiles_x) * TWV;
  };
  // branch-free halo load: out-of-image / padding chunks load a clamped in-image address and
  // are zeroed by a select
  auto load_halo = [&](int tile) {
    int b, y0, x0;
    coords(tile, b, y0, x0);
    const int t = opaque(tid);
#pragma unroll
    for (int c = 0; c < NHC; ++c) {
      const int i = t + NTHR * c;
      const int pix = i / CPP, ch = i - (i / CPP) * CPP;
      const int row = pix / HWD, col = pix - (pix / HWD) * HWD;
      const int y = y0 - 1 + row, x = x0 - 1 + col;
      const bool ok = i < HCH && y >= 0 && y < g.H && x >= 0 && x < g.W && ch * 8 < g.Cin;
      const int yc = min(max(y, 0), g.H - 1), xc = min(max(x, 0), g.W - 1);
      const int chc = ch * 8 < g.Cin ? ch : 0;
      const u32x4 v = *reinterpret_cast<const u32x4*>(X + pix_off32<IN_D2S>(b, yc, xc, g.H, g.W, g.Cin) + chc * 8);
      hr[c] = ok ? v : u32x4{0u, 0u, 0u, 0u};
    }
  };
  auto store_halo = [&]() {
    const int t = opaque(tid);
#pragma unroll
    for (int c = 0; c < NHC; ++c) {
      const int i = t + NTHR * c;
      if (HCH % NTHR == 0 || c + 1 < NHC || i < HCH) {
        const int pix = i / CPP, ch = i - (i / CPP) * CPP;
        *reinterpret_cast<u32x4*>(sX + pix * PS + ch * 8) = hr[c];
      }
    }
  };
  auto load_w = [&](int tap, u32x4 (&dst)[NWC]) {
    const bf16_t* src = Wt + (long)tap * Cout * CinP;
#pragma unroll
    for (int c = 0; c < NWC; ++c) {
      const int i = min(tid + NTHR * c, WCH - 1);
      dst[c] = *reinterpret_cast<const u32x4*>(src + (long)i * 8);
    }
  };
  auto store_w = [&](const u32x4 (&srcr)[NWC], bf16_t* dst) {
#pragma unroll
    for (int c = 0; c < NWC; ++c) {
      const int i = tid + NTHR * c;
      if (WCH % NTHR == 0 || c + 1 < NWC || i < WCH) {
        const int co = i / CPP, ch = i - (i / CPP) * CPP;
        *reinterpret_cast<u32x4*>(dst + co * PS + ch * 8) = srcr[c];
      }
    }
  };
  // ring step: write set K to LDS, refill it with W(tap); sets are named, never selected
  // through a reference, so they stay in registers
  auto ring = [&](auto K, bf16_t* dst, int tap) {
    if constexpr (decltype(K)::value == 0) { store_w(w0, dst); load_w(tap, w0); }
    else if constexpr (decltype(K)::value == 1) { store_w(w1, dst); load_w(tap, w1); }
    else { store_w(w2, dst); load_w(tap, w2); }
  };
  auto out_off = [&](int b, int y, int x, int co) -> int { return pix_off32<OUT_D2S>(b, y, x, g.H, g.W, Cout) + co; };

  int tile = blockIdx.x;
  if (tile >= ntiles) return;
  // prologue: halo of the first tile, W(0) in LDS buffer 0, W(1..3) in flight in sets 1, 2, 0
  load_halo(tile);
  if constexpr (IN_GELU && !(MSU_EXP & 2)) {
#pragma unroll
    for (int c = 0; c < NHC; ++c) hr[c] = gelu8<T>(hr[c]);
  }
  store_halo();
  load_w(0, w0);
  store_w(w0, sW);
  load_w(1, w1);
  load_w(2, w2);
  load_w(3, w0);
  __syncthreads();

  const int xl = lane & 31, kh = 8 * (lane >> 5);
  int wbuf = 0;
  for (; tile < ntiles; tile += gridDim.x) {
    const int next = tile + gridDim.x;
    int b, y0, x0;
    coords(tile, b, y0, x0);
    const int xo = x0 + xl;
    f32x16 acc[MT][NCT];
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int n = 0; n < NCT; ++n)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[m][n][r] = 0.f;

    static_for([&](auto TAP) {
      constexpr int tap = decltype(TAP)::value;
      constexpr int dy = tap / 3, dx = tap % 3;
      const bf16_t* wcur = sW + (WDB ? wbuf * WIMG : 0);
      if constexpr (WDB) {
        // W(tap+1) into the other buffer (read during tap-1, released by its barrier)
        if constexpr (!(MSU_EXP & 8)) ring(IC<(tap + 1) % 3>{}, sW + (wbuf ^ 1) * WIMG, (tap + 4) % 9);
      }
      if constexpr (tap == 0 && !(MSU_EXP & 4)) {
        if (next < ntiles) load_halo(next);
      }
      if constexpr (IN_GELU && tap >= 2 && tap <= 7 && !(MSU_EXP & 2)) {
        // GELU of the prefetched halo, a third per tap: waves 0..NW/2-1 at taps 2-4, the
        // others at taps 5-7, so on every SIMD one wave converts while its partner runs MFMAs
        constexpr int part = (tap - 2) % 3;
        constexpr int c0 = part * ((NHC + 2) / 3);
        constexpr int c1 = (c0 + (NHC + 2) / 3) < NHC ? (c0 + (NHC + 2) / 3) : NHC;
        if ((wave < NW / 2) == (tap <= 4)) {
#pragma unroll
          for (int c = c0; c < c1; ++c) hr[c] = gelu8<T>(hr[c]);
        }
      }
      if constexpr (OUT_GGRAD && tap == 5) {
        if (xo < g.W) {
#pragma unroll
          for (int m = 0; m < MT; ++m) {
            const int y = min(y0 + wave * MT + m, g.H - 1);
#pragma unroll
            for (int n = 0; n < NCT; ++n)
#pragma unroll
              for (int pp = 0; pp < 2; ++pp)
                sp[m][n][pp] = *reinterpret_cast<const u32x4*>(S + out_off(b, y, xo, 32 * n + 16 * pp + 8 * (lane >> 5)));
          }
        }
      }
      // fragments double buffered in registers: the reads of k-step ks+1 are issued before
      // the MFMAs of ks; a scheduling fence per k-step keeps the compiler from hoisting more
      const bf16_t* xb = sX + ((wave * MT + dy) * HWD + dx + xl) * PS + kh;
      const bf16_t* wb = wcur + xl * PS + kh;
      bf16x8 xa[2][MT], wf[2][NCT];
      auto read_frags = [&](int ks, int set) {
#pragma unroll
        for (int m = 0; m < MT; ++m) xa[set][m] = *reinterpret_cast<const bf16x8*>(xb + m * HWD * PS + ks * 16);
#pragma unroll
        for (int n = 0; n < NCT; ++n) wf[set][n] = *reinterpret_cast<const bf16x8*>(wb + n * 32 * PS + ks * 16);
      };
      read_frags(0, 0);
      static_for([&](auto KSI) {
        constexpr int ks = decltype(KSI)::value;
        constexpr int cur = ks & 1;
        if constexpr (ks + 1 < KS) read_frags(ks + 1, cur ^ 1);
#pragma unroll
        for (int m = 0; m < MT; ++m)
#pragma unroll
          for (int n = 0; n < NCT; ++n)
          {
            if constexpr (MSU_EXP & 32)
              acc[m][n][0] += (float)wf[cur][n][0] * (float)xa[cur][m][1];
            else
              acc[m][n] = Fmt16<T>::mma32(wf[cur][n], xa[cur][m], acc[m][n]);
          }
        __builtin_amdgcn_sched_barrier(0);
      }, std::make_integer_sequence<int, KS>{});
      if constexpr (!(MSU_EXP & 16) || tap == 8) __syncthreads();
      if constexpr (!WDB) {
        ring(IC<(tap + 1) % 3>{}, sW, (tap + 4) % 9);
      }
      if constexpr (tap == 8) {
        if (next < ntiles) store_halo();
      }
      if constexpr (!WDB || tap == 8) __syncthreads();
      if constexpr (WDB) wbuf ^= 1;
    }, std::make_integer_sequence<int, 9>{});

    // epilogue: lane holds pixel xo, channels 32n + 8q + 4(lane>>5) + e (q = 0..3) of its rows;
    // v_permlane32_swap of groups q = 2pp and 2pp+1 gives lane l < 32 channels 32n + 16pp + 0..7
    // and lane l + 32 channels 32n + 16pp + 8..15 of the same pixel: one 16-B store each
    if (xo < g.W) {
#pragma unroll
      for (int n = 0; n < NCT; ++n)
#pragma unroll
        for (int pp = 0; pp < 2; ++pp) {
          const int co = 32 * n + 16 * pp + 8 * (lane >> 5);
          float bv[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
          if constexpr (BIAS) {
            const float4 t0 = *reinterpret_cast<const float4*>(bias + co);
            const float4 t1 = *reinterpret_cast<const float4*>(bias + co + 4);
            bv[0] = t0.x; bv[1] = t0.y; bv[2] = t0.z; bv[3] = t0.w;
            bv[4] = t1.x; bv[5] = t1.y; bv[6] = t1.z; bv[7] = t1.w;
          }
#pragma unroll
          for (int m = 0; m < MT; ++m) {
            const int y = y0 + wave * MT + m;
            float v[8];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(acc[m][n][8 * pp + i]),
                                                              __float_as_uint(acc[m][n][8 * pp + 4 + i]), false, false);
              v[i] = __uint_as_float(r[0]) + bv[i];
              v[4 + i] = __uint_as_float(r[1]) + bv[4 + i];
            }
            if (y >= g.H) continue;
            if constexpr (OUT_GGRAD) {
              const u32x4 t = sp[m][n][pp];
#pragma unroll
              for (int i = 0; i < 4; ++i) {
                v[2 * i] *= gelu_grad_fast(Fmt16<T>::lo(t[i]));
                v[2 * i + 1] *= gelu_grad_fast(Fmt16<T>::hi(t[i]));
              }
            }
            const u32x4 pk = {pack2<T>(v[0], v[1]), pack2<T>(v[2], v[3]), pack2<T>(v[4], v[5]), pack2<T>(v[6], v[7])};
            if (!(MSU_EXP & 1) || v[0] == 1.2345e-30f) *reinterpret_cast<u32x4*>(Y + out_off(b, y, xo, co)) = pk;
            if constexpr (DUAL) *reinterpret_cast<u32x4*>(Y2 + out_off(b, y, xo, co)) = gelu8<T>(pk);
          }
        }
    }
  }
}

// ------------------------------------------------------------------ 16-bit fwd, v3 (C = 96)
// The v2 kernel (8 waves x one output row) spends as many LDS cycles as MFMA cycles: per tap
// and wave 24 ds_read_b128 for 18 MFMAs, plus 24 KB of register-staged weight writes per tap.
// v3 halves both per output pixel:
//   * a tile is 16 rows x 32 pixels x 96 channels; wave w owns rows 2w, 2w + 1, so each weight
//     fragment feeds two MFMAs (reads per MFMA 5/6 instead of 4/3);
//   * the halo [18][34][96] and the weight image of a tap [96][96] are stored UNPADDED with
//     the 16-B chunk c of row / pixel p at c ^ ((p >> 2) & 3): a half-wave's fragment read
//     (32 consecutive rows, one chunk) covers all 64 banks, and the 154 KB of LDS fit;
//   * the weights of tap t + 1 arrive by LDS-DMA (global_load_lds_dwordx4, source addresses
//     permuted by the same swizzle) into the other of two weight images while tap t runs --
//     no registers and no ds_write for the weight ring, one barrier per tap;
//   * the next tile's halo is loaded into registers at tap 1 and written to LDS after tap 8.
// Epilogue as v2 (bias, DUAL = GELU(Y) as a second output, GELU'(S) for the backward-data
// launches with S prefetched at tap 7, 16-B stores after a permlane32 swap).
constexpr int V3_HALO_TAP = 1;
constexpr int SPRE = 12;  // GELU' operand loads per lane (dgrad)
// ablation bit 1024: all of them at tap 7 (the round-5 placement; spilled halo registers)
constexpr bool SP_AT7 = (MSU_EXP & 1024) != 0;

MSU_DEV int swz(int p) { return (p >> 2) & 3; }
// M16 (16x16x32 MFMA) fragment reads: 16 consecutive rows, chunk (lane >> 4) of a 4-chunk group;
// the ds_read_b128 lane groups ({0-3, 12-15, 20-27}, ...) mix two chunks of 8 + 8 rows, which
// (p >> 1) & 3 spreads over all 16 bank slots for ANY first row (checked exhaustively offline)
template <bool M16> MSU_DEV int swzv(int p) { return M16 ? (p >> 1) & 3 : (p >> 2) & 3; }

// SPREAD: the next tile's halo loads are issued in seven parts at taps 1..7 (each part issued
// after that tap's weight DMA, so it only has to land two taps later) instead of all at tap 1,
// where the wait for tap 3's weights also waited for the whole 117 KB halo.
MSU_DEV constexpr int halo_part_lo(int t, int nhc) { return (t - 1) * nhc / 7; }  // t = 1..7

// Tile queue (tq, common.h): a workgroup takes its first tile statically (blockIdx.x) and claims
// every further one from counter 0, one tile ahead (the next tile's halo and weight prefetch
// need its index from tap 1 on).  Results do not depend on which workgroup computes a tile.
template <typename T, bool IN_D2S, bool OUT_D2S, bool OUT_GGRAD, bool BIAS, bool DUAL, bool SPREAD, bool M16>
__global__ void __launch_bounds__(512) conv3x3_v3_kernel(const bf16_t* __restrict__ X,
                                                         const bf16_t* __restrict__ Wt,
                                                         const float* __restrict__ bias,
                                                         const bf16_t* __restrict__ S,
                                                         bf16_t* __restrict__ Y, bf16_t* __restrict__ Y2,
                                                         ConvGeom g, int ntiles, int* __restrict__ tq) {
  constexpr int C = 96, CH = 12, NW = 8, MT = 2, TH = NW * MT, TWV = 32, HWD = TWV + 2;
  constexpr int HPIX = (TH + 2) * HWD;  // 612 halo pixels
  (void)HPIX;
  constexpr int NTHR = 64 * NW;
  constexpr int PSTEP = NTHR / CH;                // halo pixels per staging round (one channel
                                                  // chunk per thread: thread t stages chunk t % 12)
  constexpr int NHC = (HPIX + PSTEP - 1) / PSTEP;  // staging rounds
  constexpr int WIMG = C * C;                   // elements of one tap's weight image
  constexpr int WINS = WIMG * 2 / 1024;         // 18 DMA wave-instructions per tap
  constexpr int WPER = (WINS + NW - 1) / NW;    // <= 3 per wave
  static_assert(WINS * 1024 == WIMG * 2, "weight image in whole DMA instructions");

  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  bf16_t* sX = reinterpret_cast<bf16_t*>(smem_raw);
  bf16_t* sW = sX + HPIX * C;  // [2][96][96]
  float* sB = reinterpret_cast<float*>(sW + 2 * WIMG);  // [96] bias (BIAS)
  int* sQ = reinterpret_cast<int*>(sB + C);              // the claimed next tile (tq)
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int tiles_x = (g.W + TWV - 1) / TWV, tiles_y = (g.H + TH - 1) / TH;
  // output stores of a whole tile, per wave (16-B stores; DUAL: two per output chunk)
  constexpr int EST = MT * 6 * (DUAL ? 2 : 1);
  const int per_img = tiles_x * tiles_y;

  auto coords = [&](int tile, int& b, int& y0, int& x0) {
    b = tile / per_img;
    const int r = tile - b * per_img;
    y0 = (r / tiles_x) * TH;
    x0 = (r - (r / tiles_x) * tiles_x) * TWV;
  };
  u32x4 hr[NHC];
  // Halo staging: thread t < 12 * PSTEP owns channel chunk t % 12 of pixels t / 12 + PSTEP * c
  // (c = 0 .. NHC-1); the pixel's (row, col) advance incrementally, so a chunk costs a few adds
  // and one address multiply instead of the divisions of a flat chunk index
  // rounds [c0, c1) of this thread's share of tile `tile`'s halo -> registers
  auto load_halo = [&](int tile, auto C0, auto C1) {
    constexpr int c0 = decltype(C0)::value, c1 = decltype(C1)::value;
    int b, y0, x0;
    coords(tile, b, y0, x0);
    const int t = opaque(tid);  // recomputed per call: nothing pinned across the tile loop
    const bool hact = t < PSTEP * CH;
    int p = t / CH + PSTEP * c0;
    int row = p / HWD, col = p - (p / HWD) * HWD;
    const bf16_t* xc = X + (t % CH) * 8;
#pragma unroll
    for (int c = c0; c < c1; ++c) {
      const int y = y0 - 1 + row, x = x0 - 1 + col;
      const bool ok = !(MSU_EXP & 256) && hact && p < HPIX && (unsigned)y < (unsigned)g.H && (unsigned)x < (unsigned)g.W;
      // out-of-image chunks read the zero region: no select on the loaded value, so the load
      // stays in flight until the halo is stored (address select, no branch)
      const bf16_t* src = ok ? xc + pix_off32<IN_D2S>(b, y, x, g.H, g.W, C)
                             : reinterpret_cast<const bf16_t*>(zero_src(tid));
      hr[c] = *reinterpret_cast<const u32x4*>(src);
      p += PSTEP;
      col += PSTEP % HWD;
      row += PSTEP / HWD;
      if (col >= HWD) {
        col -= HWD;
        ++row;
      }
    }
  };
  auto store_halo = [&]() {
    const int t = opaque(tid);
    const bool hact = t < PSTEP * CH;
    const int hch = t % CH;
    int p = t / CH;
#pragma unroll
    for (int c = 0; c < NHC; ++c) {
      if (hact && p < HPIX) *reinterpret_cast<u32x4*>(sX + p * C + ((hch ^ swzv<M16>(p)) << 3)) = hr[c];
      p += PSTEP;
    }
  };
  // this wave's share of the DMA of tap `tap`'s weight image into buffer `buf`
  // this wave's share of the DMA of tap `tap`'s weight image into buffer `buf`
  auto dma_w = [&](int tap, int buf) {
    const bf16_t* src = Wt + (long)tap * WIMG;
    bf16_t* dst = sW + buf * WIMG;
    // piece r of this wave is slot q = 64 (wave + NW r) + lane: row q / 12, chunk q % 12,
    // advanced incrementally from r = 0 (one division per call)
    const int q0 = 64 * wave + opaque(lane);
    int row = q0 / CH, pos = q0 - (q0 / CH) * CH;
#pragma unroll
    for (int r = 0; r < WPER; ++r) {
      const int k = wave + NW * r;
      if (WINS % NW == 0 || k < WINS) glds16((MSU_EXP & 512) ? src + lane * 8 : src + row * C + ((pos ^ swzv<M16>(row)) << 3), dst + 512 * k);
      pos += (64 * NW) % CH;
      row += (64 * NW) / CH;
      if (pos >= CH) {
        pos -= CH;
        ++row;
      }
    }
  };
  // DMA wave-instructions this wave issues per tap (wave-uniform)
  const int my_wdma = (WINS - wave + NW - 1) / NW;

  // tq: claims count up from 0 (tile gridDim.x + count)
  auto finish = [&]() { tq_finish(tq); };
  // the tile thread 0 left in sQ (after a barrier); untracked read: a compiler-visible ds_read
  // would wait for the weight DMA and output stores in flight here (vmcnt(0))
  auto read_q = [&]() -> int {
    uint32_t v = ds_b32_untracked<0>(lds_u32(sQ));
    lds_wait_tie<0>(v);
    return __builtin_amdgcn_readfirstlane((int)v) + (int)gridDim.x;
  };
  int tile = blockIdx.x;
  if (tile >= ntiles) {  // (the launch keeps the grid <= ntiles)
    finish();
    return;
  }
  if (tq != nullptr && tid == 0) sQ[0] = tq_claim(tq, 0);
  if constexpr (BIAS) {
    if (tid < C) sB[tid] = bias[tid];  // read by every epilogue from LDS (no global load there)
  }
  load_halo(tile, IC<0>{}, IC<NHC>{});
  store_halo();
  dma_w(0, 0);
  __syncthreads();  // the halo's ds_writes land before any wave reads (the tap barriers are raw)
  int next = tq != nullptr ? read_q() : tile + (int)gridDim.x;
  int wbuf = 0;
  // w1_early: this tile's W(1) was DMA'd by the previous tile's epilogue, ahead of its output
  // stores; st_full: those stores are all EST of them (a whole tile) and may stay in flight
  // through tap 0 (waits at taps 0 / 1 count them) instead of draining before tap 0
  bool w1_early = false, st_full = false;

  const int xl = lane & 31, h = lane >> 5;
  // lane chunk offsets (elements) of k steps with ks even / odd, for row / pixel swizzle sw:
  // chunk 2ks + h -> 4 (ks >> 1) + ((2 (ks & 1) + h) ^ sw)
  auto koff = [&](int sw, int odd) { return ((2 * odd + h) ^ sw) << 3; };
  const int wsw = swz(xl);  // weight rows 32n + xl
  const int wk0 = xl * C + koff(wsw, 0), wk1 = xl * C + koff(wsw, 1);
  // M16: lane l reads row (l & 15) of a 16-row fragment, chunk 4 ks + (l >> 4)
  const int l15 = lane & 15, g4 = lane >> 4;
  const int wk16 = l15 * C + ((g4 ^ swzv<true>(l15)) << 3);  // weight rows 16n + l15

  for (;;) {
    int nn = 0;  // thread 0 (tq): the tile after next, claimed at tap 1
    int b, y0, x0;
    coords(tile, b, y0, x0);
    const int xo = x0 + xl;
    // accumulators: 32x32 tiles [row m][co tile n] (!M16) or 16x16 tiles [row m][pixel tile
    // pt][co tile n] (M16); the other form is a 1-element placeholder
    f32x16 acc[M16 ? 1 : MT][M16 ? 1 : 3];
    f32x4 acc4[M16 ? MT : 1][M16 ? 2 : 1][M16 ? 6 : 1];
    if constexpr (M16) {
#pragma unroll
      for (int m = 0; m < MT; ++m)
#pragma unroll
        for (int pt = 0; pt < 2; ++pt)
#pragma unroll
          for (int n = 0; n < 6; ++n) acc4[m][pt][n] = f32x4{0.f, 0.f, 0.f, 0.f};
    } else {
#pragma unroll
      for (int m = 0; m < MT; ++m)
#pragma unroll
        for (int n = 0; n < 3; ++n) acc[m][n] = f32x16{0};
    }
    // dgrad GELU' operands: 12 16-B pieces per lane in both forms
    u32x4 sp[OUT_GGRAD ? MT : 1][OUT_GGRAD ? (M16 ? 2 : 3) : 1][OUT_GGRAD ? (M16 ? 3 : 2) : 1];

    static_for([&](auto TAP) {
      constexpr int tap = decltype(TAP)::value;
      constexpr int dy = tap / 3, dx = tap % 3;
      // W(tap) landed (this wave's DMAs; the halo loads issued after them may stay in flight),
      // then the barrier: every wave's DMA landed, every wave done with the other buffer
      // loads issued at tap - 1 after that tap's weight DMA may stay in flight: the halo
      // part(s) of the next tile and (dgrad, tap 7) the GELU' operands
      constexpr int hprev = SPREAD ? (tap >= 2 ? halo_part_lo(tap, NHC) - halo_part_lo(tap - 1, NHC) : 0)
                                   : (tap == V3_HALO_TAP + 1 ? NHC : 0);
      // (only a third of them are issued at tap 7, see load_sp / load_sp16)
      constexpr int sprev = (OUT_GGRAD && tap == 8) ? (SP_AT7 ? SPRE : SPRE / 3) : 0;
      if constexpr (tap == 0) {
        // W(0) landed (DMA'd at the previous tile's tap 8); W(1) and the previous tile's output
        // stores, issued after it in that epilogue, may stay in flight
        if (!w1_early) wait_vmcnt<0>();
        else if (st_full) {
          if (my_wdma == WPER) wait_vmcnt<WPER + EST>();
          else wait_vmcnt<WPER - 1 + EST>();
        } else {
          if (my_wdma == WPER) wait_vmcnt<WPER>();
          else wait_vmcnt<WPER - 1>();
        }
      } else if constexpr (tap == 1) {
        static_assert(hprev == 0 && sprev == 0, "tap 1 waits");
        if (w1_early && st_full) wait_vmcnt<EST>();  // W(1) is older than the stores
        else wait_vmcnt<0>();
      } else if constexpr (hprev > 0) {
        if (next < ntiles) wait_vmcnt<hprev + sprev>();
        else wait_vmcnt<sprev>();
      } else {
        wait_vmcnt<sprev>();
      }
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      const bf16_t* wcur = sW + wbuf * WIMG;
      if constexpr (tap == 0) {
        if (!w1_early) dma_w(1, wbuf ^ 1);
      } else if constexpr (tap == 1) {
        // claim the tile after next (thread 0); older than W(2)'s DMA, so tap 2's counted wait
        // covers it
        // (the raw count; offset by gridDim.x on read)
        if (tq != nullptr && tid == 0 && next < ntiles) nn = tq_claim(tq, 0);
        dma_w(2, wbuf ^ 1);
      } else if constexpr (tap == 2) {
        // the claim to sQ: every wave read this tile's entry before tap 0's barrier, the next
        // read follows the tile's closing barrier.  Untracked write (a visible ds_write would
        // wait for the weight DMA in flight).
        if (tq != nullptr && tid == 0 && next < ntiles) {
          asm volatile("ds_write_b32 %0, %1" ::"v"(lds_u32(sQ)), "v"(nn) : "memory");
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        }
        dma_w(3, wbuf ^ 1);
      } else if constexpr (tap < 8) {
        dma_w(tap + 1, wbuf ^ 1);
      } else {
        if (next < ntiles) dma_w(0, wbuf ^ 1);
      }
      if constexpr (SPREAD && tap >= 1 && tap <= 7) {
        if (next < ntiles) load_halo(next, IC<halo_part_lo(tap, NHC)>{}, IC<halo_part_lo(tap + 1, NHC)>{});
      } else if constexpr (!SPREAD && tap == V3_HALO_TAP) {
        if (next < ntiles) load_halo(next, IC<0>{}, IC<NHC>{});
      }
      // dgrad, 32 x 32 form: GELU' operands of co tile n for rows m (two 16-B loads per row)
      auto load_sp = [&](int m, int y, int n) __attribute__((always_inline)) {
        const int xs = min(xo, g.W - 1);
#pragma unroll
        for (int pp = 0; pp < 2; ++pp)
          sp[m][n][pp] = *reinterpret_cast<const u32x4*>(S + pix_off32<OUT_D2S>(b, y, xs, g.H, g.W, C) + 32 * n +
                                                         16 * pp + 8 * h);
      };
      // dgrad, 16 x 16 form: the operands of channel group q (32 q .. 32 q + 31) of rows m
      auto load_sp16 = [&](int m, int y, int q) __attribute__((always_inline)) {
#pragma unroll
        for (int pt = 0; pt < 2; ++pt) {
          const int xs = min(x0 + 16 * pt + l15, g.W - 1);
          sp[m][pt][q] = *reinterpret_cast<const u32x4*>(S + pix_off32<OUT_D2S>(b, y, xs, g.H, g.W, C) + 32 * q +
                                                         16 * (g4 & 1) + 8 * (g4 >> 1));
        }
      };
      if constexpr (OUT_GGRAD && tap == 7) {
        // dgrad: the pre-activation S of this tile's outputs for the GELU' epilogue
#pragma unroll
        for (int m = 0; m < MT; ++m) {
          const int y = min(y0 + 2 * wave + m, g.H - 1);
          if constexpr (M16) {
            load_sp16(m, y, 0);
            if constexpr (SP_AT7) {
              load_sp16(m, y, 1);
              load_sp16(m, y, 2);
            }
          } else {
            load_sp(m, y, 0);
            if constexpr (SP_AT7) {
              load_sp(m, y, 1);
              load_sp(m, y, 2);
            }
          }
        }
      }
      if constexpr (M16) {
        // fragment lane offsets of this tap: X rows 2w + m + dy, pixels dx + 16 pt + l15
        int xq[MT][2];
#pragma unroll
        for (int m = 0; m < MT; ++m)
#pragma unroll
          for (int pt = 0; pt < 2; ++pt) {
            const int p = opaque((2 * wave + m + dy) * HWD + dx + 16 * pt) + l15;
            xq[m][pt] = p * C + ((g4 ^ swzv<true>(p)) << 3);
          }
        // groups (ks, m) in sequence: a group's two X fragments (pixel tiles) feed 12 MFMAs, the
        // next group's are read at its start; weight fragments in a ring of two, one co tile
        // ahead (re-read per row m: 16 reads per 24 MFMAs, within the LDS budget of 16x16x32
        // gaps; double-buffering all four X fragments of a k step spilled)
        bf16x8 xb[2][2], wf[2];
        auto read_x = [&](auto GI, int set) __attribute__((always_inline)) {
          constexpr int gi = decltype(GI)::value, ks = gi / MT, m = gi % MT;
#pragma unroll
          for (int pt = 0; pt < 2; ++pt) xb[set][pt] = *reinterpret_cast<const bf16x8*>(sX + xq[m][pt] + 32 * ks);
        };
        auto read_w = [&](auto GI, int n) __attribute__((always_inline)) -> bf16x8 {
          constexpr int ks = decltype(GI)::value / MT;
          return *reinterpret_cast<const bf16x8*>(wcur + 16 * n * C + wk16 + 32 * ks);
        };
        read_x(IC<0>{}, 0);
        wf[0] = read_w(IC<0>{}, 0);
        static_for([&](auto GI) {
          constexpr int gi = decltype(GI)::value, m = gi % MT;
          constexpr int cur = gi & 1;
          if constexpr (gi + 1 < 3 * MT) read_x(IC<gi + 1>{}, cur ^ 1);
          static_for([&](auto NI) {
            constexpr int n = decltype(NI)::value;
            constexpr int j = 6 * gi + n;  // weight fragment sequence number: register set j & 1
            if constexpr (n < 5) wf[(j + 1) & 1] = read_w(IC<gi>{}, n + 1);
            else if constexpr (gi + 1 < 3 * MT) wf[(j + 1) & 1] = read_w(IC<gi + 1>{}, 0);
#pragma unroll
            for (int pt = 0; pt < 2; ++pt) {
              if constexpr (MSU_EXP & 128) asm volatile("" ::"v"(wf[j & 1]), "v"(xb[cur][pt]));  // ablation: no MFMA
              else acc4[m][pt][n] = Fmt16<T>::mma16(wf[j & 1], xb[cur][pt], acc4[m][pt][n]);
            }
          }, std::make_integer_sequence<int, 6>{});
          __builtin_amdgcn_sched_barrier(0);
        }, std::make_integer_sequence<int, 3 * MT>{});
      } else {
        // fragment lane offsets of this tap: X rows 2w + m + dy, pixels dx + xl
        // (recomputed per tap through opaque(): hoisted, the nine taps' offsets would pin 36 VGPRs)
        int xo0[MT], xo1[MT];
#pragma unroll
        for (int m = 0; m < MT; ++m) {
          const int p = opaque((2 * wave + m + dy) * HWD + dx) + xl;
          xo0[m] = p * C + koff(swz(p), 0);
          xo1[m] = p * C + koff(swz(p), 1);
        }
        // X fragments double buffered (k step ks + 1 read before the MFMAs of ks); each weight
        // fragment is read one co tile ahead of its two MFMAs (registers: the halo prefetch
        // holds 60 VGPRs across the taps)
        bf16x8 xa[2][MT], wf[2];
        auto read_x = [&](auto KSI, int set) __attribute__((always_inline)) {
          constexpr int ks = decltype(KSI)::value;
          constexpr int kb = 32 * (ks >> 1);  // elements: 4 chunks per even / odd pair
#pragma unroll
          for (int m = 0; m < MT; ++m)
            xa[set][m] = *reinterpret_cast<const bf16x8*>(sX + ((ks & 1) ? xo1[m] : xo0[m]) + kb);
        };
        auto read_w = [&](auto KSI, int n) __attribute__((always_inline)) -> bf16x8 {
          constexpr int ks = decltype(KSI)::value;
          constexpr int kb = 32 * (ks >> 1);
          return *reinterpret_cast<const bf16x8*>(wcur + 32 * n * C + ((ks & 1) ? wk1 : wk0) + kb);
        };
        read_x(IC<0>{}, 0);
        wf[0] = read_w(IC<0>{}, 0);
        static_for([&](auto KSI) {
          constexpr int ks = decltype(KSI)::value;
          constexpr int cur = ks & 1;
          if constexpr (ks + 1 < 6) read_x(IC<ks + 1>{}, cur ^ 1);
          static_for([&](auto NI) {
            constexpr int n = decltype(NI)::value;
            constexpr int j = 3 * ks + n;  // weight fragment sequence number: register set j & 1
            // (reading it two groups ahead in a ring of three measured no faster and spills the dgrad)
            if constexpr (n < 2) wf[(j + 1) & 1] = read_w(IC<ks>{}, n + 1);
            else if constexpr (ks + 1 < 6) wf[(j + 1) & 1] = read_w(IC<ks + 1>{}, 0);
#pragma unroll
            for (int m = 0; m < MT; ++m) {
              if constexpr (MSU_EXP & 128) asm volatile("" ::"v"(wf[j & 1]), "v"(xa[cur][m]));  // ablation: no MFMA
              else acc[m][n] = Fmt16<T>::mma32(wf[j & 1], xa[cur][m], acc[m][n]);
            }
          }, std::make_integer_sequence<int, 3>{});
          __builtin_amdgcn_sched_barrier(0);
        }, std::make_integer_sequence<int, 6>{});
      }
      if constexpr (tap == 8) {
        if constexpr (OUT_GGRAD && !SP_AT7) {
          // co tiles 1-2's GELU' operands after the last MFMAs: held through taps 7-8 beside the
          // full halo prefetch they pushed the kernel past 256 VGPRs (halo registers spilled,
          // each spill store a vmcnt(0) at tap 1); their latency is exposed at the epilogue's
          // wait instead
#pragma unroll
          for (int m = 0; m < MT; ++m) {
            const int y = min(y0 + 2 * wave + m, g.H - 1);
            if constexpr (M16) {
              load_sp16(m, y, 1);
              load_sp16(m, y, 2);
            } else {
              load_sp(m, y, 1);
              load_sp(m, y, 2);
            }
          }
        }
        if (next < ntiles) {
          __syncthreads();  // every wave's last halo read done (s_barrier + lgkmcnt)
          store_halo();
        }
      }
      wbuf ^= 1;
    }, std::make_integer_sequence<int, 9>{});
    // the epilogue's start: the GELU' operands landed; then the next tile's W(1) DMA (into
    // tap 8's weight buffer: every wave passed tap 8's barrier before the halo store) ahead of
    // this tile's output stores, so tap 1 of the next tile waits for it and not for the stores
    auto epi_start = [&]() __attribute__((always_inline)) {
      // the GELU' operands landed; pinned after the wait (an empty asm redefining them), or the
      // compiler still counts them pending and puts a vmcnt(0) in front of each first use --
      // behind the previous store group's stores
      if constexpr (OUT_GGRAD) {
        wait_vmcnt<0>();
#pragma unroll
        for (int m = 0; m < MT; ++m)
#pragma unroll
          for (int n = 0; n < (M16 ? 2 : 3); ++n)
#pragma unroll
            for (int pp = 0; pp < (M16 ? 3 : 2); ++pp) vreg_pin(sp[m][n][pp]);
      }
      w1_early = next < ntiles;
      st_full = w1_early && x0 + TWV <= g.W && y0 + TH <= g.H;
      if (w1_early) dma_w(1, wbuf ^ 1);
    };

    if constexpr (M16) {
      // epilogue: lane holds pixel x0 + 16 pt + l15, channels 16n + 4 g4 + r; a permlane16 swap
      // of co tiles (2q, 2q + 1) gives every lane 8 consecutive channels co8 .. co8 + 7 with
      // co8 = 16 (2q + (g4 & 1)) + 8 (g4 >> 1) (lanes l, l ^ 16 share the pixel)
      const int cofs = 16 * (g4 & 1) + 8 * (g4 >> 1);
      float4 bq[3][2];
      if constexpr (BIAS) {
#pragma unroll
        for (int q = 0; q < 3; ++q) {
          bq[q][0] = *reinterpret_cast<const float4*>(sB + 32 * q + cofs);
          bq[q][1] = *reinterpret_cast<const float4*>(sB + 32 * q + cofs + 4);
        }
      }
      epi_start();
#pragma unroll
      for (int pt = 0; pt < 2; ++pt) {
        const int px = x0 + 16 * pt + l15;
        if (px >= g.W) continue;  // lanes l and l ^ 16 agree
#pragma unroll
        for (int q = 0; q < 3; ++q) {
          float bv[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
          if constexpr (BIAS) {
            const float4 t0 = bq[q][0], t1 = bq[q][1];
            bv[0] = t0.x; bv[1] = t0.y; bv[2] = t0.z; bv[3] = t0.w;
            bv[4] = t1.x; bv[5] = t1.y; bv[6] = t1.z; bv[7] = t1.w;
          }
#pragma unroll
          for (int m = 0; m < MT; ++m) {
            const int y = y0 + 2 * wave + m;
            float v[8];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(acc4[m][pt][2 * q][i]),
                                                              __float_as_uint(acc4[m][pt][2 * q + 1][i]), false, false);
              v[i] = __uint_as_float(r[0]) + bv[i];
              v[4 + i] = __uint_as_float(r[1]) + bv[4 + i];
            }
            if (y >= g.H) continue;
            if constexpr (OUT_GGRAD) {
              const u32x4 t = sp[m][pt][q];
#pragma unroll
              for (int i = 0; i < 4; ++i) {
                v[2 * i] *= gelu_grad_fast(Fmt16<T>::lo(t[i]));
                v[2 * i + 1] *= gelu_grad_fast(Fmt16<T>::hi(t[i]));
              }
            }
            const u32x4 pk = {pack2<T>(v[0], v[1]), pack2<T>(v[2], v[3]), pack2<T>(v[4], v[5]), pack2<T>(v[6], v[7])};
            const int off = pix_off32<OUT_D2S>(b, y, px, g.H, g.W, C) + 32 * q + cofs;
            // ablation: no output stores (results wrong; the never-true test keeps the MFMAs alive)
            if constexpr (MSU_EXP & 64) if (v[0] != 1.2345e-30f) continue;
            *reinterpret_cast<u32x4*>(Y + off) = pk;
            if constexpr (DUAL) *reinterpret_cast<u32x4*>(Y2 + off) = gelu8<T>(pk);
          }
        }
      }
    } else {
    // epilogue: lane holds pixel xo, channels 32n + 8q + 4h + e of rows 2w + m; the
    // permlane32 swap gives lane l < 32 channels 32n + 16pp + 0..7 and l + 32 the next 8
    // bias columns of this lane's 6 store groups, loaded together: one wait, not one per
    // store group behind the previous group's stores
    float4 bq[3][2][2];
    if constexpr (BIAS) {
#pragma unroll
      for (int n = 0; n < 3; ++n)
#pragma unroll
        for (int pp = 0; pp < 2; ++pp) {
          const int co = 32 * n + 16 * pp + 8 * h;
          bq[n][pp][0] = *reinterpret_cast<const float4*>(sB + co);
          bq[n][pp][1] = *reinterpret_cast<const float4*>(sB + co + 4);
        }
    }
    epi_start();
    if (xo < g.W) {
#pragma unroll
      for (int n = 0; n < 3; ++n)
#pragma unroll
        for (int pp = 0; pp < 2; ++pp) {
          const int co = 32 * n + 16 * pp + 8 * h;
          float bv[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
          if constexpr (BIAS) {
            const float4 t0 = bq[n][pp][0], t1 = bq[n][pp][1];
            bv[0] = t0.x; bv[1] = t0.y; bv[2] = t0.z; bv[3] = t0.w;
            bv[4] = t1.x; bv[5] = t1.y; bv[6] = t1.z; bv[7] = t1.w;
          }
#pragma unroll
          for (int m = 0; m < MT; ++m) {
            const int y = y0 + 2 * wave + m;
            float v[8];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(acc[m][n][8 * pp + i]),
                                                              __float_as_uint(acc[m][n][8 * pp + 4 + i]), false, false);
              v[i] = __uint_as_float(r[0]) + bv[i];
              v[4 + i] = __uint_as_float(r[1]) + bv[4 + i];
            }
            if (y >= g.H) continue;
            if constexpr (OUT_GGRAD) {
              const u32x4 t = sp[m][n][pp];
#pragma unroll
              for (int i = 0; i < 4; ++i) {
                v[2 * i] *= gelu_grad_fast(Fmt16<T>::lo(t[i]));
                v[2 * i + 1] *= gelu_grad_fast(Fmt16<T>::hi(t[i]));
              }
            }
            const u32x4 pk = {pack2<T>(v[0], v[1]), pack2<T>(v[2], v[3]), pack2<T>(v[4], v[5]), pack2<T>(v[6], v[7])};
            const int off = pix_off32<OUT_D2S>(b, y, xo, g.H, g.W, C) + co;
            // ablation: no output stores (results wrong; the never-true test keeps the MFMAs alive)
            if constexpr (MSU_EXP & 64) if (v[0] != 1.2345e-30f) continue;
            *reinterpret_cast<u32x4*>(Y + off) = pk;
            if constexpr (DUAL) *reinterpret_cast<u32x4*>(Y2 + off) = gelu8<T>(pk);
          }
        }
    }
    }
    if (next >= ntiles) break;
    // the next tile's halo (stored after tap 8) visible to every wave before its tap 0
    __syncthreads();
    tile = next;
    next = tq != nullptr ? read_q() : next + (int)gridDim.x;
  }
  finish();
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

// ------------------------------------------------------------------ bf16 wgrad, v2
// Persistent weight gradient for CinP = Cout = 96 on v_mfma_f32_16x16x32_bf16.  One
// 12-wave workgroup per CU (3 waves per SIMD) owns all 9 x 96 x 96 accumulators for its
// share of the pixels: wave w = (dy = w/4, co half, ci half) holds 3 dx x 3 co-tiles x
// 3 ci-tiles = 27 16x16 tiles (108 registers).  Per pixel tile (4 rows x 32 pixels) the
// input halo [(4+2) x 34][ci] and the dY tile [128][co] sit in LDS (pixel stride 104
// elements); both operands are read k-strided (k = pixels) with ds_read_b64_tr_b16.
// Staging is LDS-DMA (global_load_lds_dwordx4) into the other of two LDS buffers while the
// current tile is multiplied: the image is 13 16-B slots per pixel (12 data + 1 pad) filled
// lane-linearly; pad slots and out-of-image pixels read a 16-B zero block.  After its own
// DMAs land (vmcnt), each wave GELU-converts the halo slots it wrote, in place, so no
// registers are held across the tile and no extra barrier is needed.
// Partials: [block][dy][co][dx][ci] + db [block][co], the layout wgrad_reduce_kernel sums.
template <typename T, bool IN_D2S, bool IN_GELU>
__global__ void __launch_bounds__(768) conv3x3_wgrad_v2_kernel(const bf16_t* __restrict__ X,
                                                               const bf16_t* __restrict__ DY,
                                                               float* __restrict__ part,
                                                               float* __restrict__ dbpart, ConvGeom g,
                                                               int ntiles) {
  constexpr int C = 96, TH = 4, TWV = 32, NW = 12;
  constexpr int PS = C + 8;                  // LDS pixel stride (both images), 13 slots
  constexpr int SLOTS = PS / 8;
  constexpr int HWD = TWV + 2;
  constexpr int HPIX = (TH + 2) * HWD;       // 204 halo pixels
  constexpr int DPIX = TH * TWV;             // 128 dY pixels
  constexpr int NSLOT = (HPIX + DPIX) * SLOTS;
  constexpr int NINS = (NSLOT + 63) / 64;    // DMA wave-instructions per tile
  constexpr int PER_WAVE = (NINS + NW - 1) / NW;
  constexpr int BUF = NINS * 64 * 8;         // elements per LDS buffer (covers the overrun)
  typedef __attribute__((address_space(3))) void lds_void;
  typedef __attribute__((address_space(1))) void glb_void;

  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  bf16_t* lds = reinterpret_cast<bf16_t*>(smem_raw);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int dy = wave >> 2, coh = (wave >> 1) & 1, cih = wave & 1;
  const int tiles_x = (g.W + TWV - 1) / TWV, tiles_y = (g.H + TH - 1) / TH;
  const int per_img = tiles_x * tiles_y;

  auto coords = [&](int tile, int& b, int& y0, int& x0) {
    b = tile / per_img;
    const int r = tile - b * per_img;
    y0 = (r / tiles_x) * TH;
    x0 = (r - (r / tiles_x) * tiles_x) * TWV;
  };
  // issue this wave's DMAs of tile `tile` into buffer `buf`
  auto stage = [&](int tile, int buf) __attribute__((always_inline)) {
    int b, y0, x0;
    coords(tile, b, y0, x0);
    const int ln = opaque(lane);
#pragma unroll
    for (int r = 0; r < PER_WAVE; ++r) {
      const int k = wave + NW * r;
      if (k < NINS) {
        const int s = 64 * k + ln;
        const int pix = s / SLOTS, ch0 = s - (s / SLOTS) * SLOTS;
        const int ch = ch0 < SLOTS - 1 ? ch0 : 0;  // pad slot: re-read chunk 0 of the pixel
        const void* src = zero_src(s);
        if (pix < HPIX) {
          const int row = pix / HWD, col = pix - (pix / HWD) * HWD;
          const int y = y0 - 1 + row, x = x0 - 1 + col;
          if (y >= 0 && y < g.H && x >= 0 && x < g.W) src = X + pix_off32<IN_D2S>(b, y, x, g.H, g.W, C) + ch * 8;
        } else if (pix < HPIX + DPIX) {
          const int dp = pix - HPIX;
          const int y = y0 + dp / TWV, x = x0 + dp % TWV;
          if (y < g.H && x < g.W) src = DY + pix_off32<false>(b, y, x, g.H, g.W, C) + ch * 8;
        }
        // ablation 4096: no DMA (the LDS images stay stale; results wrong)
        if constexpr (!(MSU_EXP & 4096))
          __builtin_amdgcn_global_load_lds((glb_void*)src, (lds_void*)(lds + buf * BUF + 64 * 8 * k), 16, 0, 0);
      }
    }
  };
  // after this wave's DMAs landed: GELU the halo slots it wrote, in place
  auto gelu_own = [&](int buf) __attribute__((always_inline)) {
    if constexpr (IN_GELU) {
      const int ln = opaque(lane);
#pragma unroll
      for (int r = 0; r < PER_WAVE; ++r) {
        const int k = wave + NW * r;
        const int s = 64 * k + ln;
        if (k < NINS && s / SLOTS < HPIX && s % SLOTS < SLOTS - 1) {
          u32x4* p = reinterpret_cast<u32x4*>(lds + buf * BUF + 8 * s);
          *p = gelu8<T>(*p);
        }
      }
    }
  };

  f32x4 acc[3][3][3];  // [dx][co tile][ci tile]
#pragma unroll
  for (int d = 0; d < 3; ++d)
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
      for (int j = 0; j < 3; ++j) acc[d][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  float dbacc[2] = {0.f, 0.f};
  const int dbc = 2 * (tid % 48), dbg = tid / 48;  // channel pair, pixel group (16 groups)

  int tile = blockIdx.x;
  int cur = 0;
  if (tile < ntiles) {
    stage(tile, 0);
    __builtin_amdgcn_s_waitcnt(0);  // vmcnt(0) & lgkmcnt(0)
    gelu_own(0);
  }
  __syncthreads();
  for (; tile < ntiles; tile += gridDim.x) {
    const int next = tile + gridDim.x;
    if (next < ntiles) stage(next, cur ^ 1);
    const bf16_t* sX = lds + cur * BUF;
    const bf16_t* sD = sX + HPIX * PS;
    // All LDS reads of the tile are untracked (inline asm): a compiler-visible ds_read would
    // be preceded by vmcnt(0) for the next tile's pending LDS-DMA and serialise the two.
    // bias gradient: 16 groups x 48 channel pairs, 8 pixels each (ablation 65536: none)
    if constexpr (!(MSU_EXP & 65536)) {
      const uint32_t ba = lds_u32(sD + dbg * PS + dbc);
      uint32_t v[DPIX / 16];
      unroll_for<DPIX / 16>([&](auto P) {
        v[decltype(P)::value] = ds_b32_untracked<2 * 16 * PS * decltype(P)::value>(ba);
      });
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
      for (int p = 0; p < DPIX / 16; ++p) {
        vreg_pin(v[p]);
        dbacc[0] += Fmt16<T>::lo(v[p]);
        dbacc[1] += Fmt16<T>::hi(v[p]);
      }
    }
    // lane part of a k-strided fragment read: pixels 2(4g + q) + half (+16 for the second
    // half of the fragment), g = lane group within the 32-lane half, q = (lane&15)>>2,
    // columns 4(lane&3); everything else is an immediate offset.  Same pixel order for both
    // operands; pixels of one parity sit 104 * 2j B apart: distinct 32-B bank spans, so each
    // half's 32 lanes hit all 64 banks once (pixels 8(lane>>4) + q: 2-way conflicts).
    const int laneoff = opaque((2 * (4 * ((lane >> 4) & 1) + ((lane & 15) >> 2)) + (lane >> 5)) * PS + 4 * (lane & 3));
    const uint32_t xa = lds_u32(sX + laneoff + dy * HWD * PS + 48 * cih);
    const uint32_t da = lds_u32(sD + laneoff + 48 * coh);
    unroll_for<TH>([&](auto R) {
      constexpr int r = decltype(R)::value;
      // the dY fragments of row r serve all three dx (read once per row, not once per dx:
      // 12 instead of 18 fragment reads per 27 MFMAs -- the LDS reads bound this loop).
      // (Reading group g + 1's X fragments before group g's MFMAs measured no faster, r06x:
      // the loop is bound by its operand traffic, ablations r06w.)
      bf16x8 af[3];
      unroll_for<3>([&](auto I) {
        constexpr int o = 2 * (r * TWV * PS + 16 * decltype(I)::value);
        if constexpr (MSU_EXP & 32768) af[decltype(I)::value] = bf16x8{};  // ablation: no fragment reads
        else af[decltype(I)::value] = tr8_untracked<o, o + 32 * PS>(da);
      });
      unroll_for<3>([&](auto D) {
        constexpr int d = decltype(D)::value;
        bf16x8 bf[3];
        unroll_for<3>([&](auto J) {
          constexpr int o = 2 * ((r * HWD + d) * PS + 16 * decltype(J)::value);
          if constexpr (MSU_EXP & 32768) bf[decltype(J)::value] = bf16x8{};
          else bf[decltype(J)::value] = tr8_untracked<o, o + 32 * PS>(xa);
        });
        if constexpr (d == 0)
          lds_wait_tie<0>(bf[0], bf[1], bf[2], af[0], af[1], af[2]);
        else
          lds_wait_tie<0>(bf[0], bf[1], bf[2]);
#pragma unroll
        for (int i = 0; i < 3; ++i)
#pragma unroll
          for (int j = 0; j < 3; ++j)
            if constexpr (MSU_EXP & 16384) asm volatile("" ::"v"(af[i]), "v"(bf[j]));  // ablation: no MFMA
            else acc[d][i][j] = Fmt16<T>::mma16(af[i], bf[j], acc[d][i][j]);
        __builtin_amdgcn_sched_barrier(0);
      });
    });
    if (next < ntiles) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      gelu_own(cur ^ 1);
    }
    __syncthreads();
    cur ^= 1;
  }
  // partial [blk][dy][co][dx][ci]: lane holds co = co0 + 4(lane>>4) + r, ci = ci0 + (lane&15)
  float* out = part + ((long)blockIdx.x * 3 + dy) * (long)C * 3 * C;
#pragma unroll
  for (int d = 0; d < 3; ++d)
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
      for (int j = 0; j < 3; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int co = 48 * coh + 16 * i + 4 * (lane >> 4) + r;
          const int ci = 48 * cih + 16 * j + (lane & 15);
          out[((long)co * 3 + d) * C + ci] = acc[d][i][j][r];
        }
  // bias partial: reduce the 16 pixel groups through LDS
  float* red = reinterpret_cast<float*>(smem_raw);
  __syncthreads();
  red[dbg * C + dbc] = dbacc[0];
  red[dbg * C + dbc + 1] = dbacc[1];
  __syncthreads();
  if (tid < C) {
    float sum = 0.f;
#pragma unroll
    for (int q = 0; q < 16; ++q) sum += red[q * C + tid];
    dbpart[(long)blockIdx.x * C + tid] = sum;
  }
}

// chunk-summed partial [dy][co][dx][ci] -> dW[co][ci][3][3] (torch Conv2d layout)
__global__ void __launch_bounds__(256) wgrad_permute_kernel(const float* __restrict__ sum, int Cout, int Cin,
                                                            int CinP, float* __restrict__ dW, int accumulate) {
  const long n = (long)Cout * Cin * 9;
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i < n) {
    const int co = (int)(i / (Cin * 9));
    const int rem = (int)(i - (long)co * Cin * 9);
    const int ci = rem / 9, tap = rem % 9, dy = tap / 3, dx = tap % 3;
    const float v = sum[((long)dy * Cout * 3 + (long)co * 3 + dx) * CinP + ci];
    dW[i] = accumulate ? dW[i] + v : v;
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

template <typename T, int NT, bool IN_D2S, bool IN_GELU, bool OUT_D2S, bool OUT_GGRAD, bool BIAS, bool DUAL>
int launch_conv(const ConvGeom& g, const T* X, const T* Wt, const float* bias, const T* S, T* Y, T* Y2,
                hipStream_t st) {
  constexpr bool BF = sizeof(T) == 2;
  constexpr int TH = BF ? 16 : 4;
  constexpr int MT = BF ? 2 : 1;
  constexpr int NW = TH / MT;
  const size_t lds = sizeof(T) * ((size_t)(TH + 2) * (TW + 2) * g.PS + (size_t)(BF ? 2 : 1) * g.Cout * g.PSW);
  if (lds > 160 * 1024) return -4;
  auto kern = conv3x3_kernel<T, NT, TH, MT, BF, IN_D2S, IN_GELU, OUT_D2S, OUT_GGRAD, BIAS, DUAL>;
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr_set = true;
  }
  const long ntiles = (long)g.B * ((g.W + TW - 1) / TW) * ((g.H + TH - 1) / TH);
  if (ntiles == 0) return 0;
  hipLaunchKernelGGL(kern, dim3((unsigned)ntiles), dim3(64 * NW), lds, st, X, Wt, bias, S, Y, Y2, g);
  return MSU_CHECK_LAUNCH();
}

// msu_conv_mode bit 0 (default on; A/B switch MSU_CONV_DYN): conv3x3_v3_kernel takes tiles
// from the per-stream queue slot instead of the static blockIdx.x + k * gridDim.x schedule
int g_conv_dyn = 1;

int num_cus() {
  static int n = 0;
  if (n <= 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
  }
  return n;
}

template <typename T, int NCT, int KS, int NW, int MT, bool WDB, bool IN_D2S, bool IN_GELU, bool OUT_D2S,
          bool OUT_GGRAD, bool BIAS, bool DUAL>
int launch_v2(const ConvGeom& g, const bf16_t* X, const bf16_t* Wt, const float* bias, const bf16_t* S,
              bf16_t* Y, bf16_t* Y2, hipStream_t st) {
  constexpr int PS = KS * 16 + 8, TH = NW * MT;
  constexpr size_t lds = sizeof(bf16_t) * ((size_t)(TH + 2) * 34 * PS + (WDB ? 2 : 1) * (size_t)NCT * 32 * PS);
  static_assert(lds <= 160 * 1024, "LDS");
  auto kern = conv3x3_v2_kernel<T, NCT, KS, NW, MT, WDB, IN_D2S, IN_GELU, OUT_D2S, OUT_GGRAD, BIAS, DUAL>;
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr_set = true;
  }
  const long ntiles = (long)g.B * ((g.W + 31) / 32) * ((g.H + TH - 1) / TH);
  if (ntiles == 0) return 0;
  // 32-bit element offsets inside the kernel
  if ((long)g.B * g.H * g.W * (g.Cin > g.Cout ? g.Cin : g.Cout) >= (1L << 31)) return -2;
  const int grid = (int)(ntiles < num_cus() ? ntiles : num_cus());
  hipLaunchKernelGGL(kern, dim3(grid), dim3(64 * NW), lds, st, X, Wt, bias, S, Y, Y2, g, (int)ntiles);
  return MSU_CHECK_LAUNCH();
}

template <typename T, bool IN_D2S, bool OUT_D2S, bool OUT_GGRAD, bool BIAS, bool DUAL, bool SPREAD, bool M16>
int launch_v3s(const ConvGeom& g, const bf16_t* X, const bf16_t* Wt, const float* bias, const bf16_t* S, bf16_t* Y,
               bf16_t* Y2, hipStream_t st) {
  constexpr size_t lds = sizeof(bf16_t) * ((size_t)18 * 34 * 96 + 2 * 96 * 96) + 96 * sizeof(float) + 16;  // + bias, queue
  static_assert(lds <= 160 * 1024, "LDS");
  auto kern = conv3x3_v3_kernel<T, IN_D2S, OUT_D2S, OUT_GGRAD, BIAS, DUAL, SPREAD, M16>;
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr_set = true;
  }
  const long ntiles = (long)g.B * ((g.W + 31) / 32) * ((g.H + 15) / 16);
  if (ntiles == 0) return 0;
  if ((long)g.B * g.H * g.W * 96 >= (1L << 31)) return -2;
  const int grid = (int)(ntiles < num_cus() ? ntiles : num_cus());
  hipLaunchKernelGGL(kern, dim3(grid), dim3(512), lds, st, X, Wt, bias, S, Y, Y2, g, (int)ntiles,
                     g_conv_dyn ? tile_queue(st) : nullptr);
  return MSU_CHECK_LAUNCH();
}

template <typename T, bool IN_D2S, bool OUT_D2S, bool OUT_GGRAD, bool BIAS, bool DUAL>
int launch_v3(const ConvGeom& g, const bf16_t* X, const bf16_t* Wt, const float* bias, const bf16_t* S, bf16_t* Y,
              bf16_t* Y2, hipStream_t st) {
  // Forward launches on 16x16x32 MFMA (same tile, LDS images and schedule; (p >> 1) & 3
  // swizzle), since round 4: same-box kbench (r04b) conv1 2.22-2.28 vs 2.44 ms, conv2 1.48 vs
  // 1.55 ms (bare MFMA loops of this shape run at ~1.12-1.15x the FLOP/s of 32x32x16 on MI355X at
  // equal cycles: the clock it holds, MI355X_MICROARCH.md).  The dgrad keeps 32x32x16: with its
  // GELU' operands held from tap 7 the 16x16 form spills 260 B per lane.  Halo loads spread over
  // taps 1..7 (SPREAD; all at tap 1 measured equal, r03).  v4 (one wave per SIMD, 4 rows per
  // wave) was 7-10 % slower on every launch (r03l/m) and is gone.
  // (ablation 2048: the dgrad on 16 x 16 x 32 too)
  if constexpr (!OUT_GGRAD || (MSU_EXP & 2048) != 0)
    return launch_v3s<T, IN_D2S, OUT_D2S, OUT_GGRAD, BIAS, DUAL, true, true>(g, X, Wt, bias, S, Y, Y2, st);
  return launch_v3s<T, IN_D2S, OUT_D2S, OUT_GGRAD, BIAS, DUAL, true, false>(g, X, Wt, bias, S, Y, Y2, st);
}

template <typename T, bool IN_D2S, bool IN_GELU, bool OUT_D2S, bool OUT_GGRAD, bool BIAS, bool DUAL = false>
int conv_nt(const ConvGeom& g, const void* X, const void* Wt, const float* bias, const void* S,
            void* Y, void* Y2, hipStream_t st) {
  const T* x = (const T*)X; const T* w = (const T*)Wt; const T* s = (const T*)S; T* y = (T*)Y; T* y2 = (T*)Y2;
  if constexpr (sizeof(T) == 2 && !IN_GELU) {
    if (g.Cout == 96 && g.CinP == 96 && g.Cin == 96)
      return launch_v3<T, IN_D2S, OUT_D2S, OUT_GGRAD, BIAS, DUAL>(g, (const bf16_t*)x, (const bf16_t*)w, bias,
                                                                  (const bf16_t*)s, (bf16_t*)y, (bf16_t*)y2, st);
  }
  if constexpr (sizeof(T) == 2) {
    // the Swin-T/S decoder head width takes the persistent v2 kernel
    if (g.Cout == 96 && g.CinP == 96)
      return launch_v2<T, 3, 6, 8, 1, true, IN_D2S, IN_GELU, OUT_D2S, OUT_GGRAD, BIAS, DUAL>(g, (const bf16_t*)x,
                                                                                          (const bf16_t*)w, bias,
                                                                                          (const bf16_t*)s, (bf16_t*)y,
                                                                                          (bf16_t*)y2, st);
  }
  switch (g.Cout / 16) {
    case 1: return launch_conv<T, 1, IN_D2S, IN_GELU, OUT_D2S, OUT_GGRAD, BIAS, DUAL>(g, x, w, bias, s, y, y2, st);
    case 2: return launch_conv<T, 2, IN_D2S, IN_GELU, OUT_D2S, OUT_GGRAD, BIAS, DUAL>(g, x, w, bias, s, y, y2, st);
    case 4: return launch_conv<T, 4, IN_D2S, IN_GELU, OUT_D2S, OUT_GGRAD, BIAS, DUAL>(g, x, w, bias, s, y, y2, st);
    case 6: return launch_conv<T, 6, IN_D2S, IN_GELU, OUT_D2S, OUT_GGRAD, BIAS, DUAL>(g, x, w, bias, s, y, y2, st);
    case 8: return launch_conv<T, 8, IN_D2S, IN_GELU, OUT_D2S, OUT_GGRAD, BIAS, DUAL>(g, x, w, bias, s, y, y2, st);
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
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
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
int launch_wgrad_v2(const ConvGeom& g, const bf16_t* X, const bf16_t* DY, float* part, float* dbpart,
                    int nblocks, hipStream_t st) {
  constexpr int nins = ((6 * 34 + 4 * 32) * 13 + 63) / 64;
  constexpr size_t lds = 2 * sizeof(bf16_t) * (size_t)nins * 64 * 8;
  static_assert(lds <= 160 * 1024, "LDS");
  auto kern = conv3x3_wgrad_v2_kernel<T, IN_D2S, IN_GELU>;
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr_set = true;
  }
  if ((long)g.B * g.H * g.W * 96 >= (1L << 31)) return -2;
  const long ntiles = (long)g.B * ((g.W + 31) / 32) * ((g.H + 3) / 4);
  // every block writes its partial slabs, even with no tile (zeros)
  hipLaunchKernelGGL(kern, dim3((unsigned)nblocks), dim3(768), lds, st, X, DY, part, dbpart, g, (int)ntiles);
  return MSU_CHECK_LAUNCH();
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

