// Input pipeline: the reference's per-sample CPU augmentation + normalisation
// (dataset/dataset.py:20-95, RandomGenerator / DataPrepartion, albumentations + cv2 inside
// DataLoader workers) as ONE batched gfx950 pass over the decoded uint8 pixels.
//
// Per sample, the host draws the operations and builds their 256-entry uint8 LUTs exactly as
// albumentations 1.x does (dataset/augment.py); this kernel applies, per pixel and in the
// reference's Compose order (dataset.py:26-34):
//   ToGray            cv2 RGB2GRAY 8U fixed point (R 4899, G 9617, B 1868, >> 14), 3 channels
//   BrightnessContrast  lut[0] on every channel
//   HueSaturationValue  cv2 RGB2HSV_b (integer, H in [0,180)) -> lut[1..3] on H, S, V ->
//                       cv2 HSV2RGB_b (f32 sector formula, rounded half-even)
//   RandomGamma       lut[4]                     } OneOf (:30-33): at most one of the two
//   GaussianBlur      3x3 / 5x5 binomial (cv2's } fixed-point kernels for sigma 0), border
//                     reflect-101, integer-exact rounding (sum + half) >> shift
//   random_flip       horizontal (dataset.py:13-16), applied to image and label
// then the normalisation (dataset.py:65-66, :83-84): image f32 [3, H, W] = u8 / 255 (planar),
// label f32 [H, W] = (u8 > 127).
//
// Layout: img [B, H, W, 3] u8 (PIL RGB order), label [B, H, W] u8 (PIL "L"); ops [B][2] i32
// (bits, blur ksize); luts [B][5][256] u8; out [B, 3, H, W] f32, out_label [B, H, W] f32.
// HBM-bound: 4 B read + 16 B written per pixel.  One workgroup = a 64 x 16 output tile of one
// sample; the point-wise chain runs once per source pixel (halo included when the sample
// blurs) into an LDS tile that the blur and the flipped, planar float4 stores read.
#pragma clang fp contract(off)  // the HSV f32 formula must round like cv2's scalar code
#include "common.h"

namespace {

constexpr int TW = 64, TH = 16, HR = 2, SW = TW + 2 * HR, SH = TH + 2 * HR;
enum { OP_GRAY = 1, OP_BC = 2, OP_HSV = 4, OP_GAMMA = 8, OP_FLIP = 16 };

MSU_DEV int reflect101(int i, int n) {
  if (n == 1) return 0;
  while (i < 0 || i >= n) {
    if (i < 0) i = -i;
    if (i >= n) i = 2 * n - 2 - i;
  }
  return i;
}

MSU_DEV int sat_u8(float f) {
  const float r = __builtin_rintf(f);  // cvRound: nearest, ties to even
  return r <= 0.f ? 0 : (r >= 255.f ? 255 : (int)r);
}

// cv2 RGB2HSV_b (hsv_shift 12, hrange 180) on one pixel.
MSU_DEV void rgb2hsv(int r, int g, int b, const int* sdiv, const int* hdiv, int& h, int& s, int& v) {
  v = max(max(b, g), r);
  const int vmin = min(min(b, g), r);
  const int diff = v - vmin;
  const int vr = v == r ? -1 : 0, vg = v == g ? -1 : 0;
  s = (diff * sdiv[v] + (1 << 11)) >> 12;
  h = (vr & (g - b)) + (~vr & ((vg & (b - r + 2 * diff)) + ((~vg) & (r - g + 4 * diff))));
  h = (h * hdiv[diff] + (1 << 11)) >> 12;
  h += h < 0 ? 180 : 0;
  h = min(max(h, 0), 255);
}

MSU_DEV float pick4(f32x4 t, unsigned i) { return i == 0 ? t[0] : (i == 1 ? t[1] : (i == 2 ? t[2] : t[3])); }

// cv2 HSV2RGB_b (hrange 180): f32 sector formula, x255 and cvRound.
MSU_DEV void hsv2rgb(int hi, int si, int vi, int& r, int& g, int& b) {
  const float inv255 = 1.f / 255.f;
  float h = (float)hi;
  const float s = (float)si * inv255, v = (float)vi * inv255;
  float bf, gf, rf;
  if (s == 0.f) {
    bf = gf = rf = v;
  } else {
    h = h * (6.f / 180.f);
    if (h >= 6.f) h -= 6.f;  // = fmod(h, 6) on this range (h <= 180 * 6/180)
    int sector = (int)__builtin_floorf(h);
    h = h - (float)sector;
    if ((unsigned)sector >= 6u) { sector = 0; h = 0.f; }
    const f32x4 tab = {v, v * (1.f - s), v * (1.f - s * h), v * (1.f - s * (1.f - h))};
    // cv2 sector_data {{1,3,0},{1,0,2},{3,0,1},{0,2,1},{0,1,3},{2,1,0}} -> tab index of (b, g, r),
    // packed 2 bits per sector (selects, no indexed private arrays)
    const unsigned ib = (0x835u >> (2 * sector)) & 3u;  // 1,1,3,0,0,2
    const unsigned ig = (0x583u >> (2 * sector)) & 3u;  // 3,0,0,2,1,1
    const unsigned ir = (0x358u >> (2 * sector)) & 3u;  // 0,2,1,1,3,0
    bf = pick4(tab, ib);
    gf = pick4(tab, ig);
    rf = pick4(tab, ir);
  }
  b = sat_u8(bf * 255.f);
  g = sat_u8(gf * 255.f);
  r = sat_u8(rf * 255.f);
}

struct AugShared {
  uint8_t lut[5][256];
  int sdiv[256], hdiv[256];
  float norm[256];
  uint32_t tile[SH][SW];  // point-wise result, r | g << 8 | b << 16
};

MSU_DEV int chan(uint32_t p, int c) { return (int)((p >> (8 * c)) & 0xffu); }

__global__ __launch_bounds__(256) void augment_kernel(const uint8_t* __restrict__ img, const uint8_t* __restrict__ lbl,
                                                      const int* __restrict__ ops, const uint8_t* __restrict__ luts,
                                                      float* __restrict__ out, float* __restrict__ out_lbl, int H,
                                                      int W) {
  __shared__ AugShared sh;
  const int t = threadIdx.x;
  const int b = blockIdx.z;
  const int op = ops ? ops[2 * b] : 0;
  const int ks = ops ? ops[2 * b + 1] : 0;
  const bool flip = (op & OP_FLIP) != 0;

  // tables: cv2's sdiv / hdiv (saturate_cast<int> of a double = round half even), u8 / 255 in f32
  sh.sdiv[t] = t == 0 ? 0 : (int)__builtin_rint((double)(255 << 12) / (double)t);
  sh.hdiv[t] = t == 0 ? 0 : (int)__builtin_rint((double)(180 << 12) / (6.0 * (double)t));
  sh.norm[t] = (float)t / 255.f;
  if (luts) {
    const uint8_t* l = luts + (long)b * 5 * 256;
#pragma unroll
    for (int k = 0; k < 5; ++k) sh.lut[k][t] = l[k * 256 + t];
  }
  __syncthreads();

  const int oy0 = blockIdx.y * TH, ox0 = blockIdx.x * TW;
  // tile column c <-> source column sx0 + c; output column = flip ? W-1-(sx0+c) : sx0+c
  const int sx0 = flip ? W - ox0 - TW : ox0;
  const long plane = (long)H * W;
  const uint8_t* src = img + (long)b * plane * 3;
  const int halo = ks > 0 ? HR : 0;
  const int rows = TH + 2 * halo, cols = TW + 2 * halo;
  for (int i = t; i < rows * cols; i += 256) {
    const int ty = i / cols, tx = i - ty * cols;
    const int sy = reflect101(oy0 - halo + ty, H), sx = reflect101(sx0 - halo + tx, W);
    const uint8_t* p = src + ((long)sy * W + sx) * 3;
    int r = p[0], g = p[1], bl = p[2];
    if (op & OP_GRAY) {
      const int y = (r * 4899 + g * 9617 + bl * 1868 + (1 << 13)) >> 14;
      r = g = bl = y;
    }
    if (op & OP_BC) {
      r = sh.lut[0][r];
      g = sh.lut[0][g];
      bl = sh.lut[0][bl];
    }
    if (op & OP_HSV) {
      int h, s, v;
      rgb2hsv(r, g, bl, sh.sdiv, sh.hdiv, h, s, v);
      hsv2rgb(sh.lut[1][h], sh.lut[2][s], sh.lut[3][v], r, g, bl);
    }
    if (op & OP_GAMMA) {
      r = sh.lut[4][r];
      g = sh.lut[4][g];
      bl = sh.lut[4][bl];
    }
    sh.tile[ty + HR - halo][tx + HR - halo] = (uint32_t)r | ((uint32_t)g << 8) | ((uint32_t)bl << 16);
  }
  __syncthreads();

  // 16 lanes per output row, 4 consecutive output pixels per lane
  const int ty = t >> 4, j0 = (t & 15) * 4;
  const int oy = oy0 + ty;
  if (oy >= H) return;
  int px[4][3];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int j = j0 + q;
    const int c = (flip ? TW - 1 - j : j) + HR;
    const int y = ty + HR;
    if (ks == 3) {
      const int a[3] = {1, 2, 1};
#pragma unroll
      for (int ch = 0; ch < 3; ++ch) {
        int acc = 0;
#pragma unroll
        for (int dy = -1; dy <= 1; ++dy)
#pragma unroll
          for (int dx = -1; dx <= 1; ++dx) acc += a[dy + 1] * a[dx + 1] * chan(sh.tile[y + dy][c + dx], ch);
        px[q][ch] = (acc + 8) >> 4;
      }
    } else if (ks == 5) {
      const int a[5] = {1, 4, 6, 4, 1};
#pragma unroll
      for (int ch = 0; ch < 3; ++ch) {
        int acc = 0;
#pragma unroll
        for (int dy = -2; dy <= 2; ++dy)
#pragma unroll
          for (int dx = -2; dx <= 2; ++dx) acc += a[dy + 2] * a[dx + 2] * chan(sh.tile[y + dy][c + dx], ch);
        px[q][ch] = (acc + 128) >> 8;
      }
    } else {
      const uint32_t p = sh.tile[y][c];
#pragma unroll
      for (int ch = 0; ch < 3; ++ch) px[q][ch] = chan(p, ch);
    }
  }
  const int ox = ox0 + j0;
  float* o = out + (long)b * 3 * plane + (long)oy * W;
  const bool vec = (W & 3) == 0 && ox + 3 < W;
#pragma unroll
  for (int ch = 0; ch < 3; ++ch) {
    if (vec) {
      f32x4 v = {sh.norm[px[0][ch]], sh.norm[px[1][ch]], sh.norm[px[2][ch]], sh.norm[px[3][ch]]};
      *reinterpret_cast<f32x4*>(o + ch * plane + ox) = v;
    } else {
      for (int q = 0; q < 4; ++q)
        if (ox + q < W) o[ch * plane + ox + q] = sh.norm[px[q][ch]];
    }
  }
  if (lbl) {
    const uint8_t* l = lbl + (long)b * plane + (long)oy * W;
    float* ol = out_lbl + (long)b * plane + (long)oy * W;
    float lv[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int x = ox + q;
      const int sx = flip ? W - 1 - x : x;
      lv[q] = (x < W && l[sx] > 127) ? 1.f : 0.f;
    }
    if (vec) {
      *reinterpret_cast<f32x4*>(ol + ox) = f32x4{lv[0], lv[1], lv[2], lv[3]};
    } else {
      for (int q = 0; q < 4; ++q)
        if (ox + q < W) ol[ox + q] = lv[q];
    }
  }
}

}  // namespace

extern "C" {

// img [B, H, W, 3] u8, label [B, H, W] u8 or null; ops [B][2] i32 (bits, blur ksize 0/3/5) or
// null (normalisation only); luts [B][5][256] u8 (null only with ops null); out [B, 3, H, W]
// f32; out_label [B, H, W] f32 (null with label null).
int msu_augment_batch(const unsigned char* img, const unsigned char* label, const int* ops,
                      const unsigned char* luts, float* out, float* out_label, int B, int H, int W,
                      void* stream) {
  if (B <= 0 || H <= 0 || W <= 0 || !img || !out) return -2;
  if ((label == nullptr) != (out_label == nullptr)) return -2;
  if (ops && !luts) return -2;
  if ((long)B * H * W * 3 >= (1L << 40)) return -2;
  const dim3 grid((unsigned)((W + TW - 1) / TW), (unsigned)((H + TH - 1) / TH), (unsigned)B);
  if (grid.z > 65535u || grid.y > 65535u) return -2;
  hipLaunchKernelGGL(augment_kernel, grid, dim3(256), 0, (hipStream_t)stream, img, label, ops, luts, out,
                     out_label, H, W);
  return MSU_CHECK_LAUNCH();
}

}  // extern "C"
