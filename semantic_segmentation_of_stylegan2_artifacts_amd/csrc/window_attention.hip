// Shifted-window multi-head self-attention core (torchvision v1 semantics).
//
// Replaces torchvision `shifted_window_attention` (called from SwinTransformerBlock at
// network/model_parts.py:170 / :538) between the qkv and proj Linears:
//   pad-to-7 -> roll(-s) -> window partition -> q*hd^-1/2 k^T + B_rel[idx] (+ -100 shift
//   mask) -> softmax -> dropout -> @v -> un-partition -> roll(+s) -> crop.
// Pad / roll / partition / reverse are NOT materialised: every window token is mapped
// back to its source token on the unpadded [B,H,W,3C] qkv tensor; padded tokens carry
// q,k,v = qkv bias (torchvision pads AFTER norm1, so F.linear(0) = bias), and their
// output rows are never written (cropped).  Backward sums the padded tokens' dq,dk,dv
// into a qkv-bias gradient partial and the dS tiles into a relative-bias partial.
//
// One 64-lane wave owns one (window, head): Q,K,V (49 x 32, zero-padded to 64 rows) are
// staged in LDS as row images; the products run on MFMA 16x16 (bf16:
// v_mfma_f32_16x16x32_bf16, f32: v_mfma_f32_16x16x4_f32) reading operands either
// k-contiguous (one 16-B read per fragment) or k-strided (8 scalar reads) so no transposed
// copies are staged; softmax runs in registers one 16-row block at a time.
#include "common.h"
#include "reduce.h"

namespace {

constexpr int WS = 7, NT = 49, HD = 32;

// acc(16x16) += A(16x32) * B(32x16).
//   AK: A(m,k) = A[m*lda + k] (k contiguous)  else A[k*lda + m]
//   BK: B(k,n) = B[n*ldb + k] (k contiguous)  else B[k*ldb + n]
template <typename T, bool AK, bool BK> struct MM;
template <bool AK, bool BK> struct MM<bf16_t, AK, BK> {
  static MSU_DEV bf16x8 frag(const bf16_t* P, int ld, bool kc, int lane) {
    const int r = lane & 15, k0 = 8 * (lane >> 4);
    if (kc) return *reinterpret_cast<const bf16x8*>(P + r * ld + k0);
    bf16x8 f;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      bf16_t v = P[(k0 + e) * ld + r];
      f[e] = *reinterpret_cast<__bf16*>(&v);
    }
    return f;
  }
  static MSU_DEV void k32(f32x4& acc, const bf16_t* A, int lda, const bf16_t* B, int ldb, int lane) {
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(frag(A, lda, AK, lane), frag(B, ldb, BK, lane), acc, 0, 0, 0);
  }
};
template <bool AK, bool BK> struct MM<float, AK, BK> {
  static MSU_DEV void k32(f32x4& acc, const float* A, int lda, const float* B, int ldb, int lane) {
    const int r = lane & 15, k = lane >> 4;
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      const float a = AK ? A[r * lda + 4 * s + k] : A[(4 * s + k) * lda + r];
      const float b = BK ? B[r * ldb + 4 * s + k] : B[(4 * s + k) * ldb + r];
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc, 0, 0, 0);
    }
  }
};
template <typename T> constexpr int row_pad() { return sizeof(T) == 2 ? 8 : 4; }

struct WinGeom {
  int B, H, W, Hp, Wp, nWy, nWx, sh, sw, C, nh;
  long nwin;  // B * nWy * nWx
};

// torchvision mask regions on the padded grid: [0, P-ws) / [P-ws, P-s) / [P-s, P);
// with s == 0 on an axis every row lands in one region (the (-0, None) slice wins).
MSU_DEV int region(int p, int P, int s) { return s == 0 ? 0 : (p < P - WS ? 0 : (p < P - s ? 1 : 2)); }

// Token table of window `win`: sTok[t] = source token (-1: padded), sReg[t] = mask region.
MSU_DEV void window_tokens(const WinGeom& g, long win, int* sTok, int* sReg, int lane) {
  const int nw = g.nWy * g.nWx;
  const long b = win / nw;
  const int wr = (int)(win - b * nw);
  const int wy = wr / g.nWx, wx = wr - (wr / g.nWx) * g.nWx;
  const int t = lane;
  int tok = -1, reg = 0;
  if (t < NT) {
    const int py = wy * WS + t / WS, px = wx * WS + t % WS;
    int sy = py + g.sh; if (sy >= g.Hp) sy -= g.Hp;
    int sx = px + g.sw; if (sx >= g.Wp) sx -= g.Wp;
    if (sy < g.H && sx < g.W) tok = (int)((b * g.H + sy) * (long)g.W + sx);
    reg = region(py, g.Hp, g.sh) * 3 + region(px, g.Wp, g.sw);
  }
  sTok[t] = tok;
  sReg[t] = reg;
}

// Stage one [64 x 32] head slice of the window into LDS (rows >= 49 zero).  Padded tokens
// take `bias` (rounded to T) when non-null, zero otherwise.
template <typename T>
MSU_DEV void stage_rows(const int* sTok, const T* src, long row_stride, int col0,
                        const float* bias, float mul, T* dst, int ldd, int lane) {
  for (int c = lane; c < 64 * 4; c += 64) {
    const int t = c >> 2, q = c & 3;
    float v[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = 0.f;
    if (t < NT) {
      const int tok = sTok[t];
      if (tok < 0) {
        if (bias) {
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] = to_f32(from_f32<T>(bias[col0 + q * 8 + e])) * mul;
        }
      } else {
        const T* p = src + (long)tok * row_stride + col0 + q * 8;
        float a[4], b[4];
        Vec4<T>::load(p, a);
        Vec4<T>::load(p + 4, b);
#pragma unroll
        for (int e = 0; e < 4; ++e) { v[e] = a[e] * mul; v[4 + e] = b[e] * mul; }
      }
    }
    float lo[4] = {v[0], v[1], v[2], v[3]}, hi[4] = {v[4], v[5], v[6], v[7]};
    Vec4<T>::store(dst + t * ldd + q * 8, lo);
    Vec4<T>::store(dst + t * ldd + q * 8 + 4, hi);
  }
}

// Scores of 16-row block mi: S[ni] (C layout) = Q K^T + B_rel + mask; rows/cols >= 49 fixed up.
template <typename T>
MSU_DEV void scores_block(f32x4 (&S)[4], int mi, const T* sQ, const T* sK, int ld,
                          const int* sReg, bool shifted, const float* table, int nh, int h, int lane) {
#pragma unroll
  for (int ni = 0; ni < 4; ++ni) {
    S[ni] = f32x4{0.f, 0.f, 0.f, 0.f};
    MM<T, true, true>::k32(S[ni], sQ + mi * 16 * ld, ld, sK + ni * 16 * ld, ld, lane);
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int i = mi * 16 + (lane >> 4) * 4 + r;
    const int ih = i / WS, iw = i % WS;
    const int rreg = sReg[i < 64 ? i : 63];
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) {
      const int j = ni * 16 + (lane & 15);
      float s = S[ni][r];
      if (j >= NT) {
        s = -INFINITY;
      } else if (i >= NT) {
        s = 0.f;
      } else {
        const int idx = (ih - j / WS + WS - 1) * (2 * WS - 1) + (iw - j % WS + WS - 1);
        s += table[idx * nh + h];
        if (shifted && rreg != sReg[j]) s += -100.0f;
      }
      S[ni][r] = s;
    }
  }
}

MSU_DEV void softmax_block(f32x4 (&S)[4]) {
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    float m = fmaxf(fmaxf(S[0][r], S[1][r]), fmaxf(S[2][r], S[3][r]));
    m = group_max<16>(m);
    float sum = 0.f;
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) {
      const float e = __expf(S[ni][r] - m);
      S[ni][r] = e;
      sum += e;
    }
    sum = group_sum<16>(sum);
    const float inv = 1.0f / sum;
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) S[ni][r] *= inv;
  }
}

// the 16-bit kernels' mask (common.h drop streams), one element at a time
MSU_DEV float drop_keep(uint64_t seed, long win, int h, int nh, int i, int j, float p) {
  return drop_keep_bit(drop_seed32(seed), (uint32_t)(win * nh + h), i, j, drop_thresh16(p)) ? 1.0f / (1.0f - p)
                                                                                             : 0.0f;
}

template <typename T>
__global__ void __launch_bounds__(64, 4) win_attn_fwd_kernel(const T* qkv, const float* qkv_bias,
                                                          const float* table, T* out, WinGeom g,
                                                          float scale, float p_drop, uint64_t seed0,
                                                          const unsigned long long* seed_dev) {
  const uint64_t seed = launch_seed(seed0, seed_dev);
  constexpr int LD = HD + row_pad<T>();   // [64 x 32] row images
  constexpr int LDP = 64 + row_pad<T>();  // [64 x 64] P
  __shared__ __attribute__((aligned(16))) T sQ[64 * LD];
  __shared__ __attribute__((aligned(16))) T sK[64 * LD];
  __shared__ __attribute__((aligned(16))) T sV[64 * LD];
  __shared__ __attribute__((aligned(16))) T sP[64 * LDP];
  __shared__ int sTok[64], sReg[64];
  const int lane = threadIdx.x;
  const long nitems = g.nwin * g.nh;
  const long C3 = 3L * g.C;
  const bool shifted = (g.sh + g.sw) > 0;
  for (long it = xcd_remap(blockIdx.x, gridDim.x); it < nitems; it += gridDim.x) {
    const long win = it / g.nh;
    const int h = (int)(it - win * g.nh);
    window_tokens(g, win, sTok, sReg, lane);
    __syncthreads();
    stage_rows<T>(sTok, qkv, C3, h * HD, qkv_bias, scale, sQ, LD, lane);
    stage_rows<T>(sTok, qkv, C3, g.C + h * HD, qkv_bias, 1.f, sK, LD, lane);
    stage_rows<T>(sTok, qkv, C3, 2 * g.C + h * HD, qkv_bias, 1.f, sV, LD, lane);
    __syncthreads();
#pragma unroll
    for (int mi = 0; mi < 4; ++mi) {
      f32x4 S[4];
      scores_block<T>(S, mi, sQ, sK, LD, sReg, shifted, table, g.nh, h, lane);
      softmax_block(S);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int i = mi * 16 + (lane >> 4) * 4 + r;
#pragma unroll
        for (int ni = 0; ni < 4; ++ni) {
          const int j = ni * 16 + (lane & 15);
          float pv = S[ni][r];
          if (p_drop > 0.f) pv *= drop_keep(seed, win, h, g.nh, i, j, p_drop);
          sP[i * LDP + j] = from_f32<T>(pv);
        }
      }
    }
    __syncthreads();
#pragma unroll
    for (int mi = 0; mi < 4; ++mi) {
#pragma unroll
      for (int ni = 0; ni < 2; ++ni) {
        f32x4 o = {0.f, 0.f, 0.f, 0.f};
        MM<T, true, false>::k32(o, sP + mi * 16 * LDP, LDP, sV + ni * 16, LD, lane);
        MM<T, true, false>::k32(o, sP + mi * 16 * LDP + 32, LDP, sV + 32 * LD + ni * 16, LD, lane);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int i = mi * 16 + (lane >> 4) * 4 + r;
          const int tok = i < NT ? sTok[i] : -1;
          if (tok >= 0) out[(long)tok * g.C + h * HD + ni * 16 + (lane & 15)] = from_f32<T>(o[r]);
        }
      }
    }
    __syncthreads();
  }
}

// Backward.  Each block owns one head and a strided set of windows; it accumulates the
// relative-position-bias gradient (sum of dS over its windows) and the padded tokens'
// dq/dk/dv (qkv-bias gradient) in registers and writes one partial per block.
template <typename T>
__global__ void __launch_bounds__(64, 2) win_attn_bwd_kernel(
    const T* qkv, const float* qkv_bias, const float* table, const T* dout, T* dqkv,
    float* dbias_part /* [nblk, nh, 49*49] */, float* dqkvb_part /* [nblk, 3C] */,
    WinGeom g, float scale, float p_drop, uint64_t seed0, const unsigned long long* seed_dev, int nblk) {
  const uint64_t seed = launch_seed(seed0, seed_dev);
  constexpr int LD = HD + row_pad<T>();
  constexpr int LDP = 64 + row_pad<T>();
  __shared__ __attribute__((aligned(16))) T sQ[64 * LD];
  __shared__ __attribute__((aligned(16))) T sK[64 * LD];
  __shared__ __attribute__((aligned(16))) T sV[64 * LD];
  __shared__ __attribute__((aligned(16))) T sdO[64 * LD];
  __shared__ __attribute__((aligned(16))) T sPt[64 * LDP];   // (dropped P)^T  [j][i]
  __shared__ __attribute__((aligned(16))) T sdSt[64 * LDP];  // dS^T           [j][i]
  __shared__ int sTok[64], sReg[64];
  const int lane = threadIdx.x;
  const int h = blockIdx.y;
  const long C3 = 3L * g.C;
  const bool shifted = (g.sh + g.sw) > 0;
  f32x4 dB[4][4];
#pragma unroll
  for (int mi = 0; mi < 4; ++mi)
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) dB[mi][ni] = f32x4{0.f, 0.f, 0.f, 0.f};
  // padded tokens' dq/dk/dv for columns ni*16 + (lane&15), summed across lanes at the end
  float padacc[3][2] = {{0.f, 0.f}, {0.f, 0.f}, {0.f, 0.f}};
  for (long win = blockIdx.x; win < g.nwin; win += nblk) {
    window_tokens(g, win, sTok, sReg, lane);
    __syncthreads();
    stage_rows<T>(sTok, qkv, C3, h * HD, qkv_bias, scale, sQ, LD, lane);
    stage_rows<T>(sTok, qkv, C3, g.C + h * HD, qkv_bias, 1.f, sK, LD, lane);
    stage_rows<T>(sTok, qkv, C3, 2 * g.C + h * HD, qkv_bias, 1.f, sV, LD, lane);
    stage_rows<T>(sTok, dout, g.C, h * HD, nullptr, 1.f, sdO, LD, lane);
    __syncthreads();
#pragma unroll
    for (int mi = 0; mi < 4; ++mi) {
      f32x4 P[4], dP[4];
      scores_block<T>(P, mi, sQ, sK, LD, sReg, shifted, table, g.nh, h, lane);
      softmax_block(P);
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) {
        dP[ni] = f32x4{0.f, 0.f, 0.f, 0.f};
        MM<T, true, true>::k32(dP[ni], sdO + mi * 16 * LD, LD, sV + ni * 16 * LD, LD, lane);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int i = mi * 16 + (lane >> 4) * 4 + r;
        float delta = 0.f;
        float keep[4];
#pragma unroll
        for (int ni = 0; ni < 4; ++ni) {
          const int j = ni * 16 + (lane & 15);
          keep[ni] = p_drop > 0.f ? drop_keep(seed, win, h, g.nh, i, j, p_drop) : 1.f;
          sPt[j * LDP + i] = from_f32<T>(P[ni][r] * keep[ni]);
          dP[ni][r] *= keep[ni];
          delta += P[ni][r] * dP[ni][r];
        }
        delta = group_sum<16>(delta);
#pragma unroll
        for (int ni = 0; ni < 4; ++ni) {
          const int j = ni * 16 + (lane & 15);
          const float ds = P[ni][r] * (dP[ni][r] - delta);
          dB[mi][ni][r] += ds;
          sdSt[j * LDP + i] = from_f32<T>(ds);
        }
      }
    }
    __syncthreads();
    // dV = Pd^T dO ; dQs = dS K ; dK = dS^T Qs   (all [64 keys/queries x 32])
#pragma unroll
    for (int mi = 0; mi < 4; ++mi) {
#pragma unroll
      for (int ni = 0; ni < 2; ++ni) {
        f32x4 av = {0.f, 0.f, 0.f, 0.f}, aq = {0.f, 0.f, 0.f, 0.f}, ak = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
          MM<T, true, false>::k32(av, sPt + mi * 16 * LDP + ks * 32, LDP, sdO + ks * 32 * LD + ni * 16, LD, lane);
          MM<T, false, false>::k32(aq, sdSt + ks * 32 * LDP + mi * 16, LDP, sK + ks * 32 * LD + ni * 16, LD, lane);
          MM<T, true, false>::k32(ak, sdSt + mi * 16 * LDP + ks * 32, LDP, sQ + ks * 32 * LD + ni * 16, LD, lane);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int t = mi * 16 + (lane >> 4) * 4 + r;
          if (t < NT) {
            const int tok = sTok[t];
            const int col = h * HD + ni * 16 + (lane & 15);
            if (tok >= 0) {
              T* row = dqkv + (long)tok * C3;
              row[col] = from_f32<T>(aq[r] * scale);
              row[g.C + col] = from_f32<T>(ak[r]);
              row[2 * g.C + col] = from_f32<T>(av[r]);
            } else {
              padacc[0][ni] += aq[r] * scale;
              padacc[1][ni] += ak[r];
              padacc[2][ni] += av[r];
            }
          }
        }
      }
    }
    __syncthreads();
  }
#pragma unroll
  for (int w = 0; w < 3; ++w)
#pragma unroll
    for (int ni = 0; ni < 2; ++ni) {
      float v = padacc[w][ni];
      v += __shfl_xor(v, 16, 64);
      v += __shfl_xor(v, 32, 64);
      if (lane < 16) dqkvb_part[(long)blockIdx.x * C3 + w * g.C + h * HD + ni * 16 + lane] = v;
    }
  float* out = dbias_part + ((long)blockIdx.x * g.nh + h) * (NT * NT);
#pragma unroll
  for (int mi = 0; mi < 4; ++mi)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int i = mi * 16 + (lane >> 4) * 4 + r;
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) {
        const int j = ni * 16 + (lane & 15);
        if (i < NT && j < NT) out[i * NT + j] = dB[mi][ni][r];
      }
    }
}


// dB [nh, 49*49] -> d_table [169, nh]: gather the (i, j) pairs of each relative offset
__global__ void __launch_bounds__(256) rel_table_grad_kernel(const float* dB, int nh, float* dtable,
                                                             int accumulate = 0) {
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= 169 * nh) return;
  const int idx = e / nh, h = e - (e / nh) * nh;
  const int dh = idx / 13 - 6, dw = idx % 13 - 6;
  float s = 0.f;
  for (int ih = 0; ih < WS; ++ih) {
    const int jh = ih - dh;
    if (jh < 0 || jh >= WS) continue;
    for (int iw = 0; iw < WS; ++iw) {
      const int jw = iw - dw;
      if (jw < 0 || jw >= WS) continue;
      s += dB[(long)h * NT * NT + (ih * WS + iw) * NT + jh * WS + jw];
    }
  }
  dtable[e] = accumulate ? dtable[e] + s : s;
}

WinGeom make_geom(int B, int H, int W, int C, int nh, int shift) {
  WinGeom g;
  g.B = B; g.H = H; g.W = W; g.C = C; g.nh = nh;
  g.Hp = H + (WS - H % WS) % WS;
  g.Wp = W + (WS - W % WS) % WS;
  g.nWy = g.Hp / WS; g.nWx = g.Wp / WS;
  g.sh = WS >= g.Hp ? 0 : shift;   // torchvision: no shift when the window covers the map
  g.sw = WS >= g.Wp ? 0 : shift;
  g.nwin = (long)B * g.nWy * g.nWx;
  return g;
}

}  // namespace

// bf16 training path: window_attention_mfma.hip
int msu_attn_mfma_fwd(int dtype, const void* qkv, const float* qkv_bias, const float* table, void* out, int B,
                      int H, int W, int C, int nh, int shift, float p_drop, unsigned long long seed,
                      const unsigned long long* seed_dev, void* keep, float* bias_img, hipStream_t st);
int msu_attn_mfma_bwd(int dtype, const void* qkv, const float* qkv_bias, const float* table, const void* dout,
                      void* dqkv, float* dtable, float* dqkv_bias_pad, float* ws, int B, int H, int W,
                      int C, int nh, int shift, float p_drop, unsigned long long seed,
                      const unsigned long long* seed_dev, const void* keep, hipStream_t st, hipStream_t pst);
long msu_attn_mfma_bwd_workspace(long nwin, int C, int nh);
int msu_attn_mfma_bwd_tail(float* ws, float* dtable, float* dqkv_bias_pad, long nwin, int C, int nh,
                           hipStream_t st, int accumulate = 0);
long msu_attn_mfma_fwd_workspace(int C, int nh);

namespace {
int f32_bwd_blocks(long nwin, int nh) {
  long n = 2048 / nh;
  if (n > nwin) n = nwin;
  return (int)(n < 1 ? 1 : n);
}
}  // namespace

extern "C" {

long msu_win_count(int B, int H, int W) { return make_geom(B, H, W, 32, 1, 0).nwin; }

long msu_win_attn_fwd_workspace(int dtype, int C, int nh) {
  (void)C;
  return msu_is16(dtype) ? msu_attn_mfma_fwd_workspace(C, nh) : 1;
}

long msu_win_attn_keep_words(int dtype, int B, int H, int W, int nh) {
  return msu_is16(dtype) ? make_geom(B, H, W, 32 * nh, nh, 0).nwin * nh * 128 : 0;
}

int msu_win_attn_fwd(int dtype, const void* qkv, const float* qkv_bias, const float* table,
                     void* out, float* workspace, int B, int H, int W, int C, int nh, int shift,
                     float p_drop, unsigned long long seed, const unsigned long long* seed_dev, void* keep,
                     void* stream) {
  if (C != nh * HD) return -2;
  const WinGeom g = make_geom(B, H, W, C, nh, shift);
  // the MFMA kernels address qkv / dqkv rows with 32-bit products tok * 3C
  if ((long)B * H * W * 3 * C >= (1L << 32)) return -2;
  const long items = g.nwin * nh;
  if (items == 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  if (msu_is16(dtype))
    return msu_attn_mfma_fwd(dtype, qkv, qkv_bias, table, out, B, H, W, C, nh, shift, p_drop, seed, seed_dev,
                             keep, workspace, st);
  const float scale = 1.0f / sqrtf((float)HD);
  const long nb = items < 262144 ? items : 262144;
  hipLaunchKernelGGL(win_attn_fwd_kernel<float>, dim3((unsigned)nb), dim3(64), 0, st,
                     (const float*)qkv, qkv_bias, table, (float*)out, g, scale, p_drop, (uint64_t)seed, seed_dev);
  return MSU_CHECK_LAUNCH();
}

long msu_win_attn_bwd_workspace(int dtype, int B, int H, int W, int C, int nh) {
  const WinGeom g = make_geom(B, H, W, C, nh, 0);
  if (msu_is16(dtype)) return msu_attn_mfma_bwd_workspace(g.nwin, C, nh);
  const long nblk = f32_bwd_blocks(g.nwin, nh);
  return nblk * nh * NT * NT + (long)nh * NT * NT + nblk * 3 * C;
}

int msu_win_attn_bwd_tail(int dtype, float* workspace, float* dtable, float* dqkv_bias_pad, int B, int H, int W,
                          int C, int nh, void* stream);

int msu_win_attn_bwd2(int dtype, const void* qkv, const float* qkv_bias, const float* table,
                      const void* dout, void* dqkv, float* dtable, float* dqkv_bias_pad,
                      float* workspace, int B, int H, int W, int C, int nh, int shift,
                      float p_drop, unsigned long long seed, const unsigned long long* seed_dev, const void* keep,
                      void* stream, void* param_stream) {
  if (C != nh * HD) return -2;
  // the MFMA kernels address qkv / dqkv rows with 32-bit products tok * 3C
  if ((long)B * H * W * 3 * C >= (1L << 32)) return -2;
  const WinGeom g = make_geom(B, H, W, C, nh, shift);
  hipStream_t st = (hipStream_t)stream;
  hipStream_t pst = (hipStream_t)param_stream;
  if (g.nwin == 0) return 0;
  if (msu_is16(dtype))
    return msu_attn_mfma_bwd(dtype, qkv, qkv_bias, table, dout, dqkv, dtable, dqkv_bias_pad, workspace, B, H, W,
                             C, nh, shift, p_drop, seed, seed_dev, keep, st, pst);
  if (table == nullptr) return -2;  // the f32 kernel reads the table itself
  const int nblk = f32_bwd_blocks(g.nwin, nh);
  const float scale = 1.0f / sqrtf((float)HD);
  float* dB_part = workspace;
  float* dB = dB_part + (long)nblk * nh * NT * NT;
  float* qb_part = dB + (long)nh * NT * NT;
  hipLaunchKernelGGL(win_attn_bwd_kernel<float>, dim3(nblk, nh), dim3(64), 0, st,
                     (const float*)qkv, qkv_bias, table, (const float*)dout, (float*)dqkv,
                     dB_part, qb_part, g, scale, p_drop, (uint64_t)seed, seed_dev, nblk);
  if (pst == (hipStream_t)(intptr_t)-1) return MSU_CHECK_LAUNCH();  // tail issued by the caller
  const int rc = attn_param_stream(st, pst);
  if (rc) return rc;
  return msu_win_attn_bwd_tail(dtype, workspace, dtable, dqkv_bias_pad, B, H, W, C, nh, pst);
}

int msu_win_attn_bwd_tail2(int dtype, float* workspace, float* dtable, float* dqkv_bias_pad, int B, int H, int W,
                           int C, int nh, int accumulate, void* stream) {
  if (C != nh * HD) return -2;
  const WinGeom g = make_geom(B, H, W, C, nh, 0);
  hipStream_t st = (hipStream_t)stream;
  if (g.nwin == 0) return 0;
  if (msu_is16(dtype)) return msu_attn_mfma_bwd_tail(workspace, dtable, dqkv_bias_pad, g.nwin, C, nh, st, accumulate);
  const int nblk = f32_bwd_blocks(g.nwin, nh);
  float* dB_part = workspace;
  float* dB = dB_part + (long)nblk * nh * NT * NT;
  float* qb_part = dB + (long)nh * NT * NT;
  const long nB = (long)nh * NT * NT;
  colsum(dB_part, nblk, nB, nB, dB, 0, st);
  hipLaunchKernelGGL(rel_table_grad_kernel, dim3((169 * nh + 255) / 256), dim3(256), 0, st, dB, nh, dtable,
                     accumulate);
  colsum(qb_part, nblk, 3L * C, 3L * C, dqkv_bias_pad, accumulate, st);
  return MSU_CHECK_LAUNCH();
}

int msu_win_attn_bwd_tail(int dtype, float* workspace, float* dtable, float* dqkv_bias_pad, int B, int H, int W,
                          int C, int nh, void* stream) {
  return msu_win_attn_bwd_tail2(dtype, workspace, dtable, dqkv_bias_pad, B, H, W, C, nh, 0, stream);
}

int msu_win_attn_bwd(int dtype, const void* qkv, const float* qkv_bias, const float* table,
                     const void* dout, void* dqkv, float* dtable, float* dqkv_bias_pad,
                     float* workspace, int B, int H, int W, int C, int nh, int shift,
                     float p_drop, unsigned long long seed, const unsigned long long* seed_dev, const void* keep,
                     void* stream) {
  return msu_win_attn_bwd2(dtype, qkv, qkv_bias, table, dout, dqkv, dtable, dqkv_bias_pad, workspace, B, H, W,
                           C, nh, shift, p_drop, seed, seed_dev, keep, stream, nullptr);
}

}  // extern "C"
