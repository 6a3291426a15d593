// bf16 shifted-window attention on 32x32x16 MFMA, scores kept TRANSPOSED (keys on the
// accumulator rows, queries on the lanes) -- the training-mode fast path of
// msu_win_attn_fwd / msu_win_attn_bwd (torchvision shifted_window_attention semantics, see
// window_attention.hip for the pad / roll / partition folding and the f32 parity kernel).
//
// Per (window, head) item, one wave:
//   S^T[j][i] = K Q^T + B_rel^T (+ -100 shift mask)   8 x v_mfma_f32_32x32x16_bf16, the
//              accumulators start from a per-head bias image laid out in the MFMA C layout
//              (-inf on padded key rows), so the bias add costs nothing;
//   softmax over j: each lane owns one query column -> in-register max/sum + one xor-32
//              shuffle; dropout by a counter hash;
//   O^T[d][i] = V^T P^T: P^T stays in registers and is the B operand directly (sum over
//              the accumulator's row index); V^T comes from the staged V rows with
//              ds_read_b64_tr_b16 in the matching permuted k order.
// Backward recomputes S^T / P^T, forms dP^T = V dO^T, dS^T = P^T (dP^T - delta), stores
// Pd and dS once as [i][j] LDS images (8-byte stores) and runs dV = Pd^T dO,
// dQ = dS K, dK = dS^T Q with tr-read operands; relative-bias gradients accumulate in
// registers in the bias-image layout; padded tokens' dq/dk/dv go to the qkv-bias partial.
#include "common.h"
#include "reduce.h"

namespace {

constexpr int WS = 7, NT = 49, HD = 32;
constexpr int LD = 40;   // staged [64 x 32] rows: 32 + 8 pad (80 B)
constexpr int LDP = 72;  // [64 x 64] images: 64 + 8 pad (144 B)

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef short v4s __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) v4s lds_v4s;

struct Geom {
  int B, H, W, Hp, Wp, nWy, nWx, sh, sw, C, nh;
  long nwin;
};

MSU_DEV f32x16 mfma32(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

// row-major k-contiguous fragment: lane l -> row (l&31), k = k0 + 8(l>>5) .. +7
MSU_DEV bf16x8 frag_rows(const bf16_t* base, int ld, int row0, int k0, int lane) {
  return *reinterpret_cast<const bf16x8*>(base + (row0 + (lane & 31)) * ld + k0 + 8 * (lane >> 5));
}

MSU_DEV v4s tr_read(const bf16_t* p) { return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)p); }

// k-strided fragment from a [k rows][cols] image: lane l -> col col0 + (l&31),
// element e -> row r0 + 8(l>>5) + e  (natural k order)
MSU_DEV bf16x8 frag_tr(const bf16_t* img, int ld, int r0, int col0, int lane) {
  const int g = lane >> 4, li = lane & 15, q = li >> 2, p = li & 3, h = lane >> 5;
  const int col = col0 + 16 * (g & 1) + 4 * p;
  v4s both[2] = {tr_read(img + (r0 + 8 * h + q) * ld + col), tr_read(img + (r0 + 8 * h + 4 + q) * ld + col)};
  return *reinterpret_cast<bf16x8*>(both);
}

// same, in the permuted k order of an accumulator used as the other operand:
// element e of lane half h -> row r0 + 8(e>>2) + 4h + (e&3)
MSU_DEV bf16x8 frag_tr_perm(const bf16_t* img, int ld, int r0, int col0, int lane) {
  const int g = lane >> 4, li = lane & 15, q = li >> 2, p = li & 3, h = lane >> 5;
  const int col = col0 + 16 * (g & 1) + 4 * p;
  v4s both[2] = {tr_read(img + (r0 + 4 * h + q) * ld + col), tr_read(img + (r0 + 8 + 4 * h + q) * ld + col)};
  return *reinterpret_cast<bf16x8*>(both);
}

// accumulator registers 8s..8s+7 -> bf16 fragment
MSU_DEV bf16x8 pack8(const f32x16& a, int s) {
  bf16x8 f;
#pragma unroll
  for (int e = 0; e < 8; ++e) f[e] = (__bf16)a[8 * s + e];
  return f;
}

// accumulator row of register r for lane half h (32x32 C layout)
MSU_DEV constexpr int crow(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

MSU_DEV int region(int p, int P, int s) { return s == 0 ? 0 : (p < P - WS ? 0 : (p < P - s ? 1 : 2)); }

struct WinInfo {
  bool boundary;  // window touches the shifted wrap-around (mask non-trivial)
};

// Token table of the window (sTok: source token or -1 = padded, sReg: mask region)
MSU_DEV WinInfo window_tokens(const Geom& g, long win, int* sTok, int* sReg, int lane) {
  const int nw = g.nWy * g.nWx;
  const long b = win / nw;
  const int wr = (int)(win - b * nw);
  const int wy = wr / g.nWx, wx = wr - (wr / g.nWx) * g.nWx;
  int tok = -1, reg = 0;
  if (lane < NT) {
    const int py = wy * WS + lane / WS, px = wx * WS + lane % WS;
    int sy = py + g.sh; if (sy >= g.Hp) sy -= g.Hp;
    int sx = px + g.sw; if (sx >= g.Wp) sx -= g.Wp;
    if (sy < g.H && sx < g.W) tok = (int)((b * g.H + sy) * (long)g.W + sx);
    reg = region(py, g.Hp, g.sh) * 3 + region(px, g.Wp, g.sw);
  }
  sTok[lane] = tok;
  sReg[lane] = reg;
  WinInfo w;
  w.boundary = (g.sh + g.sw) > 0 && (wy == g.nWy - 1 || wx == g.nWx - 1);
  return w;
}

// stage rows t < 49 of a head slice (32 bf16 = 4 x 16 B) into sX[t][LD]; rows >= 49 zero.
// Padded tokens take the bf16-rounded bias (or zero when bias == nullptr).
MSU_DEV void stage(const int* sTok, const bf16_t* src, long stride, int col0, const float* bias,
                   float mul, bf16_t* sX, int lane) {
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const int idx = lane + 64 * c;
    const int t = idx >> 2, q = idx & 3;
    uint4 v = make_uint4(0, 0, 0, 0);
    if (t < NT) {
      const int tok = sTok[t];
      float f[8];
      if (tok >= 0) {
        const uint4 raw = *reinterpret_cast<const uint4*>(src + (long)tok * stride + col0 + q * 8);
        const uint32_t w[4] = {raw.x, raw.y, raw.z, raw.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          f[2 * e] = __uint_as_float(w[e] << 16);
          f[2 * e + 1] = __uint_as_float(w[e] & 0xffff0000u);
        }
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) f[e] = bias ? to_f32(from_f32<bf16_t>(bias[col0 + q * 8 + e])) : 0.f;
      }
      if (mul != 1.f) {
#pragma unroll
        for (int e = 0; e < 8; ++e) f[e] *= mul;
      }
      v.x = (uint32_t)from_f32<bf16_t>(f[0]) | ((uint32_t)from_f32<bf16_t>(f[1]) << 16);
      v.y = (uint32_t)from_f32<bf16_t>(f[2]) | ((uint32_t)from_f32<bf16_t>(f[3]) << 16);
      v.z = (uint32_t)from_f32<bf16_t>(f[4]) | ((uint32_t)from_f32<bf16_t>(f[5]) << 16);
      v.w = (uint32_t)from_f32<bf16_t>(f[6]) | ((uint32_t)from_f32<bf16_t>(f[7]) << 16);
    }
    *reinterpret_cast<uint4*>(sX + t * LD + q * 8) = v;
  }
}

MSU_DEV float drop_keep(uint64_t seed, long win, int h, int nh, int i, int j, float p) {
  const uint64_t idx = ((((uint64_t)win * nh + h) * 64 + i) * 64 + j);
  return hash_uniform(seed, idx) >= p ? 1.0f / (1.0f - p) : 0.0f;
}

// S^T tiles (jt, it) of one item, bias-initialised, masked, softmax-ed over j -> P^T
MSU_DEV void probs_T(f32x16 (&P)[2][2], const bf16_t* sQ, const bf16_t* sK, const float* bimg,
                     const int* sReg, bool boundary, int lane) {
#pragma unroll
  for (int jt = 0; jt < 2; ++jt)
#pragma unroll
    for (int it = 0; it < 2; ++it) {
      const float4* bp = reinterpret_cast<const float4*>(bimg + ((jt * 2 + it) * 64 + lane) * 16);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float4 v = bp[q];
        P[jt][it][4 * q] = v.x; P[jt][it][4 * q + 1] = v.y; P[jt][it][4 * q + 2] = v.z; P[jt][it][4 * q + 3] = v.w;
      }
    }
#pragma unroll
  for (int ks = 0; ks < HD; ks += 16) {
    bf16x8 a[2], b[2];
#pragma unroll
    for (int jt = 0; jt < 2; ++jt) a[jt] = frag_rows(sK, LD, jt * 32, ks, lane);
#pragma unroll
    for (int it = 0; it < 2; ++it) b[it] = frag_rows(sQ, LD, it * 32, ks, lane);
#pragma unroll
    for (int jt = 0; jt < 2; ++jt)
#pragma unroll
      for (int it = 0; it < 2; ++it) P[jt][it] = mfma32(a[jt], b[it], P[jt][it]);
  }
  const int h = lane >> 5;
  if (boundary) {
#pragma unroll
    for (int it = 0; it < 2; ++it) {
      const int i = it * 32 + (lane & 31);
      const int ri = sReg[i];
#pragma unroll
      for (int jt = 0; jt < 2; ++jt)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int j = jt * 32 + crow(r, h);
          if (sReg[j] != ri) P[jt][it][r] += -100.0f;
        }
    }
  }
#pragma unroll
  for (int it = 0; it < 2; ++it) {
    float m = -INFINITY;
#pragma unroll
    for (int jt = 0; jt < 2; ++jt)
#pragma unroll
      for (int r = 0; r < 16; ++r) m = fmaxf(m, P[jt][it][r]);
    m = fmaxf(m, __shfl_xor(m, 32, 64));
    float s = 0.f;
#pragma unroll
    for (int jt = 0; jt < 2; ++jt)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float e = __expf(P[jt][it][r] - m);
        P[jt][it][r] = e;
        s += e;
      }
    s += __shfl_xor(s, 32, 64);
    const float inv = 1.0f / s;
#pragma unroll
    for (int jt = 0; jt < 2; ++jt)
#pragma unroll
      for (int r = 0; r < 16; ++r) P[jt][it][r] *= inv;
  }
}

struct FwdLds {
  bf16_t q[64 * LD], k[64 * LD], v[64 * LD];
  int tok[64], reg[64];
};

template <int WAVES>
__global__ void __launch_bounds__(64 * WAVES, 2) attn_fwd_mfma(const bf16_t* __restrict__ qkv,
                                                            const float* __restrict__ qkv_bias,
                                                            const float* __restrict__ bimg_all,
                                                            bf16_t* __restrict__ out, Geom g,
                                                            float scale, float p_drop, uint64_t seed) {
  __shared__ __attribute__((aligned(16))) FwdLds lds_all[WAVES];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  FwdLds& L = lds_all[wave];
  const long nitems = g.nwin * g.nh;
  const long C3 = 3L * g.C;
  const long nblk = gridDim.x;
  const long b0 = xcd_remap(blockIdx.x, gridDim.x);
  for (long it0 = b0 * WAVES; it0 < nitems; it0 += nblk * WAVES) {
    const long item = it0 + wave;
    if (item >= nitems) break;  // no block-wide barriers below: waves are independent
    const long win = item / g.nh;
    const int h = (int)(item - win * g.nh);
    const WinInfo wi = window_tokens(g, win, L.tok, L.reg, lane);
    stage(L.tok, qkv, C3, h * HD, qkv_bias, scale, L.q, lane);
    stage(L.tok, qkv, C3, g.C + h * HD, qkv_bias, 1.f, L.k, lane);
    stage(L.tok, qkv, C3, 2 * g.C + h * HD, qkv_bias, 1.f, L.v, lane);
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): LDS writes of this wave done
    __builtin_amdgcn_wave_barrier();
    f32x16 P[2][2];
    probs_T(P, L.q, L.k, bimg_all + (long)h * 4 * 64 * 16, L.reg, wi.boundary, lane);
    const int hh = lane >> 5;
    if (p_drop > 0.f) {
#pragma unroll
      for (int jt = 0; jt < 2; ++jt)
#pragma unroll
        for (int it = 0; it < 2; ++it)
#pragma unroll
          for (int r = 0; r < 16; ++r)
            P[jt][it][r] *= drop_keep(seed, win, h, g.nh, it * 32 + (lane & 31), jt * 32 + crow(r, hh), p_drop);
    }
    // O^T[d][i] = sum_j V[j][d] P^T[j][i]
    f32x16 O[2];
    O[0] = f32x16{0}; O[1] = f32x16{0};
#pragma unroll
    for (int jt = 0; jt < 2; ++jt)
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const bf16x8 a = frag_tr_perm(L.v, LD, jt * 32 + 16 * s, 0, lane);
#pragma unroll
        for (int it = 0; it < 2; ++it) O[it] = mfma32(a, pack8(P[jt][it], s), O[it]);
      }
    // store: lane -> query i, registers 4g..4g+3 -> d = 8g + 4hh .. +3 (8-byte stores)
#pragma unroll
    for (int it = 0; it < 2; ++it) {
      const int i = it * 32 + (lane & 31);
      const int tok = i < NT ? L.tok[i] : -1;
      if (tok >= 0) {
        bf16_t* dst = out + (long)tok * g.C + h * HD;
#pragma unroll
        for (int gq = 0; gq < 4; ++gq) {
          uint2 w;
          w.x = (uint32_t)from_f32<bf16_t>(O[it][4 * gq]) | ((uint32_t)from_f32<bf16_t>(O[it][4 * gq + 1]) << 16);
          w.y = (uint32_t)from_f32<bf16_t>(O[it][4 * gq + 2]) | ((uint32_t)from_f32<bf16_t>(O[it][4 * gq + 3]) << 16);
          *reinterpret_cast<uint2*>(dst + 8 * gq + 4 * hh) = w;
        }
      }
    }
    __builtin_amdgcn_wave_barrier();
  }
}

struct BwdLds {
  bf16_t q[64 * LD], k[64 * LD], v[64 * LD], dO[64 * LD];
  bf16_t P[64 * LDP], dS[64 * LDP];  // [i][j] images
  int tok[64], reg[64];
};

template <int WAVES>
__global__ void __launch_bounds__(64 * WAVES) attn_bwd_mfma(
    const bf16_t* __restrict__ qkv, const float* __restrict__ qkv_bias, const float* __restrict__ bimg_all,
    const bf16_t* __restrict__ dout, bf16_t* __restrict__ dqkv, float* __restrict__ dB_part,
    float* __restrict__ qb_part, Geom g, float scale, float p_drop, uint64_t seed, int nblk) {
  // grid (nblk, nh): block owns head h, waves walk windows win = (blk*WAVES + wave) + k*nblk*WAVES
  __shared__ __attribute__((aligned(16))) BwdLds lds_all[WAVES];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  BwdLds& L = lds_all[wave];
  const int h = blockIdx.y;
  const long C3 = 3L * g.C;
  const int hh = lane >> 5;
  const float* bimg = bimg_all + (long)h * 4 * 64 * 16;
  f32x16 dB[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) dB[a][b] = f32x16{0};
  float padacc[3] = {0.f, 0.f, 0.f};  // column d = lane&31 of padded tokens' dq, dk, dv (per half)
  const long stride = (long)nblk * WAVES;
  for (long win = (long)blockIdx.x * WAVES + wave; win < g.nwin; win += stride) {
    const WinInfo wi = window_tokens(g, win, L.tok, L.reg, lane);
    stage(L.tok, qkv, C3, h * HD, qkv_bias, scale, L.q, lane);
    stage(L.tok, qkv, C3, g.C + h * HD, qkv_bias, 1.f, L.k, lane);
    stage(L.tok, qkv, C3, 2 * g.C + h * HD, qkv_bias, 1.f, L.v, lane);
    stage(L.tok, dout, g.C, h * HD, nullptr, 1.f, L.dO, lane);
    __builtin_amdgcn_s_waitcnt(0xc07f);
    __builtin_amdgcn_wave_barrier();
    f32x16 P[2][2];
    probs_T(P, L.q, L.k, bimg, L.reg, wi.boundary, lane);
    // dPd^T[j][i] = sum_d V[j][d] dO[i][d]
    f32x16 D[2][2];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b) D[a][b] = f32x16{0};
#pragma unroll
    for (int ks = 0; ks < HD; ks += 16) {
      bf16x8 a[2], b[2];
#pragma unroll
      for (int jt = 0; jt < 2; ++jt) a[jt] = frag_rows(L.v, LD, jt * 32, ks, lane);
#pragma unroll
      for (int it = 0; it < 2; ++it) b[it] = frag_rows(L.dO, LD, it * 32, ks, lane);
#pragma unroll
      for (int jt = 0; jt < 2; ++jt)
#pragma unroll
        for (int it = 0; it < 2; ++it) D[jt][it] = mfma32(a[jt], b[it], D[jt][it]);
    }
#pragma unroll
    for (int it = 0; it < 2; ++it) {
      const int i = it * 32 + (lane & 31);
      float delta = 0.f;
#pragma unroll
      for (int jt = 0; jt < 2; ++jt)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          float keep = 1.f;
          if (p_drop > 0.f) keep = drop_keep(seed, win, h, g.nh, i, jt * 32 + crow(r, hh), p_drop);
          D[jt][it][r] *= keep;                  // dP = dPd * keep/(1-p)
          delta += P[jt][it][r] * D[jt][it][r];
          if (p_drop > 0.f) D[jt][it][r] = D[jt][it][r];  // keep in D; Pd written below
        }
      delta += __shfl_xor(delta, 32, 64);
      // Pd (dropped probabilities) and dS images [i][j], 4 consecutive j per 8-byte store
#pragma unroll
      for (int jt = 0; jt < 2; ++jt)
#pragma unroll
        for (int gq = 0; gq < 4; ++gq) {
          float pd[4], ds[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int r = 4 * gq + e;
            const float p = P[jt][it][r];
            const float dsv = p * (D[jt][it][r] - delta);
            float keep = 1.f;
            if (p_drop > 0.f) keep = drop_keep(seed, win, h, g.nh, i, jt * 32 + crow(r, hh), p_drop);
            pd[e] = p * keep;
            ds[e] = dsv;
            dB[jt][it][r] += dsv;
          }
          const int j0 = jt * 32 + 8 * gq + 4 * hh;
          uint2 wp, wd;
          wp.x = (uint32_t)from_f32<bf16_t>(pd[0]) | ((uint32_t)from_f32<bf16_t>(pd[1]) << 16);
          wp.y = (uint32_t)from_f32<bf16_t>(pd[2]) | ((uint32_t)from_f32<bf16_t>(pd[3]) << 16);
          wd.x = (uint32_t)from_f32<bf16_t>(ds[0]) | ((uint32_t)from_f32<bf16_t>(ds[1]) << 16);
          wd.y = (uint32_t)from_f32<bf16_t>(ds[2]) | ((uint32_t)from_f32<bf16_t>(ds[3]) << 16);
          *reinterpret_cast<uint2*>(L.P + i * LDP + j0) = wp;
          *reinterpret_cast<uint2*>(L.dS + i * LDP + j0) = wd;
        }
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);
    __builtin_amdgcn_wave_barrier();
    // dV[j][d] = sum_i Pd[i][j] dO[i][d]; dK[j][d] = sum_i dS[i][j] Q[i][d]; dQ[i][d] = sum_j dS[i][j] K[j][d]
#pragma unroll
    for (int mt = 0; mt < 2; ++mt) {
      f32x16 av = f32x16{0}, ak = f32x16{0}, aq = f32x16{0};
#pragma unroll
      for (int ks = 0; ks < 64; ks += 16) {
        const bf16x8 bdo = frag_tr(L.dO, LD, ks, 0, lane);
        const bf16x8 bq = frag_tr(L.q, LD, ks, 0, lane);
        const bf16x8 bk = frag_tr(L.k, LD, ks, 0, lane);
        av = mfma32(frag_tr(L.P, LDP, ks, mt * 32, lane), bdo, av);
        ak = mfma32(frag_tr(L.dS, LDP, ks, mt * 32, lane), bq, ak);
        aq = mfma32(frag_rows(L.dS, LDP, mt * 32, ks, lane), bk, aq);
      }
      // rows t = mt*32 + crow(r, hh), column d = lane & 31
      const int d = lane & 31;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int t = mt * 32 + crow(r, hh);
        if (t < NT) {
          const int tok = L.tok[t];
          if (tok >= 0) {
            bf16_t* row = dqkv + (long)tok * C3 + h * HD + d;
            row[0] = from_f32<bf16_t>(aq[r] * scale);
            row[g.C] = from_f32<bf16_t>(ak[r]);
            row[2 * g.C] = from_f32<bf16_t>(av[r]);
          } else {
            padacc[0] += aq[r] * scale;
            padacc[1] += ak[r];
            padacc[2] += av[r];
          }
        }
      }
    }
    __builtin_amdgcn_wave_barrier();
  }
  // per-wave partials: relative-bias gradient image [part][h][4 tiles][64 lanes][16]
  const long part = (long)blockIdx.x * WAVES + wave;
  float* db = dB_part + (part * g.nh + h) * (4 * 64 * 16);
#pragma unroll
  for (int jt = 0; jt < 2; ++jt)
#pragma unroll
    for (int it = 0; it < 2; ++it) {
      float4* dst = reinterpret_cast<float4*>(db + ((jt * 2 + it) * 64 + lane) * 16);
#pragma unroll
      for (int q = 0; q < 4; ++q)
        dst[q] = make_float4(dB[jt][it][4 * q], dB[jt][it][4 * q + 1], dB[jt][it][4 * q + 2], dB[jt][it][4 * q + 3]);
    }
#pragma unroll
  for (int w = 0; w < 3; ++w) {
    const float v = padacc[w] + __shfl_xor(padacc[w], 32, 64);
    if (lane < 32) qb_part[part * C3 + w * g.C + h * HD + lane] = v;
  }
}

// bias image [nh][4 tiles (jt*2+it)][64 lanes][16 regs]: value for (j, i) = table[idx(i,j)][h]
// (i, j < 49), -inf for padded keys j >= 49, 0 for padded queries i >= 49.
__global__ void __launch_bounds__(256) bias_image_kernel(const float* table, int nh, float* img) {
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= nh * 4096) return;
  const int h = e / 4096, rem = e % 4096;
  const int t = rem / 1024, lane = (rem / 16) % 64, r = rem % 16;
  const int jt = t >> 1, it = t & 1;
  const int j = jt * 32 + crow(r, lane >> 5), i = it * 32 + (lane & 31);
  float v;
  if (j >= NT) v = -INFINITY;
  else if (i >= NT) v = 0.f;
  else v = table[((i / WS - j / WS + WS - 1) * (2 * WS - 1) + (i % WS - j % WS + WS - 1)) * nh + h];
  img[e] = v;
}

// d bias image [nh][4096] -> d table [169][nh]
__global__ void __launch_bounds__(256) bias_image_grad_kernel(const float* dimg, int nh, float* dtable) {
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
      const int i = ih * WS + iw, j = jh * WS + jw;
      const int jt = j >> 5, it = i >> 5, jj = j & 31;
      const int hh = (jj >> 2) & 1, r = (jj & 3) + 4 * (jj >> 3);
      const int lane = (i & 31) + 32 * hh;
      s += dimg[(long)h * 4096 + ((jt * 2 + it) * 64 + lane) * 16 + r];
    }
  }
  dtable[e] = s;
}

Geom make_geom(int B, int H, int W, int C, int nh, int shift) {
  Geom g;
  g.B = B; g.H = H; g.W = W; g.C = C; g.nh = nh;
  g.Hp = H + (WS - H % WS) % WS;
  g.Wp = W + (WS - W % WS) % WS;
  g.nWy = g.Hp / WS; g.nWx = g.Wp / WS;
  g.sh = WS >= g.Hp ? 0 : shift;
  g.sw = WS >= g.Wp ? 0 : shift;
  g.nwin = (long)B * g.nWy * g.nWx;
  return g;
}

constexpr int FWD_WAVES = 4, BWD_WAVES = 2;

}  // namespace

// entry points used by window_attention.hip for dtype == bf16
int msu_attn_mfma_bwd_parts(long nwin, int nh) {
  // per head: waves = nblk * BWD_WAVES, aim for ~2048 waves in total
  long nblk = 1024 / ((long)nh * BWD_WAVES);
  if (nblk < 1) nblk = 1;
  const long maxb = (nwin + BWD_WAVES - 1) / BWD_WAVES;
  if (nblk > maxb) nblk = maxb;
  return (int)nblk;
}

long msu_attn_mfma_bwd_workspace(long nwin, int C, int nh) {
  const long parts = (long)msu_attn_mfma_bwd_parts(nwin, nh) * BWD_WAVES;
  return parts * nh * 4096 + (long)nh * 4096 * 2 + parts * 3L * C;
}

int msu_attn_mfma_fwd(const void* qkv, const float* qkv_bias, const float* table, void* out, int B,
                      int H, int W, int C, int nh, int shift, float p_drop, unsigned long long seed,
                      float* bias_img, hipStream_t st) {
  const Geom g = make_geom(B, H, W, C, nh, shift);
  const long items = g.nwin * nh;
  if (items == 0) return 0;
  hipLaunchKernelGGL(bias_image_kernel, dim3((nh * 4096 + 255) / 256), dim3(256), 0, st, table, nh, bias_img);
  long nb = (items + FWD_WAVES - 1) / FWD_WAVES;
  if (nb > 65536) nb = 65536;
  hipLaunchKernelGGL(attn_fwd_mfma<FWD_WAVES>, dim3((unsigned)nb), dim3(64 * FWD_WAVES), 0, st,
                     (const bf16_t*)qkv, qkv_bias, bias_img, (bf16_t*)out, g, 1.0f / sqrtf((float)HD),
                     p_drop, (uint64_t)seed);
  return MSU_CHECK_LAUNCH();
}

int msu_attn_mfma_bwd(const void* qkv, const float* qkv_bias, const float* table, const void* dout,
                      void* dqkv, float* dtable, float* dqkv_bias_pad, float* ws, int B, int H, int W,
                      int C, int nh, int shift, float p_drop, unsigned long long seed, hipStream_t st) {
  const Geom g = make_geom(B, H, W, C, nh, shift);
  if (g.nwin == 0) return 0;
  const int nblk = msu_attn_mfma_bwd_parts(g.nwin, nh);
  const long parts = (long)nblk * BWD_WAVES;
  float* dB_part = ws;
  float* img = dB_part + parts * nh * 4096;
  float* dimg = img + (long)nh * 4096;
  float* qb_part = dimg + (long)nh * 4096;
  hipLaunchKernelGGL(bias_image_kernel, dim3((nh * 4096 + 255) / 256), dim3(256), 0, st, table, nh, img);
  hipLaunchKernelGGL(attn_bwd_mfma<BWD_WAVES>, dim3(nblk, nh), dim3(64 * BWD_WAVES), 0, st,
                     (const bf16_t*)qkv, qkv_bias, img, (const bf16_t*)dout, (bf16_t*)dqkv, dB_part, qb_part,
                     g, 1.0f / sqrtf((float)HD), p_drop, (uint64_t)seed, nblk);
  colsum(dB_part, (int)parts, (long)nh * 4096, (long)nh * 4096, dimg, 0, st);
  hipLaunchKernelGGL(bias_image_grad_kernel, dim3((169 * nh + 255) / 256), dim3(256), 0, st, dimg, nh, dtable);
  colsum(qb_part, (int)parts, 3L * C, 3L * C, dqkv_bias_pad, 0, st);
  return MSU_CHECK_LAUNCH();
}
