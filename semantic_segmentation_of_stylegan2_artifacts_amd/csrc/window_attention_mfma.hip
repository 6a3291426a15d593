// 16-bit (bf16 / f16) shifted-window attention on 32x32x16 MFMA, scores kept TRANSPOSED (keys on the
// accumulator rows, queries on the lanes) -- the training-mode fast path of
// msu_win_attn_fwd / msu_win_attn_bwd (torchvision shifted_window_attention semantics, see
// window_attention.hip for the pad / roll / partition folding and the f32 parity kernel).
//
// Per (window, head) item, one wave:
//   S^T[j][i] = K Q^T (+ B_rel^T / scale, + -100/scale shift mask); softmax uses
//              exp(scale * (s - max)), i.e. q * hd^-1/2 is folded into the exponent.  The
//              accumulators start from a per-head bias image laid out in the MFMA C layout
//              (-inf on padded key rows), so the bias add costs nothing.  K and Q operand
//              fragments are loaded straight from HBM (one 16-B load per lane each);
//   softmax over j: each lane owns one query column -> in-register max/sum + one xor-32
//              shuffle; dropout by a counter hash;
//   O^T[d][i] = V^T P^T: P^T stays in registers and is the B operand directly (sum over
//              the accumulator's row index); V^T comes from the staged V rows with
//              ds_read_b64_tr_b16 in the matching permuted k order.
// All global loads of an item are issued together before first use (the HBM latency is
// paid once per item, not once per row).
// Backward recomputes S^T / P^T, forms dP^T = V dO^T, dS^T = P^T (dP^T - delta), stores
// Pd and dS once as [i][j] LDS images (8-byte stores) and runs dV^T = dO^T Pd,
// dQ^T = K^T dS^T, dK^T = Q^T dS with tr-read operands, the token index on the accumulator
// columns so that every lane stores whole 16-B pieces of its token's rows; relative-bias
// gradients accumulate in registers in the bias-image layout; padded tokens' dq/dk/dv go
// to the qkv-bias partial.
#include <type_traits>
#include <utility>

#include "common.h"
#include "reduce.h"

// MSU_EXP: ablation bits for timing experiments only (tools/build_exp.sh); 0 in every real build
#ifndef MSU_EXP
#define MSU_EXP 0
#endif

namespace {

template <typename F, int... Is>
MSU_DEV void static_for(F&& f, std::integer_sequence<int, Is...>) {
  (f(std::integral_constant<int, Is>{}), ...);
}

constexpr int WS = 7, NT = 49, HD = 32;
constexpr int LD = 40;   // staged [64 x 32] rows: 32 + 8 pad (80 B)
constexpr int LDP = 72;  // [64 x 64] images: 64 + 8 pad (144 B)
constexpr int TOK_PAD = -1, TOK_ZERO = -2;

typedef short v4s __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) v4s lds_v4s;

struct Geom {
  int B, H, W, Hp, Wp, nWy, nWx, sh, sw, C, nh;
  long nwin;
};

// T (bf16_t / f16_t): the 16-bit format of the raw words stored in qkv / dout / LDS
template <typename T>
MSU_DEV f32x16 mfma32(bf16x8 a, bf16x8 b, f32x16 c) {
  return Fmt16<T>::mma32(a, b, c);
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

// k-strided fragment in the bank-spread k order: element e of lane half h -> row
// r0 + 4(e&3) + 2h + (e>>2).  Each half-wave's tr read then covers rows 4 apart, whose
// 64-B column runs start 16 dwords apart for row strides of 20 and 36 dwords (LD, LDP):
// all 64 banks once (natural order: 4 consecutive rows, 2-way conflicts).  Only for
// products whose other operand is read the same way.
MSU_DEV bf16x8 frag_tr_q4(const bf16_t* img, int ld, int r0, int col0, int lane) {
  const int g = lane >> 4, li = lane & 15, q = li >> 2, p = li & 3, h = lane >> 5;
  const int col = col0 + 16 * (g & 1) + 4 * p;
  const int row = r0 + 4 * q + 2 * h;
  v4s both[2] = {tr_read(img + row * ld + col), tr_read(img + (row + 1) * ld + col)};
  return *reinterpret_cast<bf16x8*>(both);
}

// Row of a 16-row block staged by lane quad qd = lane >> 2 (4 lanes x 16 B per 64-B row).
// ds_write_b128 banks 8 consecutive lanes (two quads) on (a/4) mod 32: at the 20-dword row
// stride rows r and r + 4 fill disjoint banks, r and r + 1 overlap (2-way), so quads 2k, 2k + 1
// take rows k', k' + 4.
MSU_DEV constexpr int stage_row(int qd) { return ((qd & 1) << 2) | ((qd >> 1) & 3) | (qd & 8); }
// Same for ds_read_b128 of staged rows (lane groups {0-3, 12-15, 20-27}, ... on (a/4) mod 64):
// a group's four quads take rows a, a + 4, a + 8, a + 12.
MSU_DEV int read_row(int qd) { return (int)((0xfeab6732dc894510ull >> (4 * qd)) & 15); }

// frag_tr_q4 on an image whose rows with bit 3 set hold their 8-B column granules (4
// values) pairwise swapped (granule ^ 1): the Pd image, written by 16-lane groups of 16
// consecutive rows (ds_write_b64 banks on (a/4) mod 32: rows i and i + 8 collide at a
// 36-dword stride; the swap moves i + 8 onto the other granule of the pair)
MSU_DEV int pswz(int i) { return (i >> 3) & 1; }
MSU_DEV bf16x8 frag_tr_q4_swz(const bf16_t* img, int ld, int r0, int col0, int lane) {
  const int g = lane >> 4, li = lane & 15, q = li >> 2, p = li & 3, h = lane >> 5;
  const int row = r0 + 4 * q + 2 * h;
  const int col = ((((col0 + 16 * (g & 1)) >> 2) + p) ^ pswz(row)) << 2;  // rows row, row + 1: same bit 3
  v4s both[2] = {tr_read(img + row * ld + col), tr_read(img + (row + 1) * ld + col)};
  return *reinterpret_cast<bf16x8*>(both);
}

// accumulator registers 8s..8s+7 -> 16-bit fragment
template <typename T>
MSU_DEV bf16x8 pack8(const f32x16& a, int s) {
  const u32x4 w = {pack2<T>(a[8 * s], a[8 * s + 1]), pack2<T>(a[8 * s + 2], a[8 * s + 3]),
                   pack2<T>(a[8 * s + 4], a[8 * s + 5]), pack2<T>(a[8 * s + 6], a[8 * s + 7])};
  return __builtin_bit_cast(bf16x8, w);
}

// accumulator row of register r for lane half h (32x32 C layout)
MSU_DEV constexpr int crow(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

MSU_DEV int region(int p, int P, int s) { return s == 0 ? 0 : (p < P - WS ? 0 : (p < P - s ? 1 : 2)); }

// Token table of the window: sTok = source token, TOK_PAD (padded) or TOK_ZERO (t >= 49);
// sReg = mask region.  Returns whether the mask is non-trivial for this window.
MSU_DEV bool window_tokens(const Geom& g, long win_l, int* sTok, int* sReg, int lane) {
  const int win = (int)win_l;  // < 2^31 windows (checked on the host)
  const int nw = g.nWy * g.nWx;
  const int b = win / nw;
  const int wr = win - b * nw;
  const int wy = wr / g.nWx, wx = wr - (wr / g.nWx) * g.nWx;
  int tok = TOK_ZERO, reg = 0;
  if (lane < NT) {
    const int py = wy * WS + lane / WS, px = wx * WS + lane % WS;
    int sy = py + g.sh; if (sy >= g.Hp) sy -= g.Hp;
    int sx = px + g.sw; if (sx >= g.Wp) sx -= g.Wp;
    tok = (sy < g.H && sx < g.W) ? (b * g.H + sy) * g.W + sx : TOK_PAD;
    reg = region(py, g.Hp, g.sh) * 3 + region(px, g.Wp, g.sw);
  }
  sTok[lane] = tok;
  sReg[lane] = reg;
  return (g.sh + g.sw) > 0 && (wy == g.nWy - 1 || wx == g.nWx - 1);
}

typedef __bf16 bf16x2_v __attribute__((ext_vector_type(2)));
typedef _Float16 f16x2_v __attribute__((ext_vector_type(2)));

// keep factor of bit N of m: s where the bit is set, +0 where clear.  v_bfe_i32 spreads the
// bit over the word and an AND keeps s's bits: two VALU ops and no lane mask (the compiler's
// select form kept one SGPR-pair compare mask per key live and spilled SGPRs to VGPR lanes)
template <int N>
MSU_DEV float keep_factor(uint32_t m, float s) {
  int b;
  asm("v_bfe_i32 %0, %1, %2, 1" : "=v"(b) : "v"(m), "n"(N));
  return __int_as_float(b & __float_as_int(s));
}

// two values -> one packed 16-bit pair with one v_cvt_pk_{bf16,f16}_f32 (RNE, as pack2)
template <typename T>
MSU_DEV uint32_t pack2v(f32x2 v) {
  if constexpr (std::is_same<T, f16_t>::value)
    return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, f16x2_v));
  else
    return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, bf16x2_v));
}

MSU_DEV f32x2 pair(const f32x16& a, int r) { return f32x2{a[r], a[r + 1]}; }
MSU_DEV void set_pair(f32x16& a, int r, f32x2 v) {
  a[r] = v.x;
  a[r + 1] = v.y;
}

// Accumulator register r of key tile jt holds key jt*32 + crow(r, hh): for jt = 1 and r >= 9
// that key is >= 49 in BOTH lane halves -- a padded key of every window (bias -inf, P = 0).
// Those 7 of the 32 score registers skip the softmax / dropout / dS work.
MSU_DEV constexpr bool live_key(int jt, int r) { return !(jt == 1 && r >= 9); }
constexpr int DROP_WORDS = 13;  // stream words holding a live key (word n: bits 2n, 2n + 1)

// keep bits of the lane's 32 keys of query column tile it: bit jt*16 + r <-> key
// jt*32 + crow(r, hh) (word n of the lane's stream holds bits 2n, 2n+1, common.h); the words
// past DROP_WORDS only cover padded keys and are not drawn (their bits stay 0)
// SERIAL: not unrolled (the backward's re-hash path, whose register peak an unrolled stream raises)
template <bool SERIAL>
MSU_DEV uint32_t drop_bits(uint32_t seed, uint32_t item, int i, int hh, uint32_t thr) {
  DropStream s = drop_stream(seed, item, i, hh);
  uint32_t m = 0;
  if constexpr (SERIAL) {
#pragma unroll 1
    for (int n = 0; n < DROP_WORDS; ++n) m |= drop_next2(s, thr) << (2 * n);
  } else {
#pragma unroll
    for (int n = 0; n < DROP_WORDS; ++n) m |= drop_next2(s, thr) << (2 * n);
  }
  return m;
}

MSU_DEV void lds_sync() {
  __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)
  __builtin_amdgcn_wave_barrier();
}

// Softmax over keys j of one query-column tile (it): the lane's column of both key tiles
// (accumulator rows) + the other half-wave (xor-32).  exp(scale (s - max)) as 2^(c s - c max).
MSU_DEV void softmax_col(f32x16 (&P)[2], float scale) {
  float m = -INFINITY;
#pragma unroll
  for (int jt = 0; jt < 2; ++jt)
#pragma unroll
    for (int r = 0; r < 16; ++r)
      if (live_key(jt, r)) m = fmaxf(m, P[jt][r]);
  m = fmaxf(m, __shfl_xor(m, 32, 64));
  const float c = scale * 1.44269504088896341f;
  const float mc = m * c;
  // pairs of registers on the packed f32 ops (v_pk_fma / v_pk_add / v_pk_mul)
  const f32x2 c2 = {c, c}, nmc2 = {-mc, -mc};
  f32x2 sum2 = {0.f, 0.f};
#pragma unroll
  for (int jt = 0; jt < 2; ++jt)
#pragma unroll
    for (int r = 0; r < 16; r += 2) {
      if (live_key(jt, r + 1)) {
        const f32x2 x = __builtin_elementwise_fma(pair(P[jt], r), c2, nmc2);
        const f32x2 e = {__builtin_amdgcn_exp2f(x.x), __builtin_amdgcn_exp2f(x.y)};
        set_pair(P[jt], r, e);
        sum2 += e;
      } else if (live_key(jt, r)) {
        P[jt][r] = __builtin_amdgcn_exp2f(fmaf(P[jt][r], c, -mc));
        P[jt][r + 1] = 0.f;
        sum2.x += P[jt][r];
      } else {
        P[jt][r] = P[jt][r + 1] = 0.f;
      }
    }
  float sum = sum2.x + sum2.y;
  sum += __shfl_xor(sum, 32, 64);
  const float inv = 1.0f / sum;
  const f32x2 inv2 = {inv, inv};
#pragma unroll
  for (int jt = 0; jt < 2; ++jt)
#pragma unroll
    for (int r = 0; r < 16; r += 2) {
      if (live_key(jt, r + 1)) set_pair(P[jt], r, pair(P[jt], r) * inv2);
      else if (live_key(jt, r)) P[jt][r] *= inv;
    }
}

// dropout of one query-column tile: P * keep / (1 - p) on register pairs (keep_factor + one
// v_pk_mul_f32 per pair; keep bit jt*16 + r as drop_bits lays them out)
MSU_DEV void drop_scale(f32x16 (&P)[2], uint32_t kmask, float kscale) {
  static_for([&](auto JT) {
    constexpr int jt = decltype(JT)::value;
    static_for([&](auto RP) {
      constexpr int r = 2 * decltype(RP)::value;
      if constexpr (live_key(jt, r + 1)) {
        const f32x2 kf = {keep_factor<jt * 16 + r>(kmask, kscale), keep_factor<jt * 16 + r + 1>(kmask, kscale)};
        set_pair(P[jt], r, pair(P[jt], r) * kf);
      } else if constexpr (live_key(jt, r)) {
        P[jt][r] *= keep_factor<jt * 16 + r>(kmask, kscale);
      }
    }, std::make_integer_sequence<int, 8>{});
  }, std::make_integer_sequence<int, 2>{});
}

// shifted-window mask of one query-column tile: -100/scale where query and key regions differ
MSU_DEV void mask_col(f32x16 (&P)[2], const int* sReg, int it, float scale, int lane) {
  const float mval = -100.0f / scale;
  const int ri = sReg[it * 32 + (lane & 31)], hh = lane >> 5;
#pragma unroll
  for (int jt = 0; jt < 2; ++jt)
#pragma unroll
    for (int r = 0; r < 16; ++r)
      if (live_key(jt, r) && sReg[jt * 32 + crow(r, hh)] != ri) P[jt][r] += mval;
}

struct Aux {
  const float* bimg;      // [nh][4096] bias image / scale
  const bf16_t* biasrow;  // [3C] 16-bit qkv bias (padded tokens' q|k|v)
  const bf16_t* zrow;     // [3C] zeros (row of a TOK_ZERO token, any column offset)
};

struct FwdLds {
  bf16_t k[64 * LD], q[64 * LD], v[64 * LD];  // q doubles as the output staging image
  int tok[2][64], reg[2][64];  // double-buffered token tables (current / prefetched item)
};

// Every token's 64-B head slice of q / k / v is fetched by 4 consecutive lanes (16 B each),
// so a load instruction moves 16 whole 64-B pieces -- not 32 tokens x 32 B as MFMA-layout
// fragment loads would (L2 request count, not bytes, bounds this kernel).

// Persistent, head-stationary: grid (nblk, nh); a workgroup keeps its head's bias image in
// LDS (read there instead of from L2 for every item) and its waves walk windows win,
// win + stride, ...; the HBM loads of window i+1 (token table, K / Q fragments, V rows) are
// issued before window i is computed, so their latency hides under window i's MFMAs and
// softmax instead of being paid per item.
template <typename T, int WAVES, bool DROP>
__global__ void __launch_bounds__(64 * WAVES, 2) attn_fwd_mfma(const bf16_t* __restrict__ qkv, Aux aux,
                                                               bf16_t* __restrict__ out, Geom g, float scale,
                                                               float p_drop, uint64_t seed0,
                                                               const unsigned long long* seed_dev,
                                                               uint32_t* __restrict__ keep_out) {
  const uint64_t seed = launch_seed(seed0, seed_dev);
  __shared__ __attribute__((aligned(16))) float4 sBimg[4 * 4 * 64];
  __shared__ __attribute__((aligned(16))) FwdLds lds_all[WAVES];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  FwdLds& L = lds_all[wave];
  const int h = blockIdx.y;
  {
    // bias image [tile][lane][16] (global) -> [tile][q][lane] float4 (LDS)
    const float4* src = reinterpret_cast<const float4*>(aux.bimg + (long)h * 4096);
    for (int e = threadIdx.x; e < 1024; e += 64 * WAVES) {
      const int t = e >> 8, q = (e >> 6) & 3, ln = e & 63;
      sBimg[e] = src[(t * 64 + ln) * 4 + q];
    }
  }
  __syncthreads();
  const long nitems = g.nwin;  // windows of this head
  const long C3 = 3L * g.C;
  const long stride = (long)gridDim.x * WAVES;
  const int hh = lane >> 5;
  long item = (long)xcd_remap(blockIdx.x, gridDim.x) * WAVES + wave;
  if (item >= nitems) return;  // no block-wide barriers after this point: waves are independent

  // row base of a window token: its qkv row, the qkv-bias row (padded token) or zeros
  auto rowbase = [&](int tok) -> const bf16_t* {
    return tok >= 0 ? qkv + (size_t)((unsigned)tok * (unsigned)C3) : (tok == TOK_PAD ? aux.biasrow : aux.zrow);
  };
  // operands of the current / next item, ping-ponged by a compile-time index so that they
  // stay in registers (a struct passed by reference ended up in scratch)
  u32x4 kr[2][4], qr[2][4], vr[2][4];
  bool bnd[2] = {false, false};
  auto prep = [&](long it, auto BUF) __attribute__((always_inline)) {
    constexpr int buf = decltype(BUF)::value;
    const int win = (int)it;
    bnd[buf] = window_tokens(g, win, L.tok[buf], L.reg[buf], lane);
    lds_sync();
    const int cq = h * HD + 8 * (lane & 3), ck = g.C + cq, cv = 2 * g.C + cq;
    static_for([&](auto CI) {
      constexpr int c = decltype(CI)::value;
      const bf16_t* rb = rowbase(L.tok[buf][stage_row(lane >> 2) + 16 * c]);
      if constexpr ((MSU_EXP & 16) != 0) {  // ablation: no q / k / v loads (compute-side time)
        const uint32_t f = 0x3c003c00u + (uint32_t)(lane & 7) + (uint32_t)c;
        kr[buf][c] = u32x4{f, f + 1, f + 2, f + 3};
        qr[buf][c] = u32x4{f + 4, f, f + 1, f + 2};
        vr[buf][c] = u32x4{f + 2, f + 3, f, f + 4};
        (void)rb;
      } else {
        kr[buf][c] = *reinterpret_cast<const u32x4*>(rb + ck);
        qr[buf][c] = *reinterpret_cast<const u32x4*>(rb + cq);
        vr[buf][c] = *reinterpret_cast<const u32x4*>(rb + cv);
      }
    }, std::make_integer_sequence<int, 4>{});
  };

  // one item: operands in `cur` (loaded during the previous item), next item's into `nx`
  auto step = [&](auto BUF, long it_cur) __attribute__((always_inline)) -> bool {
    constexpr int buf = decltype(BUF)::value;
    const int win = (int)it_cur;
    // K / Q / V rows of this item -> LDS (the previous item's reads are complete: lds_sync below)
    static_for([&](auto CI) {
      constexpr int c = decltype(CI)::value;
      const int o = (stage_row(lane >> 2) + 16 * c) * LD + (lane & 3) * 8;
      *reinterpret_cast<u32x4*>(L.k + o) = kr[buf][c];
      *reinterpret_cast<u32x4*>(L.q + o) = qr[buf][c];
      *reinterpret_cast<u32x4*>(L.v + o) = vr[buf][c];
    }, std::make_integer_sequence<int, 4>{});
    // dropout keep bits (bit jt*16 + r of kmasks[it], the backward's layout), drawn while
    // the fewest registers are live: this window's rows are in LDS, the next one's not issued
    uint32_t kmasks[2] = {~0u, ~0u};
    if constexpr (DROP && (MSU_EXP & 32) != 0) {  // ablation: no mask stream (fixed pattern)
      kmasks[0] = 0xfff7fffeu ^ (uint32_t)lane;
      kmasks[1] = 0xffeffffdu ^ (uint32_t)win;
    } else if constexpr (DROP) {
#pragma unroll
      for (int it = 0; it < 2; ++it)
        kmasks[it] = drop_bits<false>(drop_seed32(seed), (uint32_t)win * g.nh + h, it * 32 + (lane & 31), hh,
                               drop_thresh16(p_drop));
    }
    const long nxt = it_cur + stride;
    const bool more = nxt < nitems;
    if (more) prep(nxt, std::integral_constant<int, buf ^ 1>{});
    lds_sync();
    bf16x8 ka[2][2];
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) ka[t][ks] = frag_rows(L.k, LD, 32 * t, 16 * ks, lane);
    // one query column tile (it) at a time: 32 queries x 64 keys of scores live at once
#pragma unroll
    for (int it = 0; it < 2; ++it) {
      f32x16 P[2];
#pragma unroll
      for (int jt = 0; jt < 2; ++jt) {  // bias image tiles (jt, it) from the LDS copy
        const float4* bp = sBimg + (jt * 2 + it) * 256 + lane;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float4 v = bp[64 * q];
          P[jt][4 * q] = v.x; P[jt][4 * q + 1] = v.y; P[jt][4 * q + 2] = v.z; P[jt][4 * q + 3] = v.w;
        }
      }
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const bf16x8 qf = frag_rows(L.q, LD, 32 * it, 16 * ks, lane);
#pragma unroll
        for (int jt = 0; jt < 2; ++jt) P[jt] = mfma32<T>(ka[jt][ks], qf, P[jt]);  // S^T = K Q^T (+ bias)
      }
      if (bnd[buf]) mask_col(P, L.reg[buf], it, scale, lane);
      softmax_col(P, scale);
      // (a per-element select-and-scale measured 17 % faster here than folding 1/(1-p) into the
      // normaliser and masking with keep_sel, 150 vs 180 us at stage 0)
      if constexpr (DROP) drop_scale(P, kmasks[it], 1.0f / (1.0f - p_drop));
      // O^T[d][i] = sum_j V[j][d] P^T[j][i]: P^T is the B operand straight from the registers
      f32x16 O = f32x16{0};
#pragma unroll
      for (int jt = 0; jt < 2; ++jt)
#pragma unroll
        for (int sb = 0; sb < 2; ++sb)
          O = mfma32<T>(frag_tr_perm(L.v, LD, jt * 32 + 16 * sb, 0, lane), pack8<T>(P[jt], sb), O);
      // output through the q image (rows of this tile, whose fragments are consumed): lane ->
      // query i, registers 4gq..4gq+3 -> d = 8gq + 4hh .. +3
      const int i = it * 32 + (lane & 31);
#pragma unroll
      for (int gq = 0; gq < 4; ++gq) {
        uint2 w;
        w.x = pack2<T>(O[4 * gq], O[4 * gq + 1]);
        w.y = pack2<T>(O[4 * gq + 2], O[4 * gq + 3]);
        *reinterpret_cast<uint2*>(L.q + i * LD + 8 * gq + 4 * hh) = w;
      }
    }
    lds_sync();
    u32x4 ov[4];
    int otok[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int t = read_row(lane >> 2) + 16 * c;
      otok[c] = L.tok[buf][t];
      ov[c] = *reinterpret_cast<const u32x4*>(L.q + t * LD + 8 * (lane & 3));
    }
#pragma unroll
    for (int c = 0; c < 4; ++c)
      if (otok[c] >= 0 && (!(MSU_EXP & 64) || scale == 1.2345e-30f))  // ablation 64: no output stores
        *reinterpret_cast<u32x4*>(out + (size_t)((unsigned)otok[c] * (unsigned)g.C) + h * HD + 8 * (lane & 3)) = ov[c];
    if (DROP && keep_out) {
      // keep bits for the backward: [item][it][lane] words, two 256-B stores per wave.  Issued
      // after the next window's loads: vmcnt retires in order, so a store issued before them
      // would put its write latency on the next item's operand wait
      uint32_t* kp = keep_out + ((size_t)win * g.nh + h) * 128 + lane;
      kp[0] = kmasks[0];
      kp[64] = kmasks[1];
    }
    lds_sync();  // LDS reads of this item done before they are overwritten
    return more;
  };

  prep(item, std::integral_constant<int, 0>{});
  for (;;) {
    if (!step(std::integral_constant<int, 0>{}, item)) break;
    item += stride;
    if (!step(std::integral_constant<int, 1>{}, item)) break;
    item += stride;
  }
}

// Store one 32-d head slice of a lane-major accumulator (lane = token, registers 4q..4q+3 =
// d 8q + 4hh .. +3) as two 16-B stores per lane: a permlane32 swap pairs each half's 4-d
// groups into 8 consecutive d (half 0 ends with d 16p..16p+7, half 1 with 16p+8..+15).
// Every lane must execute it (the swap reads the partner half); `row` is used when ok.
template <typename T>
MSU_DEV void store_slice(bf16_t* row, const f32x16& a, float s, int hh, bool ok) {
  uint32_t w[8];
#pragma unroll
  for (int g = 0; g < 8; ++g) w[g] = pack2<T>(a[2 * g] * s, a[2 * g + 1] * s);
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    const auto s0 = __builtin_amdgcn_permlane32_swap(w[4 * p], w[4 * p + 2], false, false);
    const auto s1 = __builtin_amdgcn_permlane32_swap(w[4 * p + 1], w[4 * p + 3], false, false);
    const u32x4 v = {s0[0], s1[0], s0[1], s1[1]};
    if (ok) *reinterpret_cast<u32x4*>(row + 16 * p + 8 * hh) = v;
  }
}

// Padded tokens' rows of a lane-major accumulator, summed over the tile's lanes into
// acc (lane d = lane&31 of half hh holds d's sum when bit 2 of d is hh; the other half 0).
MSU_DEV void pad_accumulate(float& acc, const f32x16& a, float s, bool pad, int lane) {
  const int hh = lane >> 5;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    float v = pad ? a[r] * s : 0.f;
#pragma unroll
    for (int m = 1; m < 32; m <<= 1) v += __shfl_xor(v, m, 64);
    if ((lane & 31) == crow(r, hh)) acc += v;
  }
}

// source token and mask region of window token t (window_tokens, one entry per call)
MSU_DEV int token_of(const Geom& g, int win, int t, int* reg) {
  const int nw = g.nWy * g.nWx;
  const int b = win / nw;
  const int wr = win - b * nw;
  const int wy = wr / g.nWx, wx = wr - wy * g.nWx;
  if (t >= NT) {
    *reg = 0;
    return TOK_ZERO;
  }
  const int py = wy * WS + t / WS, px = wx * WS + t % WS;
  int sy = py + g.sh; if (sy >= g.Hp) sy -= g.Hp;
  int sx = px + g.sw; if (sx >= g.Wp) sx -= g.Wp;
  *reg = region(py, g.Hp, g.sh) * 3 + region(px, g.Wp, g.sw);
  return (sy < g.H && sx < g.W) ? (b * g.H + sy) * g.W + sx : TOK_PAD;
}

MSU_DEV bool window_boundary(const Geom& g, int win) {
  const int wr = win % (g.nWy * g.nWx);
  return (g.sh + g.sw) > 0 && (wr / g.nWx == g.nWy - 1 || wr % g.nWx == g.nWx - 1);
}

struct BwdLds {
  bf16_t q[64 * LD], k[64 * LD], v[64 * LD], dO[64 * LD];  // the window's head slices [t][d]
  bf16_t P[64 * LDP], dS[64 * LDP];                          // [i][j] images (Pd and dS)
  int tok[2][64], reg[2][64];                                // current / next window's token table
};

// Backward: a 2-wave workgroup per (window, head) item -- wave w owns query tile it = w in the
// score pass and key tile mt = w in the gradient pass, so each wave carries half the item's
// state (registers ~190, LDS ~20 KB) and two workgroups share a SIMD pair: one item's
// latency chain (LDS round trips, MFMA dependencies, softmax) hides under the other's.
//   score pass (it = w):  S^T[:, it] = K Q_it^T + bias, P^T by softmax over j (the lane's
//     column, + one xor-32 shuffle), dPd^T = V dO_it^T, delta, dS^T = P^T (dP^T - delta);
//     Pd and dS written as rows i of the [i][j] images; dS^T summed into dB (this wave's
//     bias-image column tiles).
//   gradient pass (mt = w): dV^T = dO^T Pd, dK^T = Q^T dS for keys j in tile mt and
//     dQ^T = K^T dS^T for queries i in tile mt -- the token index on the accumulator columns,
//     so every lane stores whole 16-B pieces of its token's rows.
// Blocks walk windows blk, blk + nblk, ...; window k+1's rows are loaded into registers (each
// wave its 32 rows) while window k is computed.
// KEPT: the forward's keep bits are read from keep_in ([item][it][lane] words) instead of
// re-hashed (16 hashes per lane per window were ~15 % of the stage-0 backward).
// HPW heads per workgroup (2 HPW waves): the heads of a window run side by side, so the 128-B
// lines their 64-B q / k / v / dO slices share are fetched once (one head per workgroup read
// them 1.55x over, r04e counters).  Each head pair has its own LDS, the workgroup shares the
// barriers.
template <typename T, bool DROP, bool KEPT, int HPW>
__global__ void __launch_bounds__(128 * HPW, HPW == 3 ? 1 : 2) attn_bwd_mfma(
    const bf16_t* __restrict__ qkv, Aux aux, const bf16_t* __restrict__ dout, bf16_t* __restrict__ dqkv,
    float* __restrict__ dB_part, float* __restrict__ qb_part, Geom g, float scale, float p_drop,
    uint64_t seed0, const unsigned long long* seed_dev, const uint32_t* __restrict__ keep_in, int nblk) {
  static_assert(DROP || !KEPT, "keep bits only with dropout");
  const uint64_t seed = launch_seed(seed0, seed_dev);
  __shared__ __attribute__((aligned(16))) BwdLds Ls[HPW];
  const int slot = HPW == 1 ? 0 : (int)(threadIdx.x >> 7), tid = threadIdx.x & 127;
  BwdLds& L = Ls[slot];
  const int lane = threadIdx.x & 63, w = tid >> 6;  // w: this wave's query / key tile
  const int h = blockIdx.y * HPW + slot;
  const long C3 = 3L * g.C;
  const int hh = lane >> 5;
  const float* bimg = aux.bimg + (long)h * 4096;
  const int cq = h * HD, ck = g.C + h * HD, cv = 2 * g.C + h * HD;
  const float kscale = 1.0f / (1.0f - p_drop);  // the forward's kept-value factor
  f32x16 dB[2];  // dS^T tiles (jt, it = w) summed over this block's windows
  dB[0] = f32x16{0};
  dB[1] = f32x16{0};
  float padacc[3] = {0.f, 0.f, 0.f};  // column d = lane&31 of padded tokens' dq, dk, dv (per half)
  u32x4 rq[2][2], rk[2][2], rv[2][2], rd[2][2];  // [buf][c]: rows 32w + (lane>>2) + 16c
  uint32_t rkeep[2] = {~0u, ~0u};                 // [buf]: the forward's keep bits (KEPT)
  bool bnd[2] = {false, false};
  auto rowbase = [&](int tok) -> const bf16_t* {
    return tok >= 0 ? qkv + (size_t)((unsigned)tok * (unsigned)C3) : (tok == TOK_PAD ? aux.biasrow : aux.zrow);
  };
  // window win's token-table entries 32w + (lane&31) and this wave's rows -> registers
  auto prep = [&](long win_l, auto BUF) __attribute__((always_inline)) {
    constexpr int buf = decltype(BUF)::value;
    const int win = (int)win_l;  // < 2^31 windows (checked on the host)
    bnd[buf] = window_boundary(g, win);
    int reg;
    const int tt = 32 * w + (lane & 31);
    const int tokt = token_of(g, win, tt, &reg);
    if (lane < 32) {
      L.tok[buf][tt] = tokt;
      L.reg[buf][tt] = reg;
    }
    const int o = 8 * (lane & 3);
    if constexpr (KEPT) rkeep[buf] = keep_in[((size_t)win * g.nh + h) * 128 + 64 * w + lane];
    static_for([&](auto CI) {
      constexpr int c = decltype(CI)::value;
      int rg;  // (a __shfl of tokt from lane (lane>>2) + 16c measured no faster)
      const int tok = token_of(g, win, 32 * w + stage_row(lane >> 2) + 16 * c, &rg);
      const bf16_t* rb = rowbase(tok);
      rq[buf][c] = *reinterpret_cast<const u32x4*>(rb + cq + o);
      rk[buf][c] = *reinterpret_cast<const u32x4*>(rb + ck + o);
      rv[buf][c] = *reinterpret_cast<const u32x4*>(rb + cv + o);
      const bf16_t* db = tok >= 0 ? dout + (size_t)((unsigned)tok * (unsigned)g.C) + h * HD : aux.zrow;
      rd[buf][c] = *reinterpret_cast<const u32x4*>(db + o);
    }, std::make_integer_sequence<int, 2>{});
  };
  auto step = [&](auto BUF, long win) __attribute__((always_inline)) -> bool {
    constexpr int buf = decltype(BUF)::value;
    static_for([&](auto CI) {
      constexpr int c = decltype(CI)::value;
      const int off = (32 * w + stage_row(lane >> 2) + 16 * c) * LD + 8 * (lane & 3);
      *reinterpret_cast<u32x4*>(L.q + off) = rq[buf][c];
      *reinterpret_cast<u32x4*>(L.k + off) = rk[buf][c];
      *reinterpret_cast<u32x4*>(L.v + off) = rv[buf][c];
      *reinterpret_cast<u32x4*>(L.dO + off) = rd[buf][c];
    }, std::make_integer_sequence<int, 2>{});
    const int it = w;
    f32x16 P[2], D[2];
    // the bias-image loads go out BEFORE the next window's prefetch: vmcnt retires in order, so
    // a load issued after the prefetch would wait for the prefetch's HBM latency here
#pragma unroll
    for (int jt = 0; jt < 2; ++jt) {
      const float4* bp = reinterpret_cast<const float4*>(bimg + ((jt * 2 + it) * 64 + lane) * 16);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float4 v = (MSU_EXP & 1) ? make_float4(0.f, 0.f, 0.f, 0.f) : bp[q];
        P[jt][4 * q] = v.x; P[jt][4 * q + 1] = v.y; P[jt][4 * q + 2] = v.z; P[jt][4 * q + 3] = v.w;
      }
      D[jt] = f32x16{0};
    }
    __syncthreads();  // rows + this window's token table visible to both waves
    const long nxt = win + nblk;
    const bool more = nxt < g.nwin;
    if (more) {
      if constexpr ((MSU_EXP & 4) != 0) {
        // ablation "no row prefetch": the next window computes on stale rows (results wrong
        // by design), but its token table must still be written -- the gradient pass forms
        // store addresses from it (skipping it faulted)
        constexpr int nb = buf ^ 1;
        bnd[nb] = window_boundary(g, (int)nxt);
        int reg;
        const int tt = 32 * w + (lane & 31);
        const int tokt = token_of(g, (int)nxt, tt, &reg);
        if (lane < 32) {
          L.tok[nb][tt] = tokt;
          L.reg[nb][tt] = reg;
        }
      } else {
        prep(nxt, std::integral_constant<int, buf ^ 1>{});
      }
    }
    const bool boundary = bnd[buf];
    const int* sTok = L.tok[buf];
    const int* sReg = L.reg[buf];
    // ---- score pass: query tile it = w
    const int i = it * 32 + (lane & 31);
    uint32_t kmask = ~0u;  // bit jt*16+r: (i, key jt*32 + crow(r, hh)) kept by the dropout
    if constexpr (KEPT)
      kmask = rkeep[buf];
    else if constexpr (DROP && !(MSU_EXP & 8))  // the forward's mask, regenerated from the seed
      kmask = drop_bits<true>(drop_seed32(seed), (uint32_t)win * g.nh + h, i, hh, drop_thresh16(p_drop));
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const bf16x8 qf = frag_rows(L.q, LD, 32 * it, 16 * ks, lane);
      const bf16x8 df = frag_rows(L.dO, LD, 32 * it, 16 * ks, lane);
#pragma unroll
      for (int jt = 0; jt < 2; ++jt) {
        P[jt] = mfma32<T>(frag_rows(L.k, LD, 32 * jt, 16 * ks, lane), qf, P[jt]);  // S^T = K Q^T (+ bias)
        D[jt] = mfma32<T>(frag_rows(L.v, LD, 32 * jt, 16 * ks, lane), df, D[jt]);  // dPd^T = V dO^T
      }
    }
    if (boundary) mask_col(P, sReg, it, scale, lane);
    softmax_col(P, scale);
    // Pd and dS images [i][j], 4 consecutive j (registers 4gq .. 4gq + 3) per 8-byte store, on
    // register pairs (packed f32 ops).  Pass 1: dP = dPd keep / (1 - p), Pd = P keep / (1 - p)
    // (-> the Pd image) and delta = sum_j P dP; pass 2: dS = P (dP - delta) (-> the dS image,
    // dB).  Group gq = 3 of key tile 1 (keys 56 .. 63) is padding in every window: its image
    // words were zeroed once before the window loop.
    f32x2 dl = {0.f, 0.f};
    static_for([&](auto JT) {
      constexpr int jt = decltype(JT)::value;
      static_for([&](auto GQ) {
        constexpr int gq = decltype(GQ)::value;
        if constexpr (jt == 0 || gq < 3) {
          f32x2 pd[2];
          static_for([&](auto E2) {
            constexpr int r = 4 * gq + 2 * decltype(E2)::value;
            if constexpr (live_key(jt, r)) {
              f32x2 p = pair(P[jt], r), d = pair(D[jt], r);
              if constexpr (!live_key(jt, r + 1)) p.y = d.y = 0.f;  // key 49 .. (P = 0)
              if constexpr (DROP) {
                const f32x2 kf = {keep_factor<jt * 16 + r>(kmask, kscale), keep_factor<jt * 16 + r + 1>(kmask, kscale)};
                d *= kf;
                pd[decltype(E2)::value] = p * kf;
              } else {
                pd[decltype(E2)::value] = p;
              }
              dl = __builtin_elementwise_fma(p, d, dl);
              set_pair(D[jt], r, d);
            } else {
              pd[decltype(E2)::value] = f32x2{0.f, 0.f};
            }
          }, std::make_integer_sequence<int, 2>{});
          const uint2 wp = {pack2v<T>(pd[0]), pack2v<T>(pd[1])};
          *reinterpret_cast<uint2*>(L.P + i * LDP + jt * 32 + 8 * gq + 4 * (hh ^ pswz(i))) = wp;
        }
      }, std::make_integer_sequence<int, 4>{});
    }, std::make_integer_sequence<int, 2>{});
    float delta = dl.x + dl.y;
    delta += __shfl_xor(delta, 32, 64);
    const f32x2 delta2 = {delta, delta};
    static_for([&](auto JT) {
      constexpr int jt = decltype(JT)::value;
      static_for([&](auto GQ) {
        constexpr int gq = decltype(GQ)::value;
        if constexpr (jt == 0 || gq < 3) {
          f32x2 ds[2];
          static_for([&](auto E2) {
            constexpr int r = 4 * gq + 2 * decltype(E2)::value;
            if constexpr (live_key(jt, r)) {
              f32x2 v = pair(P[jt], r) * (pair(D[jt], r) - delta2);
              if constexpr (!live_key(jt, r + 1)) v.y = 0.f;
              ds[decltype(E2)::value] = v;
              set_pair(dB[jt], r, pair(dB[jt], r) + v);
            } else {
              ds[decltype(E2)::value] = f32x2{0.f, 0.f};
            }
          }, std::make_integer_sequence<int, 2>{});
          const uint2 wd = {pack2v<T>(ds[0]), pack2v<T>(ds[1])};
          *reinterpret_cast<uint2*>(L.dS + i * LDP + jt * 32 + 8 * gq + 4 * hh) = wd;
        }
      }, std::make_integer_sequence<int, 4>{});
    }, std::make_integer_sequence<int, 2>{});
    __syncthreads();  // both halves of the images written
    // ---- gradient pass: key tile mt = w (dV, dK) and query tile mt (dQ)
    // dV^T[d][j] = sum_i dO[i][d] Pd[i][j]; dK^T[d][j] = scale sum_i Q[i][d] dS[i][j];
    // dQ^T[d][i] = scale sum_j K[j][d] dS[i][j]   (scores = scale * q k^T)
    const int mt = w;
    const int tok = sTok[mt * 32 + (lane & 31)];
    const bool pad = tok == TOK_PAD;
    const bool anypad = __ballot(pad) != 0;  // wave-uniform: only windows over the padded border
    bf16_t* row = dqkv + (size_t)((unsigned)(tok >= 0 ? tok : 0) * (unsigned)C3) + h * HD;
    const bool st_ok = tok >= 0 && (!(MSU_EXP & 2) || scale == 1.2345e-30f);
    {
      f32x16 av = f32x16{0}, ak = f32x16{0};
#pragma unroll 1  // unrolled, the fragment reads of all four k steps were hoisted: 17 VGPRs spilled
      for (int ks = 0; ks < 64; ks += 16) {
        av = mfma32<T>(frag_tr_q4(L.dO, LD, ks, 0, lane), frag_tr_q4_swz(L.P, LDP, ks, mt * 32, lane), av);
        ak = mfma32<T>(frag_tr_q4(L.q, LD, ks, 0, lane), frag_tr_q4(L.dS, LDP, ks, mt * 32, lane), ak);
      }
      store_slice<T>(row + g.C, ak, scale, hh, st_ok);
      store_slice<T>(row + 2 * g.C, av, 1.0f, hh, st_ok);
      if (anypad) {
        pad_accumulate(padacc[1], ak, scale, pad, lane);
        pad_accumulate(padacc[2], av, 1.0f, pad, lane);
      }
    }
    {
      f32x16 aq = f32x16{0};
#pragma unroll 1
      for (int ks = 0; ks < 64; ks += 16)
        aq = mfma32<T>(frag_tr(L.k, LD, ks, 0, lane), frag_rows(L.dS, LDP, mt * 32, ks, lane), aq);
      store_slice<T>(row, aq, scale, hh, st_ok);
      if (anypad) pad_accumulate(padacc[0], aq, scale, pad, lane);
    }
    __syncthreads();  // this window's LDS reads done before the next window's rows land
    return more;
  };

  const long win0 = blockIdx.x;
  if (win0 < g.nwin) {  // block-uniform
    long win = win0;
    {  // the padded keys 56 .. 63 of this wave's query rows: zero in both images for good
      const int zi = w * 32 + (lane & 31), zo = zi * LDP + 56;
      *reinterpret_cast<uint2*>(L.P + zo + 4 * (hh ^ pswz(zi))) = uint2{0u, 0u};
      *reinterpret_cast<uint2*>(L.dS + zo + 4 * hh) = uint2{0u, 0u};
    }
    prep(win, std::integral_constant<int, 0>{});
    for (;;) {
      if (!step(std::integral_constant<int, 0>{}, win)) break;
      win += nblk;
      if (!step(std::integral_constant<int, 1>{}, win)) break;
      win += nblk;
    }
  }

  // dB -> the 169 relative-position entries, once per block: both waves' tiles go to LDS (over
  // the images) in the bias-image layout [tile jt*2+it][lane][16], then a thread sums a table
  // entry's <= 49 (i, j) pairs.  Partials [blk][169][nh] reduce over blocks straight into d table.
  const long part = blockIdx.x;
  float* img = reinterpret_cast<float*>(L.P);  // 16 KB image + 96 floats of wave 1's pad sums
  __syncthreads();
#pragma unroll
  for (int jt = 0; jt < 2; ++jt)
#pragma unroll
    for (int q = 0; q < 4; ++q)
      *reinterpret_cast<float4*>(img + ((jt * 2 + w) * 64 + lane) * 16 + 4 * q) =
          make_float4(dB[jt][4 * q], dB[jt][4 * q + 1], dB[jt][4 * q + 2], dB[jt][4 * q + 3]);
  float padv[3];
#pragma unroll
  for (int k = 0; k < 3; ++k) padv[k] = padacc[k] + __shfl_xor(padacc[k], 32, 64);
  if (w == 1 && lane < 32) {
#pragma unroll
    for (int k = 0; k < 3; ++k) img[4096 + 32 * k + lane] = padv[k];
  }
  __syncthreads();
  for (int e = tid; e < 169; e += 128) {
    const int dh = e / 13 - 6, dw = e % 13 - 6;
    float sum = 0.f;
    for (int ih = 0; ih < WS; ++ih) {
      const int jh = ih - dh;
      if (jh < 0 || jh >= WS) continue;
      for (int iw = 0; iw < WS; ++iw) {
        const int jw = iw - dw;
        if (jw < 0 || jw >= WS) continue;
        const int ii = ih * WS + iw, j = jh * WS + jw;
        const int jj = j & 31;
        sum += img[(((j >> 5) * 2 + (ii >> 5)) * 64 + (ii & 31) + 32 * ((jj >> 2) & 1)) * 16 + (jj & 3) + 4 * (jj >> 3)];
      }
    }
    dB_part[(part * 169 + e) * g.nh + h] = sum;
  }
  if (w == 0 && lane < 32) {
#pragma unroll
    for (int k = 0; k < 3; ++k) qb_part[part * C3 + k * g.C + h * HD + lane] = padv[k] + img[4096 + 32 * k + lane];
  }
}

// bias image [nh][4 tiles (jt*2+it)][64 lanes][16 regs] = table[idx(i,j)][h] / scale
// (i, j < 49), -inf for padded keys j >= 49, 0 for padded queries i >= 49.  Block 0 also
// writes the 16-bit qkv-bias row and the zero row.
template <typename T>
__global__ void __launch_bounds__(256) aux_kernel(const float* table, const float* qkv_bias, int nh, int C3,
                                                  float inv_scale, float* img, bf16_t* biasrow, bf16_t* zrow) {
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (blockIdx.x == 0) {
    for (int c = threadIdx.x; c < C3; c += 256) biasrow[c] = (bf16_t)Fmt16<T>::bits(qkv_bias[c]);
    for (int c = threadIdx.x; c < C3; c += 256) zrow[c] = 0;
  }
  if (e >= nh * 4096) return;
  const int h = e / 4096, rem = e % 4096;
  const int t = rem / 1024, lane = (rem / 16) % 64, r = rem % 16;
  const int jt = t >> 1, it = t & 1;
  const int j = jt * 32 + crow(r, lane >> 5), i = it * 32 + (lane & 31);
  float v;
  if (j >= NT) v = -INFINITY;
  else if (i >= NT) v = 0.f;
  else v = table[((i / WS - j / WS + WS - 1) * (2 * WS - 1) + (i % WS - j % WS + WS - 1)) * nh + h] * inv_scale;
  img[e] = v;
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

constexpr int FWD_WAVES = 4;

// aux workspace (f32 units): bias image nh*4096, bf16 bias row (3C bf16), zero row (64 bf16)
long aux_floats(int C, int nh) { return (long)nh * 4096 + (6L * C + 1) / 2 + 4; }

Aux carve_aux(float* ws, int C, int nh, float** img_out, bf16_t** brow, bf16_t** zrow) {
  Aux a;
  *img_out = ws;
  *brow = reinterpret_cast<bf16_t*>(ws + (long)nh * 4096);
  *zrow = *brow + 3L * C;
  a.bimg = *img_out;
  a.biasrow = *brow;
  a.zrow = *zrow;
  return a;
}

// Workgroups per head (grid (n, nh), head-major dispatch order): min(need, cap), a multiple of
// 8 so that block (x, h) lands on XCD x % 8 for every head h.  The heads of one window then
// run on the same XCD at about the same time, and the 128-B lines they share (a head slice
// is 64 B of a token's q / k / v row) come from that XCD's L2 after the first head's miss.
long head_blocks(long need, long cap) {
  cap = cap / 8 * 8;
  if (cap < 8) cap = 8;
  if (need > cap) need = cap;
  return (need + 7) / 8 * 8;
}

// heads per backward workgroup: pairs for even nh (a 128-B line holds two heads' slices; the
// LDS still allows two 4-wave workgroups per CU), else one.  (All three heads at nh = 3 cut the
// stage-0 fetched bytes by a third, r04g: 431 vs 649 MB, but fit one 6-wave workgroup per CU
// instead of four 2-wave ones and ran 300 vs 267 us: not kept.)
int bwd_hpw(int nh) { return nh % 2 == 0 ? 2 : 1; }

// backward workgroups per head group: the LDS (40 KB per head) allows four heads per CU
// (three at nh = 3), i.e. 1024 / nh workgroups of 2 HPW waves (768 / nh at HPW = 3)
int bwd_blocks(long nwin, int nh) { return (int)head_blocks(nwin, 1024 / nh); }

template <typename T, int HPW>
void launch_bwd(dim3 grid, hipStream_t st, const void* qkv, const Aux& aux, const void* dout, void* dqkv,
                float* dB_part, float* qb_part, const Geom& g, float scale, float p_drop, unsigned long long seed,
                const unsigned long long* seed_dev, const void* keep, int nblk) {
  const dim3 blk(128 * HPW);
  if (p_drop > 0.f && keep)
    hipLaunchKernelGGL((attn_bwd_mfma<T, true, true, HPW>), grid, blk, 0, st, (const bf16_t*)qkv, aux,
                       (const bf16_t*)dout, (bf16_t*)dqkv, dB_part, qb_part, g, scale, p_drop, (uint64_t)seed,
                       seed_dev, (const uint32_t*)keep, nblk);
  else if (p_drop > 0.f)
    hipLaunchKernelGGL((attn_bwd_mfma<T, true, false, HPW>), grid, blk, 0, st, (const bf16_t*)qkv, aux,
                       (const bf16_t*)dout, (bf16_t*)dqkv, dB_part, qb_part, g, scale, p_drop, (uint64_t)seed,
                       seed_dev, nullptr, nblk);
  else
    hipLaunchKernelGGL((attn_bwd_mfma<T, false, false, HPW>), grid, blk, 0, st, (const bf16_t*)qkv, aux,
                       (const bf16_t*)dout, (bf16_t*)dqkv, dB_part, qb_part, g, scale, p_drop, (uint64_t)seed,
                       seed_dev, nullptr, nblk);
}

}  // namespace

// entry points used by window_attention.hip for the 16-bit dtypes
int msu_attn_mfma_bwd_tail(float* ws, float* dtable, float* dqkv_bias_pad, long nwin, int C, int nh,
                           hipStream_t st, int accumulate = 0);
long msu_attn_mfma_fwd_workspace(int C, int nh) { return aux_floats(C, nh); }

long msu_attn_mfma_bwd_workspace(long nwin, int C, int nh) {
  const long parts = (long)bwd_blocks(nwin, nh);
  return aux_floats(C, nh) + parts * nh * 169 + parts * 3L * C;
}

int msu_attn_mfma_fwd(int dtype, const void* qkv, const float* qkv_bias, const float* table, void* out, int B,
                      int H, int W, int C, int nh, int shift, float p_drop, unsigned long long seed,
                      const unsigned long long* seed_dev, void* keep, float* ws, hipStream_t st) {
  const Geom g = make_geom(B, H, W, C, nh, shift);
  const long items = g.nwin * nh;
  if (items == 0) return 0;
  const float scale = 1.0f / sqrtf((float)HD);
  float* img; bf16_t* brow; bf16_t* zrow;
  const Aux aux = carve_aux(ws, C, nh, &img, &brow, &zrow);
  // persistent: about two 4-wave workgroups per CU, split over the heads
  const long nb = head_blocks((g.nwin + FWD_WAVES - 1) / FWD_WAVES, 512 / nh);
  const dim3 grid((unsigned)nb, (unsigned)nh), blk(64 * FWD_WAVES);
  MSU_DISPATCH16(dtype, T,
    hipLaunchKernelGGL(aux_kernel<T>, dim3((nh * 4096 + 255) / 256), dim3(256), 0, st, table, qkv_bias, nh, 3 * C,
                       1.0f / scale, img, brow, zrow);
    if (p_drop > 0.f)
      hipLaunchKernelGGL((attn_fwd_mfma<T, FWD_WAVES, true>), grid, blk, 0, st, (const bf16_t*)qkv, aux,
                         (bf16_t*)out, g, scale, p_drop, (uint64_t)seed, seed_dev, (uint32_t*)keep);
    else
      hipLaunchKernelGGL((attn_fwd_mfma<T, FWD_WAVES, false>), grid, blk, 0, st, (const bf16_t*)qkv, aux,
                         (bf16_t*)out, g, scale, p_drop, (uint64_t)seed, seed_dev, nullptr));
  return MSU_CHECK_LAUNCH();
}

int msu_attn_mfma_bwd(int dtype, const void* qkv, const float* qkv_bias, const float* table, const void* dout,
                      void* dqkv, float* dtable, float* dqkv_bias_pad, float* ws, int B, int H, int W,
                      int C, int nh, int shift, float p_drop, unsigned long long seed,
                      const unsigned long long* seed_dev, const void* keep, hipStream_t st, hipStream_t pst) {
  const Geom g = make_geom(B, H, W, C, nh, shift);
  if (g.nwin == 0) return 0;
  const float scale = 1.0f / sqrtf((float)HD);
  const int nblk = bwd_blocks(g.nwin, nh);
  const long parts = nblk;
  float* img; bf16_t* brow; bf16_t* zrow;
  const Aux aux = carve_aux(ws, C, nh, &img, &brow, &zrow);
  float* dB_part = ws + aux_floats(C, nh);
  float* qb_part = dB_part + parts * nh * 169;
  const int hpw = bwd_hpw(nh);
  const dim3 grid(nblk, nh / hpw);
  // table null: the workspace's aux region (bias image, bias / zero rows) is the forward's, built
  // from the same table and qkv bias (one aux launch per layer and step instead of two)
  MSU_DISPATCH16(dtype, T,
    if (table != nullptr)
      hipLaunchKernelGGL(aux_kernel<T>, dim3((nh * 4096 + 255) / 256), dim3(256), 0, st, table, qkv_bias, nh, 3 * C,
                         1.0f / scale, img, brow, zrow);
    if (hpw == 2) launch_bwd<T, 2>(grid, st, qkv, aux, dout, dqkv, dB_part, qb_part, g, scale, p_drop, seed, seed_dev, keep, nblk);
    else launch_bwd<T, 1>(grid, st, qkv, aux, dout, dqkv, dB_part, qb_part, g, scale, p_drop, seed, seed_dev, keep, nblk));
  if (pst == (hipStream_t)(intptr_t)-1) return MSU_CHECK_LAUNCH();  // tail issued by the caller
  // parameter-gradient reductions: on pst (after the backward kernel) when given
  const int rc = attn_param_stream(st, pst);
  if (rc) return rc;
  return msu_attn_mfma_bwd_tail(ws, dtable, dqkv_bias_pad, g.nwin, C, nh, pst);
}

// the parameter-gradient reductions of msu_attn_mfma_bwd from its workspace partials
int msu_attn_mfma_bwd_tail(float* ws, float* dtable, float* dqkv_bias_pad, long nwin, int C, int nh,
                           hipStream_t st, int accumulate) {
  if (nwin == 0) return 0;
  const long parts = (long)bwd_blocks(nwin, nh);
  float* dB_part = ws + aux_floats(C, nh);
  float* qb_part = dB_part + parts * nh * 169;
  const ColSeg segs[2] = {{dB_part, 169L * nh, 169L * nh, dtable}, {qb_part, 3L * C, 3L * C, dqkv_bias_pad}};
  colsum_multi(segs, 2, (int)parts, accumulate, st);
  return MSU_CHECK_LAUNCH();
}

// =====================================================================================
// Fused stage-0 unit: qkv Linear + shifted-window attention in ONE kernel (the
// qkv -> attention round trip).  torchvision's block computes qkv = LN1(x) W^T + b for the
// padded, rolled window grid and runs the attention on it (model_parts.py:166-170 ->
// shifted_window_attention); here a workgroup loads a window's 64 LN1 rows (zeros for the
// padded / filler tokens: their qkv is then exactly the bias, as torchvision's pad-after-norm
// gives), multiplies them with the resident W_qkv on MFMA, keeps q / k / v in LDS and runs the
// attention of all heads on them.  The qkv tensor never has to be read back; in training it is
// still written once (the attention backward and the qkv weight gradient read it), in
// inference it is not written at all.
//   * one 6-wave workgroup per CU (persistent over windows): wave w = (head h = w >> 1, tile
//     t = w & 1) computes q, k, v of head h for tokens 32t .. 32t + 31 (3 x 32x32 tiles, K =
//     96: 18 MFMAs) and then the attention of head h for the queries of tile t;
//   * LDS: W_qkv [288][96] (55 KB, loaded once), the window's LN1 rows [64][96] (register-
//     staged one window ahead), q / k / v images per head [64][40] (46 KB), qkv bias;
//     rows of W / x use the 16-B chunk swizzle c ^ ((r >> 2) & 3) (conflict-free 32-row
//     fragment reads);
//   * attention as attn_fwd_mfma (transposed scores, bias image from the aux workspace, the
//     same dropout streams and keep-bit layout, so the existing backward consumes it).
// Stage-0 widths only (C = 96, 3 heads).
namespace {

constexpr int FQ_C = 96, FQ_NH = 3, FQ_C3 = 3 * FQ_C, FQ_CH = FQ_C / 8;  // 12 16-B chunks per row
constexpr int FQ_WAVES = 2 * FQ_NH;

struct FusedLds {
  bf16_t w[FQ_C3 * FQ_C];        // W_qkv rows (swizzled chunks)
  bf16_t wp[FQ_C * FQ_C];        // W_proj rows (swizzled chunks; PROJ)
  bf16_t x[64 * FQ_C];           // the window's LN1 rows (swizzled chunks); PROJ: then its output rows
  bf16_t qkv[FQ_NH][3][64 * LD];  // per head: q, k, v images [t][d] (padded rows); q then o
  float bias[FQ_C3];
  float pbias[FQ_C];
  int tok[64], reg[64];
};

MSU_DEV int fq_swz(int r) { return (r >> 2) & 3; }

// 32-row k-contiguous fragment of a swizzled [rows][96] image: lane -> row r0 + (lane & 31),
// k = 16 ks + 8 (lane >> 5) .. + 7
MSU_DEV bf16x8 fq_frag(const bf16_t* img, int r0, int ks, int lane) {
  const int r = r0 + (lane & 31);
  return *reinterpret_cast<const bf16x8*>(img + r * FQ_C + (((2 * ks + (lane >> 5)) ^ fq_swz(r)) << 3));
}

// PROJ: the proj Linear too -- y = o W_proj^T + b_proj from the three heads' o (in LDS) is the
// output (`out`), and o itself goes to o_out (the proj weight gradient's input) when given.
template <typename T, bool DROP, bool STORE_QKV, bool PROJ>
__global__ void __launch_bounds__(64 * FQ_WAVES) attn_qkv_fwd_mfma(const bf16_t* __restrict__ xin,
                                                                  const bf16_t* __restrict__ wqkv,
                                                                  const float* __restrict__ bqkv, Aux aux,
                                                                  bf16_t* __restrict__ out, bf16_t* __restrict__ qkv_out,
                                                                  Geom g, float scale, float p_drop, uint64_t seed0,
                                                                  const unsigned long long* seed_dev,
                                                                  uint32_t* __restrict__ keep_out,
                                                                  const bf16_t* __restrict__ wproj,
                                                                  const float* __restrict__ bproj,
                                                                  bf16_t* __restrict__ o_out) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  FusedLds& L = *reinterpret_cast<FusedLds*>(smem_raw);
  const uint64_t seed = launch_seed(seed0, seed_dev);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int h = wave >> 1, t = wave & 1, hh = lane >> 5;
  constexpr int NTHR = 64 * FQ_WAVES;
  // resident W_qkv and bias
  for (int s = tid; s < FQ_C3 * FQ_CH; s += NTHR) {
    const int r = s / FQ_CH, c = s - (s / FQ_CH) * FQ_CH;
    *reinterpret_cast<u32x4*>(L.w + r * FQ_C + ((c ^ fq_swz(r)) << 3)) =
        *reinterpret_cast<const u32x4*>(wqkv + r * FQ_C + 8 * c);
  }
  for (int s = tid; s < FQ_C3; s += NTHR) L.bias[s] = bqkv[s];
  if constexpr (PROJ) {
    for (int s = tid; s < FQ_C * FQ_CH; s += NTHR) {
      const int r = s / FQ_CH, c = s - (s / FQ_CH) * FQ_CH;
      *reinterpret_cast<u32x4*>(L.wp + r * FQ_C + ((c ^ fq_swz(r)) << 3)) =
          *reinterpret_cast<const u32x4*>(wproj + r * FQ_C + 8 * c);
    }
    for (int s = tid; s < FQ_C; s += NTHR) L.pbias[s] = bproj[s];
  }
  // the window's 64 x 12 chunks of LN1 rows: thread -> slots tid, tid + NTHR
  constexpr int XS = (64 * FQ_CH + NTHR - 1) / NTHR;  // 2
  u32x4 xr[XS];
  int tokr = TOK_ZERO, regr = 0;  // thread tid < 64: token-table entry tid of the staged window
  auto load_x = [&](long win) __attribute__((always_inline)) {
#pragma unroll
    for (int k = 0; k < XS; ++k) {
      const int s = tid + NTHR * k;
      const int r = s / FQ_CH, c = s - (s / FQ_CH) * FQ_CH;
      int rg;
      const int tok = s < 64 * FQ_CH ? token_of(g, (int)win, r, &rg) : TOK_ZERO;
      const bf16_t* src = tok >= 0 ? xin + (size_t)((unsigned)tok * (unsigned)FQ_C) + 8 * c : aux.zrow;
      xr[k] = *reinterpret_cast<const u32x4*>(src);
    }
    if (tid < 64) tokr = token_of(g, (int)win, tid, &regr);
  };
  const long stride = gridDim.x;
  long win = xcd_remap(blockIdx.x, gridDim.x);
  if (win < g.nwin) load_x(win);
  const float kscale = 1.0f / (1.0f - p_drop);
  const float* bimg = aux.bimg + (long)h * 4096;
  for (; win < g.nwin; win += stride) {
    // ---- stage the window: rows -> LDS, token table (the previous window's readers are done:
    // every wave passed the barrier after its attention below)
#pragma unroll
    for (int k = 0; k < XS; ++k) {
      const int s = tid + NTHR * k;
      const int r = s / FQ_CH, c = s - (s / FQ_CH) * FQ_CH;
      if (s < 64 * FQ_CH) *reinterpret_cast<u32x4*>(L.x + r * FQ_C + ((c ^ fq_swz(r)) << 3)) = xr[k];
    }
    if (tid < 64) {
      L.tok[tid] = tokr;
      L.reg[tid] = regr;
    }
    __syncthreads();
    const bool bnd = window_boundary(g, (int)win);
    // bias-image tiles (jt, it = t) of this wave's scores: issued now, consumed after the qkv GEMM
    f32x16 P[2];
#pragma unroll
    for (int jt = 0; jt < 2; ++jt) {
      const float4* bp = reinterpret_cast<const float4*>(bimg + ((jt * 2 + t) * 64 + lane) * 16);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float4 v = bp[q];
        P[jt][4 * q] = v.x; P[jt][4 * q + 1] = v.y; P[jt][4 * q + 2] = v.z; P[jt][4 * q + 3] = v.w;
      }
    }
    // next window's rows -> registers (latency hidden under this window)
    const long nxt = win + stride;
    if (nxt < g.nwin) load_x(nxt);
    // ---- q, k, v of head h for tokens 32t .. 32t + 31: D[ch][token], W rows as the A operand
    f32x16 acc[3];
#pragma unroll
    for (int m = 0; m < 3; ++m) acc[m] = f32x16{0};
#pragma unroll
    for (int ks = 0; ks < FQ_C / 16; ++ks) {
      const bf16x8 xf = fq_frag(L.x, 32 * t, ks, lane);
#pragma unroll
      for (int m = 0; m < 3; ++m) acc[m] = mfma32<T>(fq_frag(L.w, m * FQ_C + 32 * h, ks, lane), xf, acc[m]);
    }
    // + bias, round to 16 bits, rows of the q / k / v images (lane = token, registers 4g .. 4g+3 =
    // channels 8g + 4hh .. + 3)
    const int tk = 32 * t + (lane & 31);
#pragma unroll
    for (int m = 0; m < 3; ++m) {
      bf16_t* img = L.qkv[h][m];
#pragma unroll
      for (int gq = 0; gq < 4; ++gq) {
        const float4 b = *reinterpret_cast<const float4*>(L.bias + m * FQ_C + 32 * h + 8 * gq + 4 * hh);
        uint2 wv;
        wv.x = pack2<T>(acc[m][4 * gq] + b.x, acc[m][4 * gq + 1] + b.y);
        wv.y = pack2<T>(acc[m][4 * gq + 2] + b.z, acc[m][4 * gq + 3] + b.w);
        *reinterpret_cast<uint2*>(img + tk * LD + 8 * gq + 4 * hh) = wv;
      }
    }
    __syncthreads();  // q / k / v of every head and token tile in LDS; the LN1 rows are free
    if constexpr (STORE_QKV) {
      // the training path keeps qkv for the backward: this wave's tokens, head h's three
      // 64-B slices, 4 lanes per slice (16 whole slices per store instruction)
#pragma unroll
      for (int m = 0; m < 3; ++m)
#pragma unroll
        for (int c = 0; c < 2; ++c) {
          const int r = 32 * t + read_row(lane >> 2) + 16 * c;
          const int tok = L.tok[r];
          const u32x4 v = *reinterpret_cast<const u32x4*>(L.qkv[h][m] + r * LD + 8 * (lane & 3));
          if (tok >= 0)
            *reinterpret_cast<u32x4*>(qkv_out + (size_t)((unsigned)tok * (unsigned)FQ_C3) + m * FQ_C + h * HD +
                                      8 * (lane & 3)) = v;
        }
    }
    // ---- attention of head h, query tile t (as attn_fwd_mfma)
    const bf16_t* Lq = L.qkv[h][0];
    const bf16_t* Lk = L.qkv[h][1];
    const bf16_t* Lv = L.qkv[h][2];
    uint32_t kmask = ~0u;
    if constexpr (DROP)
      kmask = drop_bits<false>(drop_seed32(seed), (uint32_t)win * g.nh + h, t * 32 + (lane & 31), hh,
                               drop_thresh16(p_drop));
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const bf16x8 qf = frag_rows(Lq, LD, 32 * t, 16 * ks, lane);
#pragma unroll
      for (int jt = 0; jt < 2; ++jt) P[jt] = mfma32<T>(frag_rows(Lk, LD, 32 * jt, 16 * ks, lane), qf, P[jt]);
    }
    if (bnd) mask_col(P, L.reg, t, scale, lane);
    softmax_col(P, scale);
    if constexpr (DROP) drop_scale(P, kmask, kscale);
    f32x16 O = f32x16{0};
#pragma unroll
    for (int jt = 0; jt < 2; ++jt)
#pragma unroll
      for (int sb = 0; sb < 2; ++sb) O = mfma32<T>(frag_tr_perm(Lv, LD, jt * 32 + 16 * sb, 0, lane), pack8<T>(P[jt], sb), O);
    // output through this tile's q rows (read only by this wave)
    bf16_t* Lo = L.qkv[h][0];
    const int i = t * 32 + (lane & 31);
#pragma unroll
    for (int gq = 0; gq < 4; ++gq) {
      uint2 wv;
      wv.x = pack2<T>(O[4 * gq], O[4 * gq + 1]);
      wv.y = pack2<T>(O[4 * gq + 2], O[4 * gq + 3]);
      *reinterpret_cast<uint2*>(Lo + i * LD + 8 * gq + 4 * hh) = wv;
    }
    lds_sync();
    bf16_t* const odst = PROJ ? o_out : out;
    if (!PROJ || o_out != nullptr) {
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const int r = 32 * t + read_row(lane >> 2) + 16 * c;
        const int tok = L.tok[r];
        const u32x4 v = *reinterpret_cast<const u32x4*>(Lo + r * LD + 8 * (lane & 3));
        if (tok >= 0)
          *reinterpret_cast<u32x4*>(odst + (size_t)((unsigned)tok * (unsigned)FQ_C) + h * HD + 8 * (lane & 3)) = v;
      }
    }
    if (DROP && keep_out) keep_out[((size_t)win * g.nh + h) * 128 + 64 * t + lane] = kmask;
    if constexpr (PROJ) {
      __syncthreads();  // o of every head in LDS (q image rows)
      // y[token][n] = sum_d o[token][d] W_proj[n][d] + b: wave -> (token tile t, n tile h); the
      // k steps of 16 d walk the heads' o images (d = 32 h' + 16 (ks & 1) + ...)
      f32x16 ya = f32x16{0};
#pragma unroll
      for (int ks = 0; ks < FQ_C / 16; ++ks) {
        const bf16x8 of = frag_rows(L.qkv[ks >> 1][0], LD, 32 * t, 16 * (ks & 1), lane);
        ya = mfma32<T>(fq_frag(L.wp, 32 * h, ks, lane), of, ya);
      }
      // + bias, rows of the output image (the LN1 rows' buffer, free since the qkv GEMM)
      const int tk2 = 32 * t + (lane & 31);
#pragma unroll
      for (int gq = 0; gq < 4; ++gq) {
        const int n = 32 * h + 8 * gq + 4 * hh;
        const float4 b = *reinterpret_cast<const float4*>(L.pbias + n);
        uint2 wv;
        wv.x = pack2<T>(ya[4 * gq] + b.x, ya[4 * gq + 1] + b.y);
        wv.y = pack2<T>(ya[4 * gq + 2] + b.z, ya[4 * gq + 3] + b.w);
        // chunk n / 8 of row tk2, 8-B half 4hh / 4 of it (swizzled chunks as the LN1 rows)
        *reinterpret_cast<uint2*>(L.x + tk2 * FQ_C + (((n >> 3) ^ fq_swz(tk2)) << 3) + 4 * hh) = wv;
      }
      __syncthreads();
#pragma unroll
      for (int k = 0; k < XS; ++k) {
        const int s = tid + NTHR * k;
        const int r = s / FQ_CH, c = s - (s / FQ_CH) * FQ_CH;
        if (s < 64 * FQ_CH) {
          const int tok = L.tok[r];
          const u32x4 v = *reinterpret_cast<const u32x4*>(L.x + r * FQ_C + ((c ^ fq_swz(r)) << 3));
          if (tok >= 0) *reinterpret_cast<u32x4*>(out + (size_t)((unsigned)tok * (unsigned)FQ_C) + 8 * c) = v;
        }
      }
    }
    __syncthreads();  // every wave done with this window's images before the next is staged
  }
}

int num_cus_fq() {
  static const int cus = [] {
    int n = 0, dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
    return n;
  }();
  return cus;
}

template <typename T, bool DROP, bool STORE_QKV, bool PROJ>
void launch_fq(dim3 grid, const void* x, const void* w, const float* b, const Aux& aux, void* out, void* qkv, Geom g,
               float scale, float p_drop, unsigned long long seed, const unsigned long long* seed_dev, void* keep,
               const void* wp, const float* bp, void* o_out, hipStream_t st) {
  auto kern = attn_qkv_fwd_mfma<T, DROP, STORE_QKV, PROJ>;
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)sizeof(FusedLds));
    attr_set = true;
  }
  hipLaunchKernelGGL(kern, grid, dim3(64 * FQ_WAVES), sizeof(FusedLds), st, (const bf16_t*)x, (const bf16_t*)w, b, aux,
                     (bf16_t*)out, (bf16_t*)qkv, g, scale, p_drop, (uint64_t)seed, seed_dev, (uint32_t*)keep,
                     (const bf16_t*)wp, bp, (bf16_t*)o_out);
}

template <typename T, bool PROJ>
void launch_fq4(dim3 grid, const void* x, const void* w, const float* b, const Aux& aux, void* out, void* qkv, Geom g,
                float scale, float p_drop, unsigned long long seed, const unsigned long long* seed_dev, void* keep,
                const void* wp, const float* bp, void* o_out, hipStream_t st) {
  const bool drop = p_drop > 0.f;
  if (drop && qkv) launch_fq<T, true, true, PROJ>(grid, x, w, b, aux, out, qkv, g, scale, p_drop, seed, seed_dev, keep, wp, bp, o_out, st);
  else if (drop) launch_fq<T, true, false, PROJ>(grid, x, w, b, aux, out, qkv, g, scale, p_drop, seed, seed_dev, keep, wp, bp, o_out, st);
  else if (qkv) launch_fq<T, false, true, PROJ>(grid, x, w, b, aux, out, qkv, g, scale, p_drop, seed, seed_dev, keep, wp, bp, o_out, st);
  else launch_fq<T, false, false, PROJ>(grid, x, w, b, aux, out, qkv, g, scale, p_drop, seed, seed_dev, keep, wp, bp, o_out, st);
}

}  // namespace

extern "C" {

// Whether msu_win_attn_qkv_fwd covers a block of width C with nh heads (16-bit only).
int msu_win_attn_qkv_supported(int C, int nh) { return C == FQ_C && nh == FQ_NH ? 1 : 0; }

// Fused qkv Linear + window attention (stage 0): out[B,H,W,C] = attention(x W_qkv^T + b_qkv);
// x = LN1 rows [B,H,W,C] 16-bit, W_qkv [3C][C] 16-bit, b_qkv f32; qkv_out [B,H,W,3C] (x W^T + b,
// what the qkv Linear would store) or null; keep / dropout / seeds and the aux workspace
// (msu_win_attn_fwd_workspace) as msu_win_attn_fwd.
int msu_win_attn_qkv_fwd2(int dtype, const void* x, const void* w_qkv, const float* b_qkv, const float* table,
                          const void* w_proj, const float* b_proj, void* out, void* o_out, void* qkv_out, void* keep,
                          float* workspace, int B, int H, int W, int C, int nh, int shift, float p_drop,
                          unsigned long long seed, const unsigned long long* seed_dev, void* stream) {
  if (!msu_is16(dtype) || !msu_win_attn_qkv_supported(C, nh)) return -2;
  if ((long)B * H * W * 3 * C >= (1L << 32)) return -2;
  const Geom g = make_geom(B, H, W, C, nh, shift);
  if (g.nwin == 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  const float scale = 1.0f / sqrtf((float)HD);
  float* img; bf16_t* brow; bf16_t* zrow;
  const Aux aux = carve_aux(workspace, C, nh, &img, &brow, &zrow);
  const long nb = g.nwin < num_cus_fq() ? g.nwin : num_cus_fq();
  const dim3 grid((unsigned)nb);
  if ((w_proj == nullptr) != (b_proj == nullptr)) return -3;
  MSU_DISPATCH16(dtype, T,
    hipLaunchKernelGGL(aux_kernel<T>, dim3((nh * 4096 + 255) / 256), dim3(256), 0, st, table, b_qkv, nh, 3 * C,
                       1.0f / scale, img, brow, zrow);
    if (w_proj) launch_fq4<T, true>(grid, x, w_qkv, b_qkv, aux, out, qkv_out, g, scale, p_drop, seed, seed_dev, keep,
                                    w_proj, b_proj, o_out, st);
    else launch_fq4<T, false>(grid, x, w_qkv, b_qkv, aux, out, qkv_out, g, scale, p_drop, seed, seed_dev, keep,
                              nullptr, nullptr, nullptr, st));
  return MSU_CHECK_LAUNCH();
}

int msu_win_attn_qkv_fwd(int dtype, const void* x, const void* w_qkv, const float* b_qkv, const float* table,
                         void* out, void* qkv_out, void* keep, float* workspace, int B, int H, int W, int C, int nh,
                         int shift, float p_drop, unsigned long long seed, const unsigned long long* seed_dev,
                         void* stream) {
  return msu_win_attn_qkv_fwd2(dtype, x, w_qkv, b_qkv, table, nullptr, nullptr, out, nullptr, qkv_out, keep, workspace,
                               B, H, W, C, nh, shift, p_drop, seed, seed_dev, stream);
}

}  // extern "C"
