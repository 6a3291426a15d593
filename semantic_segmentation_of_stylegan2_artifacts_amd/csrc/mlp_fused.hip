// Stage-0 Swin MLP forward in ONE kernel (torchvision MLP, model_parts.py:538):
//
//   y = mlp.3(GELU(mlp.0(x)))      x, y: [M][96], hidden 384
//
// Without autograd (the reference's discarded branches layers_cent1[-1] / layers_cent2[-1] at
// model_parts.py:795 / :807, and evaluation) the 384-wide hidden activation never leaves the
// chip: the GEMM pair wrote GELU(H) (403 MB at 8 x 256^2 tokens) and read it back.  In training
// (H_OUT) the kernel also stores the pre-activation H -- the one tensor the backward needs (mlp.3's
// input gradient applies GELU'(H), its weight gradient re-derives GELU(H) from H while staging:
// msu_linear_bwd with X = null); the pair wrote H and GELU(H) and read GELU(H) back.
// Per 32-token tile and per 32-wide hidden chunk a wave runs
//   * fc1 on MFMA with W1 as the A operand and the tile's token rows as B (the tokens end up on
//     the accumulator columns, the hidden units on its rows), + b1, rounded to 16 bits, GELU
//     (the unfused epilogue's arithmetic: gelu_fast of the rounded pre-activation), rounded
//     again and packed -- each lane's 16 values are directly the B operand of
//   * fc2 (y^T += W2[:, chunk] . G^T[chunk, :]), whose A fragments are read from W2 rows in the
//     accumulator's row order (two 8-B pieces per fragment), three 32-channel output tiles.
// W1 [384][96] (16-B chunks swizzled c ^ ((r >> 2) & 3): conflict-free 32-row fragment reads)
// and W2 [96][388] (194-dword rows: the 32 rows of a ds_read_b64 half-wave fill the 64 banks
// once) stay in LDS for the workgroup's life; the token rows come from HBM straight into
// registers one tile ahead.  One 8-wave workgroup per CU (150 KB of LDS), two waves per SIMD:
// the GELU of one overlaps the other's MFMAs.
#include "common.h"

namespace {

constexpr int MC = 96, MH = 384, MT = 32, MW = 8;
constexpr int LW2 = MH + 4;

struct MlpLds {
  bf16_t w1[MH * MC];
  bf16_t w2[MC * LW2];
  float b1[MH];
  float b2[MC];
};

MSU_DEV int w1_swz(int r) { return (r >> 2) & 3; }

// accumulator row of register r for lane half h (32x32 C layout)
MSU_DEV constexpr int acc_row(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

template <typename T, bool H_OUT>
__global__ void __launch_bounds__(64 * MW) mlp_fused_kernel(const bf16_t* __restrict__ x, const bf16_t* __restrict__ w1,
                                                          const float* __restrict__ b1, const bf16_t* __restrict__ w2,
                                                          const float* __restrict__ b2, bf16_t* __restrict__ y,
                                                          bf16_t* __restrict__ hout, long M) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  MlpLds& L = *reinterpret_cast<MlpLds*>(smem_raw);
  const int tid = threadIdx.x, lane = tid & 63, hh = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  for (int s = tid; s < MH * (MC / 8); s += 64 * MW) {
    const int r = s / (MC / 8), c = s % (MC / 8);
    *reinterpret_cast<u32x4*>(L.w1 + r * MC + ((c ^ w1_swz(r)) << 3)) = *reinterpret_cast<const u32x4*>(w1 + r * MC + 8 * c);
  }
  for (int s = tid; s < MC * (MH / 8); s += 64 * MW) {
    const int r = s / (MH / 8), c = s % (MH / 8);
    const u32x4 v = *reinterpret_cast<const u32x4*>(w2 + r * MH + 8 * c);
    // 8-B aligned rows (388 elements): two 8-B stores
    *reinterpret_cast<u32x2*>(L.w2 + r * LW2 + 8 * c) = u32x2{v.x, v.y};
    *reinterpret_cast<u32x2*>(L.w2 + r * LW2 + 8 * c + 4) = u32x2{v.z, v.w};
  }
  for (int s = tid; s < MH; s += 64 * MW) L.b1[s] = b1[s];
  for (int s = tid; s < MC; s += 64 * MW) L.b2[s] = b2[s];
  __syncthreads();

  const long ntiles = (M + MT - 1) / MT;
  const long stride = (long)gridDim.x * MW;
  long tile = (long)blockIdx.x * MW + wave;
  if (tile >= ntiles) return;  // no block-wide barriers after this point
  const int tl = lane & 31;
  // token rows of a tile as the fc1 B operand: lane (token tl, half hh) holds k = 16 ks + 8 hh .. + 7
  auto load_x = [&](long t, u32x4 (&xr)[6]) __attribute__((always_inline)) {
    const long row = t * MT + tl;
    const bool ok = row < M;
    const bf16_t* p = x + (ok ? row : 0) * MC + 8 * hh;
#pragma unroll
    for (int ks = 0; ks < 6; ++ks) {
      const u32x4 v = *reinterpret_cast<const u32x4*>(p + 16 * ks);
      xr[ks] = ok ? v : u32x4{0u, 0u, 0u, 0u};
    }
  };
  u32x4 xc[6], xn[6];
  load_x(tile, xc);
  // fc2 A fragment of output tile ct, hidden k step n0 .. n0 + 15 in the accumulator row order:
  // element e of half hh <-> hidden n0 + 8 (e >> 2) + 4 hh + (e & 3)
  const bf16_t* w2row = L.w2 + tl * LW2 + 4 * hh;
  for (;;) {
    const long nxt = tile + stride;
    const bool more = nxt < ntiles;
    if (more) load_x(nxt, xn);
    f32x16 yacc[3];
#pragma unroll
    for (int ct = 0; ct < 3; ++ct) yacc[ct] = f32x16{0};
    const long hrow_i = tile * MT + tl;
    const bool hok = hrow_i < M;
    bf16_t* hrow = H_OUT ? hout + (hok ? hrow_i : 0) * MH : nullptr;
#pragma unroll(H_OUT ? 1 : 2)
    for (int nc = 0; nc < MH / 32; ++nc) {
      // fc1: C1^T[n][t] for hidden n in chunk nc
      f32x16 h = f32x16{0};
      const int wr = nc * 32 + tl;
#pragma unroll
      for (int ks = 0; ks < 6; ++ks) {
        const bf16x8 wf = *reinterpret_cast<const bf16x8*>(L.w1 + wr * MC + (((2 * ks + hh) ^ w1_swz(wr)) << 3));
        h = Fmt16<T>::mma32(wf, __builtin_bit_cast(bf16x8, xc[ks]), h);
      }
      // + b1, 16-bit pre-activation, GELU, 16-bit activation (the unfused epilogues' roundings)
      uint32_t g[8], hw[8];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float4 bq = *reinterpret_cast<const float4*>(L.b1 + nc * 32 + 8 * q + 4 * hh);
        const float u0 = round16<T>(h[4 * q] + bq.x), u1 = round16<T>(h[4 * q + 1] + bq.y);
        const float u2 = round16<T>(h[4 * q + 2] + bq.z), u3 = round16<T>(h[4 * q + 3] + bq.w);
        if constexpr (H_OUT) {
          hw[2 * q] = pack2<T>(u0, u1);
          hw[2 * q + 1] = pack2<T>(u2, u3);
        }
        g[2 * q] = pack2<T>(gelu_fast(u0), gelu_fast(u1));
        g[2 * q + 1] = pack2<T>(gelu_fast(u2), gelu_fast(u3));
      }
      if constexpr (H_OUT) {
        // H row piece: a permlane32 swap pairs the halves' 4-unit groups into 8 consecutive
        // hidden units per lane (hidden nc*32 + 16p + 8hh .. + 7), one 16-B store each
#pragma unroll
        for (int p = 0; p < 2; ++p) {
          const auto s0 = __builtin_amdgcn_permlane32_swap(hw[4 * p], hw[4 * p + 2], false, false);
          const auto s1 = __builtin_amdgcn_permlane32_swap(hw[4 * p + 1], hw[4 * p + 3], false, false);
          const u32x4 v = {s0[0], s1[0], s0[1], s1[1]};
          if (hok) *reinterpret_cast<u32x4*>(hrow + nc * 32 + 16 * p + 8 * hh) = v;
        }
      }
      // fc2: two 16-deep k steps over the chunk (registers 8s .. 8s + 7 of the fc1 accumulator)
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const bf16x8 gb = __builtin_bit_cast(bf16x8, u32x4{g[4 * s], g[4 * s + 1], g[4 * s + 2], g[4 * s + 3]});
        const int n0 = nc * 32 + 16 * s;
#pragma unroll
        for (int ct = 0; ct < 3; ++ct) {
          const bf16_t* a = w2row + ct * 32 * LW2 + n0;
          const u32x2 lo = *reinterpret_cast<const u32x2*>(a);
          const u32x2 hi = *reinterpret_cast<const u32x2*>(a + 8);
          const bf16x8 af = __builtin_bit_cast(bf16x8, u32x4{lo.x, lo.y, hi.x, hi.y});
          yacc[ct] = Fmt16<T>::mma32(af, gb, yacc[ct]);
        }
      }
    }
    // y[t][c] = y^T + b2: lane (token tl) holds channels 32 ct + 8 q + 4 hh + i in register 4q + i;
    // a permlane32 swap pairs the halves' 4-channel groups into 8 consecutive channels per
    // lane, so every store is one 16-B piece (every lane executes the swaps)
    const long row = tile * MT + tl;
    const bool ok = row < M;
    bf16_t* yr = y + (ok ? row : 0) * MC;
#pragma unroll
    for (int ct = 0; ct < 3; ++ct) {
      uint32_t w[8];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float4 bq = *reinterpret_cast<const float4*>(L.b2 + ct * 32 + 8 * q + 4 * hh);
        w[2 * q] = pack2<T>(yacc[ct][4 * q] + bq.x, yacc[ct][4 * q + 1] + bq.y);
        w[2 * q + 1] = pack2<T>(yacc[ct][4 * q + 2] + bq.z, yacc[ct][4 * q + 3] + bq.w);
      }
#pragma unroll
      for (int p = 0; p < 2; ++p) {
        const auto s0 = __builtin_amdgcn_permlane32_swap(w[4 * p], w[4 * p + 2], false, false);
        const auto s1 = __builtin_amdgcn_permlane32_swap(w[4 * p + 1], w[4 * p + 3], false, false);
        const u32x4 v = {s0[0], s1[0], s0[1], s1[1]};
        if (ok) *reinterpret_cast<u32x4*>(yr + ct * 32 + 16 * p + 8 * hh) = v;
      }
    }
    if (!more) break;
    tile = nxt;
#pragma unroll
    for (int ks = 0; ks < 6; ++ks) xc[ks] = xn[ks];
  }
}

int num_cus_mlp() {
  static const int cus = [] {
    int n = 0, dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
    return n;
  }();
  return cus;
}

template <typename T, bool H_OUT>
int launch_mlp(const void* x, const void* w1, const float* b1, const void* w2, const float* b2, void* y, void* h,
               long M, hipStream_t st) {
  auto kern = mlp_fused_kernel<T, H_OUT>;
  static bool attr_set = false;
  if (!attr_set) {
    if (hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)sizeof(MlpLds)) !=
        hipSuccess)
      return -4;
    attr_set = true;
  }
  const long ntiles = (M + MT - 1) / MT;
  long grid = num_cus_mlp();
  if (grid * MW > ntiles) grid = (ntiles + MW - 1) / MW;
  hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(64 * MW), sizeof(MlpLds), st, (const bf16_t*)x,
                     (const bf16_t*)w1, b1, (const bf16_t*)w2, b2, (bf16_t*)y, (bf16_t*)h, M);
  return MSU_CHECK_LAUNCH();
}

}  // namespace

extern "C" {

// Whether msu_mlp_fused_fwd covers a (channels, hidden) shape: the stage-0 MLP, 96 -> 384 -> 96.
int msu_mlp_fused_supported(int C, int Hd) { return C == MC && Hd == MH ? 1 : 0; }

// y = fc2(GELU(fc1(x))) with the hidden activation kept on chip; h (nullable) receives the
// 16-bit pre-activation fc1(x) [M][384] for the backward.  dtype bf16 / f16; x, y [M][96]
// (16-B aligned rows), w1 [384][96], w2 [96][384] in x's format, b1 [384] / b2 [96] f32.
int msu_mlp_fused_fwd(int dtype, const void* x, const void* w1, const float* b1, const void* w2, const float* b2,
                      void* y, void* h, long M, int C, int Hd, void* stream) {
  if (!msu_is16(dtype) || !msu_mlp_fused_supported(C, Hd) || M < 0) return -2;
  if ((((uintptr_t)x | (uintptr_t)y | (uintptr_t)h | (uintptr_t)w1 | (uintptr_t)w2 | (uintptr_t)b1 | (uintptr_t)b2) &
       15) != 0)
    return -2;
  if (M == 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  if (h != nullptr) {
    MSU_DISPATCH16(dtype, T, return launch_mlp<T, true>(x, w1, b1, w2, b2, y, h, M, st));
  } else {
    MSU_DISPATCH16(dtype, T, return launch_mlp<T, false>(x, w1, b1, w2, b2, y, h, M, st));
  }
  return -3;
}

}  // extern "C"
