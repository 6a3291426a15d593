// ------------------------------------------------------------------ 16-bit fwd, v5 (C = 96)
// (included by conv3x3.h after the v3 kernel; same helpers, same Wt / halo layouts)
//
// v3 re-stages a tap's [96][96] weight image by LDS-DMA before every tap, one barrier per tap,
// and its next-tile halo loads share the in-order vmcnt with those DMAs: each halo part has ~2
// taps of latency budget and the loads cost 25 % of a launch (r05j/k ablations); the epilogue's
// stores drain before the next tile.  v5 keeps the weights resident instead: a workgroup owns
// one half of the output channels (48), whose 9 x 48 x 96 weights (81 KB) stay in LDS for the
// whole launch beside a 10 x 34 pixel halo (64 KB) of an 8 x 32 output tile.  A tile's nine taps
// then run without a barrier; the next tile's halo loads are issued at the tile's start (a whole
// tile of latency budget) and the output stores leave while the next tile computes.
//   * workgroups b and b + 8 run on one XCD (round-robin dispatch) and take the two channel halves
//     of the same tiles in the same order, so the second halo read of a tile is an L2 hit;
//   * wave w owns output row w: 2 pixel tiles x 3 channel tiles of 16x16x32 MFMAs, 18 per tap;
//   * fragment reads per tap and wave: 6 pixel + 9 weight (ds_read_b128, conflict-free (p >> 1) & 3
//     swizzle of v3's M16 form), the LDS at ~0.8 of its peak when the MFMAs run at theirs.
// Epilogue: channel tiles 0 / 1 paired by permlane16 swap (16-B stores of 8 channels), tile 2 as
// 8-B stores of 4 channels; bias from LDS; DUAL as v3; backward data (OUT_GGRAD): times
// GELU'(S) of the output pixels, S loaded at the tile's start (registers are plentiful here, v3's
// dgrad had to stay on 32x32x16 MFMAs for them).
template <typename T, bool IN_D2S, bool OUT_D2S, bool OUT_GGRAD, bool BIAS, bool DUAL>
__global__ void __launch_bounds__(512) conv3x3_v5_kernel(const bf16_t* __restrict__ X,
                                                         const bf16_t* __restrict__ Wt,
                                                         const float* __restrict__ bias,
                                                         const bf16_t* __restrict__ S, bf16_t* __restrict__ Y,
                                                         bf16_t* __restrict__ Y2, ConvGeom g, int ntiles) {
  constexpr int C = 96, CH = 12, NW = 8, TH = NW, TWV = 32, HWD = TWV + 2;
  constexpr int HPIX = (TH + 2) * HWD;              // 340 halo pixels
  constexpr int CO = 48;                            // output channels of a workgroup
  constexpr int WROWS = 9 * CO;                     // weight rows (tap, channel)
  constexpr int WINS = WROWS * CH / 64;             // 81 DMA wave-instructions
  static_assert(WINS * 64 == WROWS * CH, "weight image in whole DMA instructions");
  constexpr int NTHR = 64 * NW;
  constexpr int PSTEP = NTHR / CH;                  // halo pixels per staging round
  constexpr int NHC = (HPIX + PSTEP - 1) / PSTEP;   // staging rounds (9)

  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  bf16_t* sW = reinterpret_cast<bf16_t*>(smem_raw);  // [432][96]
  bf16_t* sX = sW + WROWS * C;                       // [340][96]
  float* sB = reinterpret_cast<float*>(sX + HPIX * C);  // [48]
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int half = (blockIdx.x >> 3) & 1;
  const int pair = (blockIdx.x & 7) + 8 * (blockIdx.x >> 4);
  const int npairs = gridDim.x >> 1;  // the grid is a multiple of 16
  const int tiles_x = (g.W + TWV - 1) / TWV, tiles_y = (g.H + TH - 1) / TH;
  const int per_img = tiles_x * tiles_y;
  int tile = pair;
  if (tile >= ntiles) return;  // both workgroups of a pair

  auto coords = [&](int t, int& b, int& y0, int& x0) {
    b = t / per_img;
    const int r = t - b * per_img;
    y0 = (r / tiles_x) * TH;
    x0 = (r - (r / tiles_x) * tiles_x) * TWV;
  };
  // halo staging as v3: thread t < 12 PSTEP owns channel chunk t % 12 of pixels t / 12 + PSTEP c
  u32x4 hr[NHC];
  auto load_halo = [&](int t) __attribute__((always_inline)) {
    int b, y0, x0;
    coords(t, b, y0, x0);
    const int u = opaque(tid);
    const bool hact = u < PSTEP * CH;
    int p = u / CH;
    int row = p / HWD, col = p - (p / HWD) * HWD;
    const bf16_t* xc = X + (u % CH) * 8;
#pragma unroll
    for (int c = 0; c < NHC; ++c) {
      const int y = y0 - 1 + row, x = x0 - 1 + col;
      const bool ok = hact && p < HPIX && (unsigned)y < (unsigned)g.H && (unsigned)x < (unsigned)g.W;
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
  auto store_halo = [&]() __attribute__((always_inline)) {
    const int u = opaque(tid);
    const bool hact = u < PSTEP * CH;
    const int hch = u % CH;
    int p = u / CH;
#pragma unroll
    for (int c = 0; c < NHC; ++c) {
      if (hact && p < HPIX) *reinterpret_cast<u32x4*>(sX + p * C + ((hch ^ swzv<true>(p)) << 3)) = hr[c];
      p += PSTEP;
    }
  };

  // resident weights of this channel half: LDS row r = tap * 48 + co' <- Wt row tap * 96 + 48 half + co'
  // (slot q = 64 k + lane: row q / 12, chunk position q % 12 holds chunk pos ^ swz(row))
  for (int k = wave; k < WINS; k += NW) {
    const int q = 64 * k + lane;
    const int r = q / CH, pos = q - (q / CH) * CH;
    const int tap = r / CO, co = r - (r / CO) * CO;
    glds16(Wt + ((long)tap * C + CO * half + co) * C + ((pos ^ swzv<true>(r)) << 3), sW + 512 * k);
  }
  if constexpr (BIAS) {
    if (tid < CO) sB[tid] = bias[CO * half + tid];
  }
  load_halo(tile);
  store_halo();
  wait_vmcnt<0>();
  __syncthreads();

  const int l15 = lane & 15, g4 = lane >> 4;
  const int wk16 = l15 * C + ((g4 ^ swzv<true>(l15)) << 3);  // weight row 16 n + l15 of a tap
  const int cofs = 16 * (g4 & 1) + 8 * (g4 >> 1);            // epilogue: channels after the swap
  // pixel-fragment lane offsets of every (tap, pixel tile): halo row wave + dy, pixels dx + 16 pt
  // + l15 -- the same for every tile, computed once (18 registers)
  int xq[9][2];
#pragma unroll
  for (int tap = 0; tap < 9; ++tap)
#pragma unroll
    for (int pt = 0; pt < 2; ++pt) {
      const int p = (wave + tap / 3) * HWD + tap % 3 + 16 * pt + l15;
      xq[tap][pt] = p * C + ((g4 ^ swzv<true>(p)) << 3);
    }

  for (; tile < ntiles; tile += npairs) {
    const int next = tile + npairs;
    int b, y0, x0;
    coords(tile, b, y0, x0);
    const int co0 = CO * half;
    // dgrad: this tile's pre-activations for the GELU' epilogue (lane: its pixel of each pixel
    // tile, the channels it stores), then the next tile's halo; both in flight through the taps
    u32x4 s8[OUT_GGRAD ? 2 : 1];
    u32x2 s4[OUT_GGRAD ? 2 : 1];
    if constexpr (OUT_GGRAD) {
#pragma unroll
      for (int pt = 0; pt < 2; ++pt) {
        const int px = min(x0 + 16 * pt + l15, g.W - 1), y = min(y0 + wave, g.H - 1);
        const bf16_t* sp = S + pix_off32<OUT_D2S>(b, y, px, g.H, g.W, C) + co0;
        s8[pt] = *reinterpret_cast<const u32x4*>(sp + cofs);
        s4[pt] = *reinterpret_cast<const u32x2*>(sp + 32 + 4 * g4);
      }
    }
    if (next < ntiles) load_halo(next);  // in flight through all nine taps
    f32x4 acc[2][3];
#pragma unroll
    for (int pt = 0; pt < 2; ++pt)
#pragma unroll
      for (int n = 0; n < 3; ++n) acc[pt][n] = f32x4{0.f, 0.f, 0.f, 0.f};
    // 27 steps (tap, k step), software pipelined: the fragments of step s + 1 are read while
    // the six MFMAs of step s run (two register sets)
    bf16x8 xf[2][2], wf[2][3];
    auto rd = [&](auto SI, auto SET) __attribute__((always_inline)) {
      constexpr int st = decltype(SI)::value, set = decltype(SET)::value;
      constexpr int tap = st / 3, ks = st % 3;
      if constexpr (MSU_EXP & 1024) {  // ablation: no fragment reads (results wrong)
#pragma unroll
        for (int pt = 0; pt < 2; ++pt) xf[set][pt] = __builtin_bit_cast(bf16x8, u32x4{(uint32_t)xq[tap][pt], 1u, 2u, (uint32_t)ks});
#pragma unroll
        for (int n = 0; n < 3; ++n) wf[set][n] = __builtin_bit_cast(bf16x8, u32x4{(uint32_t)wk16, (uint32_t)n, 3u, (uint32_t)tap});
        return;
      }
#pragma unroll
      for (int pt = 0; pt < 2; ++pt) xf[set][pt] = *reinterpret_cast<const bf16x8*>(sX + xq[tap][pt] + 32 * ks);
#pragma unroll
      for (int n = 0; n < 3; ++n)
        wf[set][n] = *reinterpret_cast<const bf16x8*>(sW + tap * CO * C + wk16 + 16 * n * C + 32 * ks);
    };
    rd(IC<0>{}, IC<0>{});
    static_for([&](auto SI) {
      constexpr int st = decltype(SI)::value, cur = st & 1;
      if constexpr (st + 1 < 27) rd(IC<st + 1>{}, IC<cur ^ 1>{});
#pragma unroll
      for (int n = 0; n < 3; ++n)
#pragma unroll
        for (int pt = 0; pt < 2; ++pt) {
          if constexpr (MSU_EXP & 2048) asm volatile("" ::"v"(wf[cur][n]), "v"(xf[cur][pt]));  // ablation: no MFMA
          else acc[pt][n] = Fmt16<T>::mma16(wf[cur][n], xf[cur][pt], acc[pt][n]);
        }
      __builtin_amdgcn_sched_barrier(0);
    }, std::make_integer_sequence<int, 27>{});

    // every wave done reading this tile's halo: the next one goes in (its loads have had the
    // whole tile); this tile's output stores then leave while the next tile computes
    if (next < ntiles) {
      __syncthreads();
      store_halo();
    }
#pragma unroll
    for (int pt = 0; pt < 2; ++pt) {
      const int px = x0 + 16 * pt + l15;
      const int y = y0 + wave;
      const bool ok = px < g.W && y < g.H;
      const int off = ok ? pix_off32<OUT_D2S>(b, y, px, g.H, g.W, C) + co0 : 0;
      {  // channel tiles 0, 1: 8 consecutive channels cofs .. cofs + 7 per lane
        float v[8];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(acc[pt][0][i]),
                                                          __float_as_uint(acc[pt][1][i]), false, false);
          v[i] = __uint_as_float(r[0]);
          v[4 + i] = __uint_as_float(r[1]);
        }
        if constexpr (BIAS) {
#pragma unroll
          for (int i = 0; i < 8; ++i) v[i] += sB[cofs + i];
        }
        if constexpr (OUT_GGRAD) {
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            v[2 * i] *= gelu_grad_fast(Fmt16<T>::lo(s8[pt][i]));
            v[2 * i + 1] *= gelu_grad_fast(Fmt16<T>::hi(s8[pt][i]));
          }
        }
        const u32x4 pk = {pack2<T>(v[0], v[1]), pack2<T>(v[2], v[3]), pack2<T>(v[4], v[5]), pack2<T>(v[6], v[7])};
        if (ok) {
          *reinterpret_cast<u32x4*>(Y + off + cofs) = pk;
          if constexpr (DUAL) *reinterpret_cast<u32x4*>(Y2 + off + cofs) = gelu8<T>(pk);
        }
      }
      {  // channel tile 2: channels 32 + 4 g4 .. + 3
        float v[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] = acc[pt][2][i] + (BIAS ? sB[32 + 4 * g4 + i] : 0.f);
        if constexpr (OUT_GGRAD) {
#pragma unroll
          for (int i = 0; i < 2; ++i) {
            v[2 * i] *= gelu_grad_fast(Fmt16<T>::lo(s4[pt][i]));
            v[2 * i + 1] *= gelu_grad_fast(Fmt16<T>::hi(s4[pt][i]));
          }
        }
        const u32x2 pk = {pack2<T>(v[0], v[1]), pack2<T>(v[2], v[3])};
        if (ok) {
          *reinterpret_cast<u32x2*>(Y + off + 32 + 4 * g4) = pk;
          if constexpr (DUAL) {
            const u32x4 gq = gelu8<T>(u32x4{pk[0], pk[1], 0u, 0u});
            *reinterpret_cast<u32x2*>(Y2 + off + 32 + 4 * g4) = u32x2{gq[0], gq[1]};
          }
        }
      }
    }
    if (next < ntiles) __syncthreads();  // the next tile's halo visible to every wave
  }
}

template <typename T, bool IN_D2S, bool OUT_D2S, bool OUT_GGRAD, bool BIAS, bool DUAL>
int launch_v5(const ConvGeom& g, const bf16_t* X, const bf16_t* Wt, const float* bias, const bf16_t* S, bf16_t* Y,
              bf16_t* Y2, hipStream_t st) {
  constexpr size_t lds = sizeof(bf16_t) * ((size_t)9 * 48 * 96 + 10 * 34 * 96) + 48 * sizeof(float);
  static_assert(lds <= 160 * 1024, "LDS");
  auto kern = conv3x3_v5_kernel<T, IN_D2S, OUT_D2S, OUT_GGRAD, BIAS, DUAL>;
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr_set = true;
  }
  const long ntiles = (long)g.B * ((g.W + 31) / 32) * ((g.H + 7) / 8);
  if (ntiles == 0) return 0;
  if ((long)g.B * g.H * g.W * 96 >= (1L << 31) || ntiles >= (1L << 30)) return -2;
  // pairs of workgroups (b, b + 8) on one XCD: a multiple of 16, at most one per CU
  long grid = (long)num_cus() / 16 * 16;
  const long need = (2 * ntiles + 15) / 16 * 16;
  if (grid > need) grid = need;
  if (grid < 16) grid = 16;
  hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(512), lds, st, X, Wt, bias, S, Y, Y2, g, (int)ntiles);
  return MSU_CHECK_LAUNCH();
}
