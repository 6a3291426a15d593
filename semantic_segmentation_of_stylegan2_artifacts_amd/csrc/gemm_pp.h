// Ping-pong 16-bit NT GEMM for the stage 1-3 Linears (included by gemm_nt.hip; same NtArgs and
// epilogues as gemm_nt_kernel except GELU'): Y[M][N] = epi(A[M][K] . W[N][K]^T + bias), f32 accumulation.
//
// Why another form: the persistent 2-barrier kernel (gemm_nt_kernel) runs its two waves per SIMD
// in lockstep -- both reach every barrier together, both read LDS together, both issue MFMAs
// together -- and keeps the MFMA pipe busy 25 % of the time (r04i counters at 32768 x 1152 x
// 384: 623 TF/s).  Here the 8 waves form two groups of four, one wave of each group per SIMD
// (waves w and w + 4 share a SIMD), and group 1 runs one barrier behind group 0: between any two
// barriers one group issues MFMAs while the other reads its next fragments from LDS and issues
// its share of the LDS-DMA prefetch, so each SIMD has one wave feeding its matrix pipe while the
// other loads (the 8-phase schedule of cdna_hip_programming.md section 5, "The 256^2 8-phase
// template", in two phases per K-step).
//
// Tile BM x BN = 256 x 256 (N % 256 == 0) or 256 x 192; group g owns output columns
// [g BN/2, (g+1) BN/2), its wave q the rows [64 q, 64 q + 64): a 64 x BN/2 wave tile of 16x16x32
// MFMAs computed transposed (W rows on the accumulator rows, tokens on the lanes), so after a
// permlane16 swap each lane stores 8 consecutive columns of its token row (16-B stores).
// A K-step (64) is two phases (k-slice 0 / 1), 4 x BN/32 MFMAs each.  The K-step halves
// h_j = [A k-slice][W k-slice] ([rows][32 k] images, 64-B rows, XOR-swizzled 16-B chunks, filled by
// global_load_lds_dwordx4) live in a ring of four LDS slots.  Load slot k (the k-th phase of the
// workgroup) issues h_{k+3} into the slot h_{k-1} left (read in load slot k - 1, its lgkmcnt(0)
// before that slot's barrier), waits for its own share of h_{k+1} (read in the NEXT load slot,
// after a barrier every wave passes after its wait: DMA data written by all eight waves is read
// one phase after the waits that retire it) and reads h_k: every half has two slots to land.
// Every wait is a counted vmcnt with compile-time counts (the waves' DMA shares differ at BN =
// 192), never 0 in the loop but for the last three phases.
// The workgroup is persistent over its tiles (XCD-contiguous tile ranges; the DMA stream runs
// across tile boundaries); a tile's epilogue runs in the load slot of the next tile's first
// phase, its bias staged into LDS (one DMA per wave) a K-step earlier.
// Shapes: M % 256 == 0, N % BN == 0, K % 64 == 0, K >= 128 (gemm_nt.hip falls back to
// gemm_nt_kernel).
#pragma once

// MSU_EXP: ablation bits for timing experiments only (tools/build_exp.sh); 0 in every real build
#ifndef MSU_EXP
#define MSU_EXP 0
#endif

namespace pp {

constexpr int BM = 256;

// chunk c of row r of a [rows][32] k-slice image sits at chunk c ^ qsw(r): with 64-B rows four
// rows share a 256-B bank row, and the 16 lanes of each ds_read_b128 lane group ({0-3, 12-15,
// 20-27}, ...) then hit 16 distinct 16-B slots (g = {0, 2, 3, 1} by (r >> 2) & 3, checked for
// the four lane groups of a 16-row fragment)
MSU_DEV int qsw(int r) { return (0x78 >> (2 * ((r >> 2) & 3))) & 3; }

template <int OFF>
MSU_DEV bf16x8 ds_b128_untracked(uint32_t addr) {
  bf16x8 v;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v) : "v"(addr), "i"(OFF));
  return v;
}
template <int OFF>
MSU_DEV f32x4 ds_f4_untracked(uint32_t addr) {
  f32x4 v;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v) : "v"(addr), "i"(OFF));
  return v;
}

// vmcnt(A + (f1 ? B : 0) + (f2 ? C : 0)) with compile-time counts
template <int A, int B, int C>
MSU_DEV void wait3(bool f1, bool f2) {
  if (f1) {
    if (f2) wait_vmcnt<A + B + C>();
    else wait_vmcnt<A + B>();
  } else {
    if (f2) wait_vmcnt<A + C>();
    else wait_vmcnt<A>();
  }
}

// vmcnt(base + S * n) for base in 6..9 (a wave's DMA shares, +1 for a bias DMA) and n in 0..2
// (put slots in flight, S stores each), compile-time immediates
template <int S, int B = 6>
MSU_DEV void wait_plus(int base, int n) {
  if constexpr (B <= 9) {
    if (base == B) {
      if (n == 0) wait_vmcnt<B>();
      else if (n == 1) wait_vmcnt<B + S>();
      else wait_vmcnt<B + 2 * S>();
      return;
    }
    wait_plus<S, B + 1>(base, n);
  }
}

template <typename F, int... Is>
MSU_DEV void for_ic(F&& f, std::integer_sequence<int, Is...>) {
  (f(std::integral_constant<int, Is>{}), ...);
}

template <typename T, int EPI, int BN>
__global__ void __launch_bounds__(512) gemm_pp_kernel(NtArgs a) {
  static_assert(EPI != EPI_GELU_GRAD, "GELU' stays on gemm_nt_kernel");
  constexpr int NT = BN / 32;  // 16-column tiles of a wave (its group owns BN / 2 columns)
  constexpr int MT = 4;        // 16-row token tiles of a wave
  constexpr int HB = BN / 2;
  constexpr int QA = BM * 32, QW = BN * 32;  // elements of an A / W k-slice image
  constexpr int HALF = QA + QW;              // one k-slice half of a K-step (a ring slot)
  constexpr int IW = BN / 16;                // wave instructions of a W k-slice image
  static_assert(NT % 2 == 0, "column tiles in permlane16 pairs");
  // four ring slots, then one 1-KB bias image per wave
  __shared__ __attribute__((aligned(16))) bf16_t lds[4 * HALF + 8 * 512];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int grp = wave >> 2, wq = wave & 3;
  // this wave issues 2 DMA instructions per A k-slice and 2 (or, at BN = 192, waves 4-7: 1) per W
  const bool w2 = IW % 8 == 0 || wave < IW % 8;
  const int G = gridDim.x;
  const int L = xcd_remap(blockIdx.x, G);
  const int ntiles = a.tiles_m * a.tiles_n;
  const int nk = a.K / 64;
  const int mine = L < ntiles ? (ntiles - 1 - L) / G + 1 : 0;
  const int nsteps = mine * nk;
  if (nsteps == 0) return;

  // per-lane DMA element offsets (row r = 16 i + lane / 4 of instruction i = wave + 8 j, its
  // chunk swizzled): A with row stride K1 (and K - K1 for the concatenation's second input), W
  const int ldA = a.K1, ldA2 = a.K - a.K1;
  int offA[2], offA2[2], offW[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int r = 16 * (wave + 8 * j) + (lane >> 2);
    const int c = 8 * ((lane & 3) ^ qsw(r));
    offA[j] = r * ldA + c;
    offA2[j] = r * ldA2 + c;
    offW[j] = r * a.K + c;
  }
  // operand bases of the tile being loaded (scalar; refreshed once per tile)
  const bf16_t *pa = nullptr, *pa2 = nullptr, *pw = nullptr;
  auto set_bases = [&](int m0, int n0) __attribute__((always_inline)) {
    pa = a.A + (size_t)m0 * ldA;
    pa2 = a.A2 + (size_t)m0 * ldA2 - a.K1;  // (only dereferenced when A2 is given)
    pw = a.W + (size_t)n0 * a.K;
  };
  // half h (k-slice) of the K-step at column kcol of the tile being loaded, into ring slot j
  auto issue = [&](int h, int j4, int kcol) __attribute__((always_inline)) {
    if constexpr (MSU_EXP & 1) return;  // ablation: no DMA (results wrong)
    bf16_t* ia = lds + j4 * HALF;
    bf16_t* iw = ia + QA;
    const int kc = kcol + 32 * h;
    if (kc < a.K1) {  // K1 == K without a concatenation
#pragma unroll
      for (int j = 0; j < 2; ++j) glds16(pa + kc + offA[j], ia + 512 * (wave + 8 * j));
    } else {
#pragma unroll
      for (int j = 0; j < 2; ++j) glds16(pa2 + kc + offA2[j], ia + 512 * (wave + 8 * j));
    }
    glds16(pw + kc + offW[0], iw + 512 * wave);
    if (w2) glds16(pw + kc + offW[1], iw + 512 * (wave + 8));
  };
  // the tile's bias columns [n0, n0 + BN) into this wave's bias image (lanes past BN re-read the
  // last 16 B; a null bias reads zeros)
  bf16_t* bias_img = lds + 4 * HALF + 512 * wave;
  auto issue_bias = [&](int n0) __attribute__((always_inline)) {
    const int c = 4 * min(lane, BN / 4 - 1);
    glds16(a.bias ? (const void*)(a.bias + n0 + c) : zero_src(lane), bias_img);
  };

  // the step being multiplied (c), the step whose halves are being issued (d), the tile whose
  // epilogue is pending (e)
  int c_kk = 0, c_t = L;
  int c_n0 = (c_t % a.tiles_n) * BN;
  int d_kk = 0, d_t = L;
  int d_m0 = (d_t / a.tiles_n) * BM, d_n0 = (d_t % a.tiles_n) * BN;
  int e_m0 = d_m0, e_n0 = d_n0;
  set_bases(d_m0, d_n0);
  auto advance_d = [&]() __attribute__((always_inline)) {
    if (++d_kk == nk) {
      d_kk = 0;
      d_t += G;
      d_m0 = (d_t / a.tiles_n) * BM;
      d_n0 = (d_t % a.tiles_n) * BN;
      set_bases(d_m0, d_n0);
    }
  };

  // fragment lane offset (bytes) in a k-slice image: row l & 15 of a 16-row fragment, chunk l >> 4
  const uint32_t loff = 2u * ((lane & 15) * 32 + 8 * ((lane >> 4) ^ qsw(lane & 15)));
  const uint32_t lds0 = lds_u32(lds);
  const uint32_t w_row = 2u * QA + (uint32_t)(grp * HB) * 64u + loff;  // this group's first W row
  const uint32_t x_row = (uint32_t)(64 * wq) * 64u + loff;            // this wave's first token row
  const int g4 = lane >> 4, l15 = lane & 15;
  const int cofs = 16 * (g4 & 1) + 8 * (g4 >> 1);  // first of the lane's 8 columns after the swap
  const uint32_t bias_lds = lds_u32(bias_img) + 4u * (grp * HB + cofs);

  f32x4 acc[NT][MT];
#pragma unroll
  for (int n = 0; n < NT; ++n)
#pragma unroll
    for (int m = 0; m < MT; ++m) acc[n][m] = f32x4{0.f, 0.f, 0.f, 0.f};

  // Epilogue, in two parts so the output writes overlap the next tile's MFMAs instead of every
  // CU writing its tile at once (the whole chip's HBM write burst stalled every MFMA pipe: the
  // kernel ran 1.8x faster with the stores removed, r05e ablation):
  //   pack: at the next tile's first load slot, permlane-swap + bias + round the accumulators
  //         into 16-bit words (48 registers), freeing them for the next tile;
  //   put(m): the stores of token tile m, one m per load slot of the next tile's first two
  //         K-steps (GELU of the rounded values computed there for the dual epilogue).
  u32x4 outp[MT][NT / 2];
  int o_m0 = 0, o_n0 = 0;  // the tile outp holds
  auto pack = [&]() __attribute__((always_inline)) {
    f32x4 bq[NT / 2][2];
    for_ic([&](auto QI) {
      constexpr int q = decltype(QI)::value;
      bq[q][0] = ds_f4_untracked<128 * q>(bias_lds);
      bq[q][1] = ds_f4_untracked<128 * q + 16>(bias_lds);
    }, std::make_integer_sequence<int, NT / 2>{});
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int q = 0; q < NT / 2; ++q) {
      vreg_pin(bq[q][0]);
      vreg_pin(bq[q][1]);
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int q = 0; q < NT / 2; ++q) {
        float v[8];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(acc[2 * q][m][i]),
                                                          __float_as_uint(acc[2 * q + 1][m][i]), false, false);
          v[i] = __uint_as_float(r[0]) + bq[q][0][i];
          v[4 + i] = __uint_as_float(r[1]) + bq[q][1][i];
        }
        outp[m][q] = u32x4{pack2<T>(v[0], v[1]), pack2<T>(v[2], v[3]), pack2<T>(v[4], v[5]), pack2<T>(v[6], v[7])};
      }
  };
  // store I of the tile in outp (token tile I / (NT/2), column group I % (NT/2)); D stores
  constexpr int NST = MT * (NT / 2);                 // puts per tile
  constexpr int D = EPI == EPI_GELU_DUAL ? 2 : 1;    // stores per put
  auto put = [&](auto II) __attribute__((always_inline)) {
    constexpr int m = decltype(II)::value / (NT / 2), q = decltype(II)::value % (NT / 2);
    // ablation: no output stores (results wrong; this also leaves the MFMAs dead code, so it
    // times neither stores nor MFMAs: r05g's "no-store" numbers are no-store-no-MFMA ones)
    if constexpr (MSU_EXP & 8) return;
    const size_t off = (size_t)(o_m0 + 64 * wq + 16 * m + l15) * a.N + o_n0 + grp * HB + 32 * q + cofs;
    *reinterpret_cast<u32x4*>(a.Y + off) = outp[m][q];
    if constexpr (EPI == EPI_GELU_DUAL) {
      // GELU of the rounded pre-activation, as the unfused GELU kernel would see it
      const u32x4 h = outp[m][q];
      u32x4 g;
#pragma unroll
      for (int i = 0; i < 4; ++i) g[i] = pack2<T>(gelu_fast(Fmt16<T>::lo(h[i])), gelu_fast(Fmt16<T>::hi(h[i])));
      *reinterpret_cast<u32x4*>(a.Y2 + off) = g;
    }
  };
  // the puts of slot j of a tile (the previous tile's output): token tile j (NT / 2 puts) in
  // each of the first MT slots (nk >= 3 keeps the tile's last two slots free of puts).  One put
  // per slot over all slots of the tile was slower (r05g: 62.0 vs 55.3 us at 32768 x 1152 x 384).
  constexpr int sps = NT / 2, nsl = MT;
  auto put_m = [&](auto MI) __attribute__((always_inline)) {
    for_ic([&](auto QI) __attribute__((always_inline)) {
      put(std::integral_constant<int, sps * decltype(MI)::value + decltype(QI)::value>{});
    }, std::make_integer_sequence<int, sps>{});
  };
  static_assert(nsl == 4, "puts_at");
  auto puts_at = [&](int j) __attribute__((always_inline)) {
    if (j == 0) put_m(std::integral_constant<int, 0>{});
    else if (j == 1) put_m(std::integral_constant<int, 1>{});
    else if (j == 2) put_m(std::integral_constant<int, 2>{});
    else put_m(std::integral_constant<int, 3>{});
  };

  // prologue: the first tile's bias, h_0, h_1 (step 0) and h_2 (step 1, half 0); wait for the
  // bias and h_0 (younger: h_1, h_2), then group 1 falls one barrier behind
  const int nhalf = 2 * nsteps;
  issue_bias(d_n0);
  issue(0, 0, 0);
  issue(1, 1, 0);
  advance_d();
  if (nhalf > 2) issue(0, 2, 64 * d_kk);
  if (nhalf > 2) {
    if (w2) wait_vmcnt<8>();
    else wait_vmcnt<6>();
  } else {
    wait_vmcnt<0>();
  }
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  if (grp == 1) __builtin_amdgcn_s_barrier();

  for (int s = 0; s < nsteps; ++s) {
    const bool epi = c_kk == 0 && s > 0;
    const bool last = c_kk == nk - 1;
    bf16x8 wf[NT], xf[MT];
    for_ic([&](auto PI) __attribute__((always_inline)) {
      constexpr int p = decltype(PI)::value;
      const int k = 2 * s + p;
      // ---------------- load slot k
      if constexpr (p == 1) {
        // every step re-stages its tile's bias (the previous tile's epilogue read the image at
        // phase 0 of this step, lgkmcnt(0) before its barrier): one DMA per step
        issue_bias(c_n0);
      }
      const bool tail = k + 3 >= nhalf;
      if (!tail) {
        // h_{k+3}: half 1 of step s + 1 (p = 0) or half 0 of step s + 2 (p = 1), ring slot (k+3) % 4
        issue(p ^ 1, (k + 3) & 3, 64 * d_kk);
        if constexpr (p == 0) advance_d();
      }
      // this wave's share of h_{k+1} landed (read in the next load slot).  Younger than h_{k+1}
      // (issued in slot k - 2 before its wait): the output stores of slots k - 2 and k - 1, the
      // bias DMA of whichever of slots k - 1, k has p = 1, h_{k+2}, h_{k+3}.  Slot j = 2 c_kk + p
      // of a tile puts token tile j of the previous tile (j < 4): ns = puts among slots k-2, k-1.
      const int j = 2 * c_kk + p;
      // puts in flight from slots k - 2, k - 1 (sps each, D stores a put); slot i of the tile
      // puts when i < nsl and it is not the first tile (none in the last two slots of a tile)
      auto puts_in = [&](int jj) { return s >= nk && jj >= 0 && jj < nsl; };
      const int ns = sps * (puts_in(j - 1) + puts_in(j - 2));
      constexpr int Q2 = 8;  // 2 x the DMA share of a half of a w2 wave (2 + 2; others 2 + 1)
      if (tail) {
        wait_vmcnt<0>();
      } else if (p == 0 && epi) {
        // the previous slot's bias DMA too (pack reads it): younger are h_{k+2} and h_{k+3}
        if (w2) wait_vmcnt<Q2>();
        else wait_vmcnt<Q2 - 2>();
      } else {
        // the +1: the bias DMA of slot k - 1 (p = 0) or k (p = 1); none before slot 0
        const int base = (w2 ? Q2 : Q2 - 2) + (k > 0);
        wait_plus<D * sps>(base, ns / sps);
      }
      if constexpr (p == 0) {
        if (epi) {
          pack();
          o_m0 = e_m0;
          o_n0 = e_n0;
#pragma unroll
          for (int n = 0; n < NT; ++n)
#pragma unroll
            for (int m = 0; m < MT; ++m) acc[n][m] = f32x4{0.f, 0.f, 0.f, 0.f};
        }
      }
      if (s >= nk && j < nsl) puts_at(j);
      const uint32_t img = lds0 + (uint32_t)((k & 3) * HALF * 2);
      if constexpr (!(MSU_EXP & 2)) {  // ablation: no fragment reads (results wrong)
        for_ic([&](auto NI) { wf[decltype(NI)::value] = ds_b128_untracked<1024 * decltype(NI)::value>(img + w_row); },
               std::make_integer_sequence<int, NT>{});
        for_ic([&](auto MI) { xf[decltype(MI)::value] = ds_b128_untracked<1024 * decltype(MI)::value>(img + x_row); },
               std::make_integer_sequence<int, MT>{});
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
      for (int n = 0; n < NT; ++n) vreg_pin(wf[n]);
#pragma unroll
      for (int m = 0; m < MT; ++m) vreg_pin(xf[m]);
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      // ---------------- MFMA slot k
      __builtin_amdgcn_s_setprio(1);
      if constexpr (!(MSU_EXP & 4)) {  // ablation: no MFMAs (results wrong)
#pragma unroll
        for (int n = 0; n < NT; ++n)
#pragma unroll
          for (int m = 0; m < MT; ++m) acc[n][m] = Fmt16<T>::mma16(wf[n], xf[m], acc[n][m]);
      }
      __builtin_amdgcn_s_setprio(0);
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
    }, std::make_integer_sequence<int, 2>{});
    // advance the step state
    if (last) {
      e_m0 = (c_t / a.tiles_n) * BM;
      e_n0 = c_n0;
    }
    if (++c_kk == nk) {
      c_kk = 0;
      c_t += G;
      c_n0 = (c_t % a.tiles_n) * BN;
    }
  }
  if (grp == 0) __builtin_amdgcn_s_barrier();  // group 1's extra barrier at the start
  // the last tile (its bias DMA'd in its last step, retired by the tail's vmcnt(0))
  pack();
  o_m0 = e_m0;
  o_n0 = e_n0;
  for_ic([&](auto II) { put(II); }, std::make_integer_sequence<int, NST>{});
}

}  // namespace pp
