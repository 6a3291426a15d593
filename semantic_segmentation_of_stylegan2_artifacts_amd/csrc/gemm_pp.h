// Ping-pong 16-bit NT GEMM for the stage 1-3 Linears (included by gemm_nt.hip; same NtArgs and
// epilogues as gemm_nt_kernel): Y[M][N] = epi(A[M][K] . W[N][K]^T + bias), f32 accumulation.
//
// Why another form: the persistent 2-barrier kernel (gemm_nt_kernel) runs its two waves per SIMD
// in lockstep -- both reach every barrier together, both read LDS together, both issue MFMAs
// together -- and keeps the MFMA pipe busy 25 % of the time (r04i counters at 32768 x 1152 x
// 384: 623 TF/s).  Here the 8 waves form two groups of four, one wave of each group per SIMD
// (waves w and w + 4 share a SIMD), and group 1 runs one barrier behind group 0: between any two
// barriers one group issues MFMAs while the other reads its next fragments from LDS and issues
// its share of the LDS-DMA prefetch, so each SIMD always has one wave feeding its matrix pipe
// (the 8-phase schedule of cdna_hip_programming.md section 5, "The 256^2 8-phase template").
//
// Tile BM x BN = 256 x 256 (N % 256 == 0) or 256 x 192; group g owns output columns
// [g BN/2, (g+1) BN/2), its wave q the rows [64 q, 64 q + 64): a 64 x BN/2 wave tile of 16x16x32
// MFMAs computed transposed (W rows on the accumulator rows, tokens on the lanes), so after a
// permlane16 swap each lane stores 8 consecutive columns of its token row (16-B stores).
// A K-step (64) is four phases (k-slice s = p / 2, token half h = p % 2): 2 x BN/32 MFMAs each.
// The LDS holds two K-steps, each as four "quarters" [A k0-31][W k0-31][A k32-63][W k32-63]
// ([rows][32 k] images, 64-B rows, XOR-swizzled 16-B chunks, filled by global_load_lds_dwordx4):
// the load slot of phase p of step s issues quarter p of step s + 1, so every quarter has a whole
// K-step (eight slots) to land; the waits are counted (vmcnt) at phases 1 and 3, never 0.
// The workgroup is persistent over its tiles (XCD-contiguous tile ranges; the DMA stream runs
// across tile boundaries); a tile's epilogue runs in the load slot of the next tile's first
// phase, its operands (bias / GELU' pre-activations) loaded a K-step earlier.
// Shapes: M % 256 == 0, N % BN == 0, K % 64 == 0 (gemm_nt.hip falls back to gemm_nt_kernel).
#pragma once

namespace pp {

constexpr int BM = 256;

// chunk c of row r of a [rows][32] quarter image sits at chunk c ^ qsw(r): with 64-B rows four
// rows share a 256-B bank row, and the 16 lanes of each ds_read_b128 lane group ({0-3, 12-15,
// 20-27}, ...) then hit 16 distinct 16-B slots (g = {0, 2, 3, 1} by (r >> 2) & 3, checked for
// the four lane groups of a 16-row fragment)
MSU_DEV int qsw(int r) { return (0x78 >> (2 * ((r >> 2) & 3))) & 3; }

// one quarter (32 k columns from kcol) of a ROWS-row operand into its image: wave instruction i
// (16 rows x 4 chunks, 1 KB) is issued by wave i % 8; rows past `rows` never occur (M, N tiled)
template <int ROWS>
MSU_DEV void stage_q(const bf16_t* __restrict__ src, long ld, long row0, int kcol, bf16_t* img, int wave,
                     int lane) {
  constexpr int NI = ROWS / 16;
#pragma unroll
  for (int j = 0; j < (NI + 7) / 8; ++j) {
    const int i = wave + 8 * j;
    if (NI % 8 == 0 || i < NI) {
      const int r = 16 * i + (lane >> 2);
      const int c = (lane & 3) ^ qsw(r);
      glds16(src + (row0 + r) * ld + kcol + 8 * c, img + 512 * i);
    }
  }
}

template <int OFF>
MSU_DEV bf16x8 ds_b128_untracked(uint32_t addr) {
  bf16x8 v;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v) : "v"(addr), "i"(OFF));
  return v;
}

// s_waitcnt vmcnt(n) for a wave-uniform n (the counts depend on the wave's DMA share and on
// which slot the epilogue / its operand loads fell into); larger n than any real count = 0
MSU_DEV void wait_vm(int n) {
  switch (n) {
#define MSU_PP_W(N) \
  case N: wait_vmcnt<N>(); break;
    MSU_PP_W(0) MSU_PP_W(1) MSU_PP_W(2) MSU_PP_W(3) MSU_PP_W(4) MSU_PP_W(5) MSU_PP_W(6) MSU_PP_W(7)
    MSU_PP_W(8) MSU_PP_W(9) MSU_PP_W(10) MSU_PP_W(11) MSU_PP_W(12) MSU_PP_W(13) MSU_PP_W(14) MSU_PP_W(15)
    MSU_PP_W(16) MSU_PP_W(17) MSU_PP_W(18) MSU_PP_W(19) MSU_PP_W(20) MSU_PP_W(21) MSU_PP_W(22) MSU_PP_W(23)
    MSU_PP_W(24) MSU_PP_W(25) MSU_PP_W(26) MSU_PP_W(27) MSU_PP_W(28) MSU_PP_W(29) MSU_PP_W(30) MSU_PP_W(31)
    MSU_PP_W(32) MSU_PP_W(33) MSU_PP_W(34) MSU_PP_W(35) MSU_PP_W(36) MSU_PP_W(37) MSU_PP_W(38) MSU_PP_W(39)
    MSU_PP_W(40) MSU_PP_W(41) MSU_PP_W(42) MSU_PP_W(43) MSU_PP_W(44) MSU_PP_W(45) MSU_PP_W(46) MSU_PP_W(47)
    MSU_PP_W(48) MSU_PP_W(49) MSU_PP_W(50) MSU_PP_W(51) MSU_PP_W(52) MSU_PP_W(53) MSU_PP_W(54) MSU_PP_W(55)
#undef MSU_PP_W
    default: wait_vmcnt<0>(); break;
  }
}

template <int I> using ic = std::integral_constant<int, I>;
template <typename F, int... Is>
MSU_DEV void for_ic(F&& f, std::integer_sequence<int, Is...>) {
  (f(ic<Is>{}), ...);
}

template <typename T, int EPI, int BN>
__global__ void __launch_bounds__(512) gemm_pp_kernel(NtArgs a) {
  constexpr int NT = BN / 32;  // 16-column tiles of a wave (its group owns BN / 2 columns)
  constexpr int MT = 4;        // 16-row token tiles of a wave
  constexpr int HB = BN / 2;
  constexpr int QA = BM * 32, QW = BN * 32;  // elements of an A / W quarter image
  constexpr int STG = 2 * (QA + QW);         // one K-step
  constexpr int IW = BN / 16;                // wave instructions of a W quarter
  constexpr int E = MT * (NT / 2) * (EPI == EPI_GELU_DUAL ? 2 : 1);  // epilogue stores per wave
  constexpr int EOP = EPI == EPI_GELU_GRAD ? MT * (NT / 2) : NT;     // epilogue operand loads per wave
  static_assert(NT % 2 == 0, "column tiles in permlane16 pairs");
  __shared__ __attribute__((aligned(16))) bf16_t lds[2 * STG];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int grp = wave >> 2, wq = wave & 3;
  // this wave's DMA instructions per A + W quarter pair (A: 2; W: IW / 8, rounded by wave)
  const int qcnt = 2 + (IW - wave + 7) / 8;
  const int G = gridDim.x;
  const int L = xcd_remap(blockIdx.x, G);
  const int ntiles = a.tiles_m * a.tiles_n;
  const int nk = a.K / 64;
  const int mine = L < ntiles ? (ntiles - 1 - L) / G + 1 : 0;
  const int nsteps = mine * nk;
  if (nsteps == 0) return;

  // tile / K-step state: c = the step being multiplied, l = the step being loaded (c + 1),
  // e = the tile whose epilogue is pending
  int c_t = L, c_kk = 0;
  int c_m0 = (c_t / a.tiles_n) * BM, c_n0 = (c_t % a.tiles_n) * BN;
  int l_t = c_t, l_kk = 1, l_m0 = c_m0, l_n0 = c_n0;
  if (l_kk == nk) {
    l_kk = 0;
    l_t += G;
    l_m0 = (l_t / a.tiles_n) * BM;
    l_n0 = (l_t % a.tiles_n) * BN;
  }
  int e_m0 = c_m0, e_n0 = c_n0;

  auto issue = [&](auto QI, bf16_t* buf, int m0, int n0, int kk) __attribute__((always_inline)) {
    constexpr int qi = decltype(QI)::value;
    const int kcol = kk * 64 + 32 * (qi >> 1);
    bf16_t* img = buf + (qi >> 1) * (QA + QW) + (qi & 1) * QA;
    if constexpr ((qi & 1) == 0) {
      if (a.A2 == nullptr || kcol < a.K1) stage_q<BM>(a.A, a.K1, m0, kcol, img, wave, lane);
      else stage_q<BM>(a.A2, a.K - a.K1, m0, kcol - a.K1, img, wave, lane);
    } else {
      stage_q<BN>(a.W, a.K, n0, kcol, img, wave, lane);
    }
  };

  // fragment lane offset (bytes) in a quarter image: row l & 15 of a 16-row fragment, chunk l >> 4
  const uint32_t loff = 2u * ((lane & 15) * 32 + 8 * ((lane >> 4) ^ qsw(lane & 15)));
  const uint32_t lds0 = lds_u32(lds);
  const uint32_t w_row = (uint32_t)(grp * HB) * 64u + loff;  // this group's first W row
  const uint32_t x_row = (uint32_t)(64 * wq) * 64u + loff;   // this wave's first token row

  f32x4 acc[NT][MT];
#pragma unroll
  for (int n = 0; n < NT; ++n)
#pragma unroll
    for (int m = 0; m < MT; ++m) acc[n][m] = f32x4{0.f, 0.f, 0.f, 0.f};
  float4 bq[EPI == EPI_GELU_GRAD ? 1 : NT / 2][2];
  u32x4 hq[EPI == EPI_GELU_GRAD ? MT : 1][EPI == EPI_GELU_GRAD ? NT / 2 : 1];
  const int g4 = lane >> 4, l15 = lane & 15;
  const int cofs = 16 * (g4 & 1) + 8 * (g4 >> 1);  // first of the lane's 8 columns after the swap

  // epilogue operands of the tile at (m0, n0): bias columns / GELU' pre-activations
  auto load_eop = [&](int m0, int n0) __attribute__((always_inline)) {
    if constexpr (EPI == EPI_GELU_GRAD) {
#pragma unroll
      for (int m = 0; m < MT; ++m)
#pragma unroll
        for (int q = 0; q < NT / 2; ++q)
          hq[m][q] = *reinterpret_cast<const u32x4*>(a.H + (size_t)(m0 + 64 * wq + 16 * m + l15) * a.N + n0 +
                                                     grp * HB + 32 * q + cofs);
    } else {
#pragma unroll
      for (int q = 0; q < NT / 2; ++q) {
        const float* bp = a.bias ? a.bias + n0 + grp * HB + 32 * q + cofs
                                 : reinterpret_cast<const float*>(zero_src(2 * q));
        bq[q][0] = *reinterpret_cast<const float4*>(bp);
        bq[q][1] = *reinterpret_cast<const float4*>(a.bias ? bp + 4 : bp);
      }
    }
  };
  auto epilogue = [&](int m0, int n0) __attribute__((always_inline)) {
#pragma unroll
    for (int m = 0; m < MT; ++m) {
      const size_t row = (size_t)(m0 + 64 * wq + 16 * m + l15) * a.N;
#pragma unroll
      for (int q = 0; q < NT / 2; ++q) {
        float v[8];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(acc[2 * q][m][i]),
                                                          __float_as_uint(acc[2 * q + 1][m][i]), false, false);
          v[i] = __uint_as_float(r[0]);
          v[4 + i] = __uint_as_float(r[1]);
        }
        if constexpr (EPI == EPI_GELU_GRAD) {
          const u32x4 h = hq[m][q];
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            v[2 * i] *= gelu_grad_fast(Fmt16<T>::lo(h[i]));
            v[2 * i + 1] *= gelu_grad_fast(Fmt16<T>::hi(h[i]));
          }
        } else {
          const float4 b0 = bq[q][0], b1 = bq[q][1];
          v[0] += b0.x; v[1] += b0.y; v[2] += b0.z; v[3] += b0.w;
          v[4] += b1.x; v[5] += b1.y; v[6] += b1.z; v[7] += b1.w;
        }
        const size_t off = row + n0 + grp * HB + 32 * q + cofs;
        const u32x4 pk = {pack2<T>(v[0], v[1]), pack2<T>(v[2], v[3]), pack2<T>(v[4], v[5]), pack2<T>(v[6], v[7])};
        *reinterpret_cast<u32x4*>(a.Y + off) = pk;
        if constexpr (EPI == EPI_GELU_DUAL) {
          float gv[8];
#pragma unroll
          for (int i = 0; i < 8; ++i) gv[i] = gelu_fast(round16<T>(v[i]));
          const u32x4 pg = {pack2<T>(gv[0], gv[1]), pack2<T>(gv[2], gv[3]), pack2<T>(gv[4], gv[5]),
                            pack2<T>(gv[6], gv[7])};
          *reinterpret_cast<u32x4*>(a.Y2 + off) = pg;
        }
      }
    }
  };

  // prologue: all of step 0, wait for its first half (quarters 0, 1), then group 1 falls one
  // barrier behind
  for_ic([&](auto QI) { issue(QI, lds, c_m0, c_n0, 0); }, std::make_integer_sequence<int, 4>{});
  wait_vm(qcnt);
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  if (grp == 1) __builtin_amdgcn_s_barrier();

  for (int s = 0; s < nsteps; ++s) {
    const bool has_next = s + 1 < nsteps;
    const bool first = c_kk == 0, last = c_kk == nk - 1;
    const uint32_t cur = lds0 + (uint32_t)((s & 1) * STG * 2);
    bf16_t* nbuf = lds + ((s + 1) & 1) * STG;
    bf16x8 wf[NT], xf[2];
    for_ic([&](auto PI) __attribute__((always_inline)) {
      constexpr int p = decltype(PI)::value, ks = p >> 1, h = p & 1;
      // ---------------- load slot
      if constexpr (p == 0) {
        if (first && s > 0) {
          epilogue(e_m0, e_n0);
#pragma unroll
          for (int n = 0; n < NT; ++n)
#pragma unroll
            for (int m = 0; m < MT; ++m) acc[n][m] = f32x4{0.f, 0.f, 0.f, 0.f};
        }
        if (last) load_eop(c_m0, c_n0);
      }
      if (has_next) issue(PI, nbuf, l_m0, l_n0, l_kk);
      if constexpr (p == 1) {
        // quarters 2, 3 of this step (issued a step ago) landed; younger: the epilogue stores,
        // its operand loads and quarters 0, 1 of the next step
        wait_vm((first && s > 0 ? E : 0) + (last ? EOP : 0) + (has_next ? qcnt : 0));
      } else if constexpr (p == 3) {
        // quarters 0, 1 of the next step landed; younger: its quarters 2, 3
        wait_vm(has_next ? qcnt : 0);
      }
      const uint32_t wimg = cur + (uint32_t)(ks * (QA + QW) * 2 + QA * 2) + w_row;
      const uint32_t ximg = cur + (uint32_t)(ks * (QA + QW) * 2) + x_row;
      if constexpr (h == 0) {
        for_ic([&](auto NI) { wf[decltype(NI)::value] = ds_b128_untracked<1024 * decltype(NI)::value>(wimg); },
               std::make_integer_sequence<int, NT>{});
      }
      xf[0] = ds_b128_untracked<1024 * (2 * h)>(ximg);
      xf[1] = ds_b128_untracked<1024 * (2 * h + 1)>(ximg);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
      for (int n = 0; n < NT; ++n) vreg_pin(wf[n]);
      vreg_pin(xf[0]);
      vreg_pin(xf[1]);
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      // ---------------- MFMA slot
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int n = 0; n < NT; ++n)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[n][2 * h + j] = Fmt16<T>::mma16(wf[n], xf[j], acc[n][2 * h + j]);
      __builtin_amdgcn_s_setprio(0);
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
    }, std::make_integer_sequence<int, 4>{});
    // advance the step state
    if (last) {
      e_m0 = c_m0;
      e_n0 = c_n0;
    }
    c_t = l_t;
    c_kk = l_kk;
    c_m0 = l_m0;
    c_n0 = l_n0;
    if (++l_kk == nk) {
      l_kk = 0;
      l_t += G;
      l_m0 = (l_t / a.tiles_n) * BM;
      l_n0 = (l_t % a.tiles_n) * BN;
    }
  }
  if (grp == 0) __builtin_amdgcn_s_barrier();  // group 1's extra barrier at the start
  epilogue(e_m0, e_n0);
  (void)c_t;
}

}  // namespace pp
