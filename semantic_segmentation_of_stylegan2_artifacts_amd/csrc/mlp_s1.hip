// Stage-1 Swin MLP forward in ONE kernel (torchvision MLP, model_parts.py:538, via the stage-1
// BasicLayer / BasicLayer_up blocks at dim 192):
//
//   y = mlp.3(GELU(mlp.0(x)))      x, y: [M][192], hidden 768
//
// The GEMM pair this replaces wrote H and GELU(H) (2 x 201 MB at 8 x 128^2 tokens) and read
// GELU(H) back; here the training form writes H only (the backward's GELU' operand) and GELU(H)
// never leaves the chip.  Unlike the stage-0 kernel (mlp_fused.hip) the weights (2 x 295 KB) do
// not fit one CU's LDS, so they are STREAMED: the hidden dimension is cut into 24 chunks of 32
// units, each chunk's W1 rows [32][192] and W2 columns [192][32] (24 KB) go global -> LDS by
// LDS-DMA into a ring of NS slots, and the workgroup's waves walk the chunks in step with one
// barrier per chunk (the slot of chunk j - 1 is refilled with chunk j + NS - 1 as chunk j starts).
// The ring runs across the workgroup's token tiles as one flat chunk sequence.
//
// Per wave: a 32-token tile (workgroup: 8 waves, 256 tokens).  The tile's x rows stay in registers
// as fc1's B operand (12 k steps); per chunk
//   * fc1 on MFMA (W1 rows as A, tokens on the accumulator columns), + b1, rounded to 16 bits
//     (stored as H), GELU, rounded again: the unfused epilogues' arithmetic;
//   * the packed GELU(H) registers are directly fc2's B operand: the chunk's W1 rows sit in the
//     slot PERMUTED (slot row rho holds hidden unit pi(rho), pi swapping bits 2 and 3), so that
//     accumulator registers 8s .. 8s + 7 of lane half hh hold hidden units 16s + 8hh .. + 7 --
//     consecutive, i.e. ONE 16-B W2 fragment read per fc2 MFMA and one 16-B H store per 8 units;
//   * fc2 accumulates y^T (six 32-channel tiles, 96 registers) over the 24 chunks.
// Slot images: W1 rows 384 B with 16-B chunk c at c ^ ((rho >> 1) & 7), W2 rows 64 B with chunk c at
// c ^ ((row >> 2) & 3): the 16-lane groups of the ds_read_b128 fragment reads cover the 64 banks
// once.  LDS reads of the ring are untracked inline asm (a compiler-visible ds_read behind a
// pending LDS-DMA gets a vmcnt(0) that drains the ring); the DMA waits are counted per wave.
#include "common.h"
#include "mfma_frag.h"

namespace {

// MSU_EXP: ablation / variant bits for timing experiments only (tools/build_exp.sh); 0 in every
// real build.  2: fragment reads one MFMA ahead instead of three; 4: waves 4-7 staggered by half a
// chunk (measured slower: 169 vs 160 us, r06h); 8: no GELU (identity); 16: no H stores; 32: no fc2
// MFMAs; 64: no fc1 MFMAs (results wrong by design for 8 / 16 / 32 / 64)
#ifndef MSU_EXP
#define MSU_EXP 0
#endif

constexpr int SC = 192, SH = 768, SW = 8, STT = 32 * SW;
constexpr int UH = 32;                      // hidden units per chunk (one barrier per chunk)
constexpr int NU = SH / UH;                 // chunks per token tile (24)
constexpr int SNS = 6;                      // ring slots (147 KB)
constexpr int FD = (MSU_EXP & 2) ? 1 : 3;   // fragment reads in flight ahead of the MFMA using one
constexpr bool STAG = (MSU_EXP & 4) != 0;   // waves 4-7 run half a chunk behind waves 0-3
constexpr int W1S = UH * SC;                // elements of a slot's W1 image [32][192]
constexpr int W2S = SC * UH;                // elements of a slot's W2 image [192][32]
constexpr int SLOT = W1S + W2S;
constexpr int DMA_PER_UNIT = SLOT * 2 / 1024;  // 1-KB DMA instructions per chunk (24)
constexpr int DMA_PER_WAVE = DMA_PER_UNIT / SW;
static_assert(DMA_PER_WAVE * SW == DMA_PER_UNIT, "whole DMA instructions per wave");

struct S1Lds {
  bf16_t ring[SNS * SLOT];
  float b1[SH];
  float b2[SC];
};
static_assert(sizeof(S1Lds) <= 160 * 1024, "LDS");

struct S1Args {
  const bf16_t* x;
  const bf16_t* w1;  // [768][192]
  const float* b1;
  const bf16_t* w2;  // [192][768]
  const float* b2;
  bf16_t* y;
  bf16_t* hout;      // H_OUT: [M][768]
  long M;
};

// hidden unit (within a chunk) held by slot row rho: bits 2 and 3 swapped
MSU_DEV constexpr int s1_pi(int rho) { return (rho & ~12) | ((rho & 4) << 1) | ((rho & 8) >> 1); }
// 16-B chunk swizzle of a W2 slot row (4 chunks per row)
MSU_DEV constexpr int w2_swz(int row) { return (row >> 2) & 3; }

// s_waitcnt vmcnt(n) for a wave-uniform runtime n (capped: waiting for more is always safe)
MSU_DEV void wait_vmcnt_le(int n) {
  switch (n < 0 ? 0 : (n > 40 ? 40 : n)) {
#define MSU_W(k) case k: wait_vmcnt<k>(); break;
    MSU_W(0) MSU_W(1) MSU_W(2) MSU_W(3) MSU_W(4) MSU_W(5) MSU_W(6) MSU_W(7) MSU_W(8) MSU_W(9)
    MSU_W(10) MSU_W(11) MSU_W(12) MSU_W(13) MSU_W(14) MSU_W(15) MSU_W(16) MSU_W(17) MSU_W(18) MSU_W(19)
    MSU_W(20) MSU_W(21) MSU_W(22) MSU_W(23) MSU_W(24) MSU_W(25) MSU_W(26) MSU_W(27) MSU_W(28) MSU_W(29)
    MSU_W(30) MSU_W(31) MSU_W(32) MSU_W(33) MSU_W(34) MSU_W(35) MSU_W(36) MSU_W(37) MSU_W(38) MSU_W(39)
    MSU_W(40)
#undef MSU_W
    default: wait_vmcnt<0>();
  }
}

template <int OFF>
MSU_DEV bf16x8 ds_b128_untracked(uint32_t addr) {
  bf16x8 v;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v) : "v"(addr), "i"(OFF));
  return v;
}

// Per chunk a wave runs three phases: fc1 (12 MFMAs), the epilogue (b1, H, GELU: VALU), fc2 (12
// MFMAs).  With one barrier per chunk the two waves of a SIMD (w, w + 4) would run them in phase --
// both on MFMAs, then both on VALU.  So waves 4-7 are STAGGERED: in the interval after chunk j's
// barrier waves 0-3 run fc1(j), epi(j), fc2(j) while waves 4-7 run epi(j - 1), fc2(j - 1), fc1(j)
// (their fc1 accumulator crosses the barrier): each SIMD pairs one wave's MFMAs with the other's
// VALU.  Chunk j - 1's slot is then read up to the end of interval j, so the ring prefetches
// SNS - 2 chunks ahead and interval j refills chunk j - 2's slot; one extra interval at the end
// lets waves 4-7 finish the last chunk.
template <typename T, bool H_OUT>
__global__ void __launch_bounds__(64 * SW) mlp_s1_kernel(S1Args A) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  S1Lds& L = *reinterpret_cast<S1Lds*>(smem_raw);
  const int tid = threadIdx.x, lane = tid & 63, hh = lane >> 5, tl = lane & 31;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const bool late = STAG && wave >= 4;  // wave-uniform
  const long M = A.M;
  const long ntiles = (M + STT - 1) / STT;
  const int G = gridDim.x;
  const long first = blockIdx.x;
  if (first >= ntiles) return;
  const long mine = (ntiles - 1 - first) / G + 1;
  const long nunits = mine * NU;

  for (int s = tid; s < SH; s += 64 * SW) L.b1[s] = A.b1[s];
  for (int s = tid; s < SC; s += 64 * SW) L.b2[s] = A.b2[s];
  __syncthreads();  // before any LDS-DMA is in flight (this barrier drains nothing)

  // chunk q (0 .. 23) of the weights into ring slot `slot`: this wave's 3 of the chunk's 24 1-KB
  // DMA instructions (W1 rows permuted by pi and chunk-swizzled; W2 columns chunk-swizzled)
  auto dma_unit = [&](int q, int slot) __attribute__((always_inline)) {
    bf16_t* base = L.ring + slot * SLOT;
    const int ln = opaque(lane);
#pragma unroll
    for (int r = 0; r < DMA_PER_WAVE; ++r) {
      const int i = wave + SW * r;  // instruction (wave-uniform)
      if (i < 12) {
        const int p = 64 * i + ln, rho = p / 24, pos = p - (p / 24) * 24;
        const int gc = pos ^ ((rho >> 1) & 7);
        glds16(A.w1 + (long)(UH * q + s1_pi(rho)) * SC + 8 * gc, base + 512 * i);
      } else {
        const int i2 = i - 12;
        const int p = 64 * i2 + ln, row = p >> 2, pos = p & 3;
        const int gc = pos ^ w2_swz(row);
        glds16(A.w2 + (long)row * SH + UH * q + 8 * gc, base + W1S + 512 * i2);
      }
    }
  };
  // the tile's token rows as fc1's B operand: lane (token tl, half hh) holds k = 16 ks + 8 hh .. + 7
  u32x4 xc[12];
  auto load_x = [&](long t) __attribute__((always_inline)) {
    const long row = t * STT + 32 * wave + tl;
    const bool ok = row < M;
    const bf16_t* p = A.x + (ok ? row : 0) * SC + 8 * hh;
#pragma unroll
    for (int ks = 0; ks < 12; ++ks) {
      const u32x4 v = *reinterpret_cast<const u32x4*>(p + 16 * ks);
      xc[ks] = ok ? v : u32x4{0u, 0u, 0u, 0u};
    }
  };

  // vector-memory ops this wave issued (wave-uniform), and the count right after each pending
  // chunk's DMA (a queue of SNS - 2: the chunk waited for next first): the vmcnt waits let every
  // younger op stay in flight.  Stores are counted only when the whole wave issues them (full
  // tile rows): an uncounted op only makes a wait stricter.
  int issued = 0;
  int mark[SNS - 2];
  load_x(first);
  issued += 12;
  int mark_x = issued;
#pragma unroll
  for (int s = 0; s < SNS - 2; ++s) {
    if (s < nunits) {
      dma_unit(s % NU, s);
      issued += DMA_PER_WAVE;
    }
    mark[s] = issued;
  }

  f32x16 yacc[6];
#pragma unroll
  for (int ct = 0; ct < 6; ++ct) yacc[ct] = f32x16{0};
  f32x16 h = f32x16{0};  // fc1 accumulator (waves 4-7: carried to the next interval)
  // untracked-read lane addresses (bytes)
  const uint32_t ring0 = lds_u32(L.ring);
  const uint32_t a1_lane = (uint32_t)(tl * SC * 2);              // + slot, + 16 * pos(ks)
  const int w1sw = (tl >> 1) & 7;
  const uint32_t a2_lane = (uint32_t)(W1S * 2 + tl * UH * 2);    // + slot, + 2048 ct, + 16 * pos
  const int w2sw = w2_swz(tl);                                   // (32 ct + tl: same swizzle)
  const uint32_t b1_lane = lds_u32(L.b1) + 4u * (uint32_t)(8 * hh);
  const uint32_t b2_lane = lds_u32(L.b2) + 4u * (uint32_t)(4 * hh);

  // ---- the three phases of a chunk
  auto fc1 = [&](int slot) __attribute__((always_inline)) {
    const uint32_t a1 = ring0 + (uint32_t)(slot * SLOT * 2) + a1_lane;
    h = f32x16{0};
    bf16x8 wf[FD + 1];
    auto addr1 = [&](int ks) { return a1 + 16u * (uint32_t)((2 * ks + hh) ^ w1sw); };
    unroll_for<FD>([&](auto KS) { wf[decltype(KS)::value] = ds_b128_untracked<0>(addr1(decltype(KS)::value)); });
    unroll_for<12>([&](auto KS) {
      constexpr int ks = decltype(KS)::value;
      if constexpr (ks + FD < 12) wf[(ks + FD) % (FD + 1)] = ds_b128_untracked<0>(addr1(ks + FD));
      lds_wait_tie<(ks + FD < 12 ? FD : 11 - ks)>(wf[ks % (FD + 1)]);
      if constexpr (MSU_EXP & 64) {
        const bf16x8 wv = wf[ks % (FD + 1)];
        const u32x4 xv = xc[ks];
        asm volatile("" ::"v"(wv), "v"(xv));
      } else h = Fmt16<T>::mma32(wf[ks % (FD + 1)], __builtin_bit_cast(bf16x8, xc[ks]), h);
    });
  };
  // + b1, 16-bit H (stored), GELU, 16-bit GELU(H): registers 8s + e <-> hidden 32 q + 16 s + 8 hh + e
  auto epi = [&](int q, long t, u32x4 (&g)[2]) __attribute__((always_inline)) {
    u32x4 bq[4];
    unroll_for<4>([&](auto BI) {
      constexpr int bi = decltype(BI)::value;
      bq[bi] = __builtin_bit_cast(u32x4, ds_b128_untracked<(bi >> 1) * 64 + (bi & 1) * 16>(
                                             b1_lane + 4u * (uint32_t)(UH * q)));
    });
    lds_wait_tie<0>(bq[0], bq[1], bq[2], bq[3]);
    const long hrow = t * STT + 32 * wave + tl;
    const bool hok = hrow < M;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      float uu[8];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        uu[e] = round16<T>(h[8 * s + e] + __uint_as_float(bq[2 * s][e]));
        uu[4 + e] = round16<T>(h[8 * s + 4 + e] + __uint_as_float(bq[2 * s + 1][e]));
      }
      if constexpr (H_OUT) {
        const u32x4 hv = {pack2<T>(uu[0], uu[1]), pack2<T>(uu[2], uu[3]), pack2<T>(uu[4], uu[5]),
                          pack2<T>(uu[6], uu[7])};
        if constexpr (MSU_EXP & 16) {
          const u32x4 hv2 = hv;
          asm volatile("" ::"v"(hv2));
        }
        else if (hok) *reinterpret_cast<u32x4*>(A.hout + hrow * SH + UH * q + 16 * s + 8 * hh) = hv;
      }
      uint32_t gp[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const f32x2 gv = (MSU_EXP & 8) ? f32x2{uu[2 * e], uu[2 * e + 1]}
                                       : gelu_fast2(f32x2{uu[2 * e], uu[2 * e + 1]});  // bitwise two gelu_fast
        gp[e] = pack2<T>(gv.x, gv.y);
      }
      g[s] = u32x4{gp[0], gp[1], gp[2], gp[3]};
    }
    if (H_OUT && !(MSU_EXP & 16) && t * STT + 32 * wave + 32 <= M) issued += 2;
  };
  // y^T[c][t] += W2[c][chunk] . GELU(H)^T: six 32-channel tiles, two 16-deep k steps
  auto fc2 = [&](int slot, const u32x4 (&g)[2]) __attribute__((always_inline)) {
    const uint32_t a2 = ring0 + (uint32_t)(slot * SLOT * 2) + a2_lane;
    auto addr2 = [&](int ct, int s) { return a2 + (uint32_t)(ct * 32 * UH * 2) + 16u * (uint32_t)((2 * s + hh) ^ w2sw); };
    bf16x8 af[FD + 1];
    unroll_for<FD>([&](auto I) {
      constexpr int i = decltype(I)::value;
      af[i] = ds_b128_untracked<0>(addr2(i % 6, i / 6));
    });
    unroll_for<12>([&](auto I) {
      constexpr int i = decltype(I)::value, s = i / 6, ct = i % 6;
      if constexpr (i + FD < 12) af[(i + FD) % (FD + 1)] = ds_b128_untracked<0>(addr2((i + FD) % 6, (i + FD) / 6));
      lds_wait_tie<(i + FD < 12 ? FD : 11 - i)>(af[i % (FD + 1)]);
      if constexpr (MSU_EXP & 32) {
        const bf16x8 av = af[i % (FD + 1)];
        const u32x4 gv = g[s];
        asm volatile("" ::"v"(av), "v"(gv));
      } else yacc[ct] = Fmt16<T>::mma32(af[i % (FD + 1)], __builtin_bit_cast(bf16x8, g[s]), yacc[ct]);
    });
  };
  // tile epilogue: y = y^T + b2; lane (token tl) holds channels 32 ct + 8 r4 + 4 hh + i in
  // register 4 r4 + i; a permlane32 swap pairs the halves into 8 consecutive channels per lane
  auto y_out = [&](long t) __attribute__((always_inline)) {
    const long row = t * STT + 32 * wave + tl;
    const bool ok = row < M;
    bf16_t* yr = A.y + (ok ? row : 0) * SC;
#pragma unroll
    for (int ct = 0; ct < 6; ++ct) {
      uint32_t w[8];
#pragma unroll
      for (int r4 = 0; r4 < 4; ++r4) {
        u32x4 bq;
        asm volatile("ds_read_b128 %0, %1" : "=v"(bq) : "v"(b2_lane + 4u * (uint32_t)(ct * 32 + 8 * r4)));
        lds_wait_tie<0>(bq);
        w[2 * r4] = pack2<T>(yacc[ct][4 * r4] + __uint_as_float(bq[0]), yacc[ct][4 * r4 + 1] + __uint_as_float(bq[1]));
        w[2 * r4 + 1] = pack2<T>(yacc[ct][4 * r4 + 2] + __uint_as_float(bq[2]),
                                 yacc[ct][4 * r4 + 3] + __uint_as_float(bq[3]));
      }
#pragma unroll
      for (int p = 0; p < 2; ++p) {
        const auto s0 = __builtin_amdgcn_permlane32_swap(w[4 * p], w[4 * p + 2], false, false);
        const auto s1 = __builtin_amdgcn_permlane32_swap(w[4 * p + 1], w[4 * p + 3], false, false);
        const u32x4 v = {s0[0], s1[0], s0[1], s1[1]};
        if (ok) *reinterpret_cast<u32x4*>(yr + ct * 32 + 16 * p + 8 * hh) = v;
      }
      yacc[ct] = f32x16{0};
    }
    if (t * STT + 32 * wave + 32 <= M) issued += 12;
  };
  // fc1 of chunk (q, slot) of tile t, after which the last chunk of a tile loads the next tile's x
  auto fc1_step = [&](int q, int slot, long t) __attribute__((always_inline)) {
    if (q == 0) wait_vmcnt_le(issued - mark_x);  // the tile's x rows
    fc1(slot);
    if (q == NU - 1 && t + G < ntiles) {  // xc is free once the tile's last fc1 has issued
      load_x(t + G);
      issued += 12;
      mark_x = issued;
    }
  };

  // interval j (0 .. nunits): chunk j = weights chunk q in ring slot `slot` of tile `tile`;
  // (qp, slotp, tilep) the previous chunk; the DMA issued in interval j is chunk j + SNS - 2
  int q = 0, slot = 0, qn = (SNS - 2) % NU, sn = SNS - 2, qp = 0, slotp = 0;
  long tile = first, tilep = first;
  for (long j = 0; j <= nunits; ++j) {
    const bool cur = j < nunits;
    if (cur) {
      // steady state (full tiles, no tile boundary among the younger ops): a constant count
      constexpr int STEADY = (SNS - 3) * DMA_PER_WAVE + (H_OUT && !(MSU_EXP & 16) ? 2 * (SNS - 2) : 0);
      const int younger = issued - mark[0];
      if (younger >= STEADY) wait_vmcnt<STEADY>();
      else wait_vmcnt_le(younger);
    }
    // chunk j's DMA (every wave's share) has landed; every wave is done with chunk j - 2's slot
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
#pragma unroll
    for (int s = 0; s < SNS - 3; ++s) mark[s] = mark[s + 1];
    if (j + SNS - 2 < nunits) {
      dma_unit(qn, sn);
      issued += DMA_PER_WAVE;
    }
    mark[SNS - 3] = issued;
    qn = qn + 1 == NU ? 0 : qn + 1;
    sn = sn + 1 == SNS ? 0 : sn + 1;
    // one straight sequence for both wave groups (two branch-separated copies of the phases
    // made the register allocator keep both copies' operands: 300+ VGPRs of spills)
    const bool second = late ? j > 0 : cur;  // the epi + fc2 of this interval exists
    const int qe = late ? qp : q, se = late ? slotp : slot;
    const long te = late ? tilep : tile;
    if (late && second) {
      u32x4 g[2];
      epi(qe, te, g);
      fc2(se, g);
      if (qe == NU - 1) y_out(te);
    }
    if (cur) fc1_step(q, slot, tile);
    if (!late && second) {
      u32x4 g[2];
      epi(qe, te, g);
      fc2(se, g);
      if (qe == NU - 1) y_out(te);
    }
    qp = q;
    slotp = slot;
    tilep = tile;
    if (q == NU - 1) tile += G;
    q = q + 1 == NU ? 0 : q + 1;
    slot = slot + 1 == SNS ? 0 : slot + 1;
  }
  wait_vmcnt<0>();  // no LDS-DMA outstanding when the workgroup retires
}

int num_cus_s1() {
  static const int cus = [] {
    int n = 0, dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
    return n;
  }();
  return cus;
}

template <typename T, bool H_OUT>
int launch_s1(const S1Args& a, hipStream_t st) {
  auto kern = mlp_s1_kernel<T, H_OUT>;
  static bool attr_set = false;
  if (!attr_set) {
    if (hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)sizeof(S1Lds)) !=
        hipSuccess)
      return -4;
    attr_set = true;
  }
  const long ntiles = (a.M + STT - 1) / STT;
  long grid = num_cus_s1();
  if (grid > ntiles) grid = ntiles;
  hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(64 * SW), sizeof(S1Lds), st, a);
  return MSU_CHECK_LAUNCH();
}

}  // namespace

// the stage-1 form of msu_mlp_fused_fwd (mlp_fused.hip dispatches here for C = 192, Hd = 768)
int msu_mlp_s1_launch(int dtype, const void* x, const void* w1, const float* b1, const void* w2, const float* b2,
                      void* y, void* h, long M, void* stream) {
  S1Args a{};
  a.x = (const bf16_t*)x;
  a.w1 = (const bf16_t*)w1;
  a.b1 = b1;
  a.w2 = (const bf16_t*)w2;
  a.b2 = b2;
  a.y = (bf16_t*)y;
  a.hout = (bf16_t*)h;
  a.M = M;
  hipStream_t st = (hipStream_t)stream;
  if (h != nullptr) {
    MSU_DISPATCH16(dtype, T, return (launch_s1<T, true>(a, st)));
  } else {
    MSU_DISPATCH16(dtype, T, return (launch_s1<T, false>(a, st)));
  }
  return -3;
}
