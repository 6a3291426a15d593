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

constexpr int SC = 192, SH = 768, SCH = 32, NCH = SH / SCH, SW = 8, STT = 32 * SW, SNS = 6;
constexpr int W1S = SCH * SC;          // elements of a slot's W1 image
constexpr int W2S = SC * SCH;          // elements of a slot's W2 image
constexpr int SLOT = W1S + W2S;        // 24 KB
constexpr int DMA_PER_CHUNK = SLOT * 2 / 1024;  // 1-KB DMA instructions per chunk (24)
constexpr int DMA_PER_WAVE = DMA_PER_CHUNK / SW;         // 3
static_assert(DMA_PER_WAVE * SW == DMA_PER_CHUNK, "whole DMA instructions per wave");

struct S1Lds {
  bf16_t ring[SNS * SLOT];
  float b1[SH];
  float b2[SC];
};

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

// hidden unit (within the chunk) held by slot row rho: bits 2 and 3 swapped
MSU_DEV constexpr int s1_pi(int rho) { return (rho & ~12) | ((rho & 4) << 1) | ((rho & 8) >> 1); }

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
// 8 consecutive f32 (bias values) from LDS, untracked, after lgkmcnt(0)
MSU_DEV void ds_f32x8_untracked(uint32_t addr, float (&v)[8]) {
  u32x4 a, b;
  asm volatile("ds_read_b128 %0, %1" : "=v"(a) : "v"(addr));
  asm volatile("ds_read_b128 %0, %1 offset:16" : "=v"(b) : "v"(addr));
  lds_wait_tie<0>(a, b);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    v[i] = __uint_as_float(a[i]);
    v[4 + i] = __uint_as_float(b[i]);
  }
}

template <typename T, bool H_OUT>
__global__ void __launch_bounds__(64 * SW) mlp_s1_kernel(S1Args A) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  S1Lds& L = *reinterpret_cast<S1Lds*>(smem_raw);
  const int tid = threadIdx.x, lane = tid & 63, hh = lane >> 5, tl = lane & 31;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const long M = A.M;
  const long ntiles = (M + STT - 1) / STT;
  const int G = gridDim.x;
  const long first = blockIdx.x;
  if (first >= ntiles) return;
  const long mine = (ntiles - 1 - first) / G + 1;
  const long nchunks = mine * NCH;

  for (int s = tid; s < SH; s += 64 * SW) L.b1[s] = A.b1[s];
  for (int s = tid; s < SC; s += 64 * SW) L.b2[s] = A.b2[s];
  __syncthreads();  // before any LDS-DMA is in flight (this barrier drains nothing)

  // chunk q (0 .. 23) of the weights into ring slot `slot`: this wave's 3 of the 24 1-KB DMA
  // instructions (W1 rows permuted by pi and chunk-swizzled; W2 columns chunk-swizzled)
  auto dma_chunk = [&](int q, int slot) __attribute__((always_inline)) {
    bf16_t* base = L.ring + slot * SLOT;
    const int ln = opaque(lane);
#pragma unroll
    for (int r = 0; r < DMA_PER_WAVE; ++r) {
      const int i = wave + SW * r;  // instruction 0 .. 23 (wave-uniform)
      if (i < 12) {
        const int p = 64 * i + ln, rho = p / 24, pos = p - (p / 24) * 24;
        const int gc = pos ^ ((rho >> 1) & 7);
        glds16(A.w1 + (long)(SCH * q + s1_pi(rho)) * SC + 8 * gc, base + 512 * i);
      } else {
        const int p = 64 * (i - 12) + ln, row = p >> 2, pos = p & 3;
        const int gc = pos ^ ((row >> 2) & 3);
        glds16(A.w2 + (long)row * SH + SCH * q + 8 * gc, base + W1S + 512 * (i - 12));
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
  // chunk's DMA (a queue of SNS - 1: the chunk waited for next first): the vmcnt waits let every
  // younger op stay in flight.  Stores are counted only when the whole wave issues them (full
  // tile rows): an uncounted op only makes a wait stricter.
  int issued = 0;
  int mark[SNS - 1];
  long tile = first;
  load_x(tile);
  issued += 12;
  int mark_x = issued;
#pragma unroll
  for (int s = 0; s < SNS - 1; ++s) {
    if (s < nchunks) {
      dma_chunk(s % NCH, s);
      issued += DMA_PER_WAVE;
    }
    mark[s] = issued;
  }

  f32x16 yacc[6];
#pragma unroll
  for (int ct = 0; ct < 6; ++ct) yacc[ct] = f32x16{0};
  // untracked-read lane addresses (bytes) within a slot
  const uint32_t ring0 = lds_u32(L.ring);
  const uint32_t a1_lane = (uint32_t)(tl * SC * 2);              // + slot, + 16 * pos(ks)
  const int w1sw = (tl >> 1) & 7;
  const uint32_t a2_lane = (uint32_t)(W1S * 2 + tl * SCH * 2);   // + slot, + 2048 ct, + 16 * pos(s)
  const int w2sw = (tl >> 2) & 3;
  // bias reads (untracked: a visible ds_read would wait for the ring) -- lane offsets
  const uint32_t b1_lane = lds_u32(L.b1) + 4u * (uint32_t)(8 * hh);
  const uint32_t b2_lane = lds_u32(L.b2) + 4u * (uint32_t)(4 * hh);

  // chunk j: weights chunk q = j % 24 in slot j % SNS; the DMA issued at chunk j is chunk
  // j + SNS - 1 (weights qn, slot sn)
  int q = 0, slot = 0, qn = (SNS - 1) % NCH, sn = SNS - 1;
  for (long j = 0; j < nchunks; ++j) {
    // chunk j's DMA (every wave's share, after the barrier) has landed; every wave is done with
    // chunk j - 1's slot, which is refilled next
    {
      // steady state (full tiles, no tile boundary among the younger ops): a constant count
      constexpr int STEADY = (SNS - 2) * DMA_PER_WAVE + (H_OUT ? 2 * (SNS - 1) : 0);
      const int younger = issued - mark[0];
      if (younger >= STEADY) wait_vmcnt<STEADY>();
      else wait_vmcnt_le(younger);
    }
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
#pragma unroll
    for (int s = 0; s < SNS - 2; ++s) mark[s] = mark[s + 1];
    if (j + SNS - 1 < nchunks) {
      dma_chunk(qn, sn);
      issued += DMA_PER_WAVE;
    }
    mark[SNS - 2] = issued;
    qn = qn + 1 == NCH ? 0 : qn + 1;
    sn = sn + 1 == SNS ? 0 : sn + 1;
    if (q == 0) wait_vmcnt_le(issued - mark_x);  // the tile's x rows
    const long row0 = tile * STT + 32 * wave;
    const bool full = row0 + 32 <= M;
    // ---- fc1: C1^T[rho][t] for the chunk's 32 hidden units (slot rows rho)
    const uint32_t a1 = ring0 + (uint32_t)(slot * SLOT * 2) + a1_lane;
    f32x16 h = f32x16{0};
    bf16x8 wf[2];
    // fragment reads two k steps apart in flight: (2 ks + hh) ^ w1sw is the slot chunk
    auto addr1 = [&](int ks) { return a1 + 16u * (uint32_t)((2 * ks + hh) ^ w1sw); };
    wf[0] = ds_b128_untracked<0>(addr1(0));
    unroll_for<12>([&](auto KS) {
      constexpr int ks = decltype(KS)::value;
      if constexpr (ks + 1 < 12) {
        wf[(ks + 1) & 1] = ds_b128_untracked<0>(addr1(ks + 1));
        lds_wait_tie<1>(wf[ks & 1]);
      } else {
        lds_wait_tie<0>(wf[ks & 1]);
      }
      h = Fmt16<T>::mma32(wf[ks & 1], __builtin_bit_cast(bf16x8, xc[ks]), h);
    });
    if (q == NCH - 1 && tile + G < ntiles) {
      // the next tile's x rows: xc is free once the last chunk's fc1 has issued
      load_x(tile + G);
      issued += 12;
      mark_x = issued;
    }
    // ---- + b1, 16-bit H (stored), GELU, 16-bit GELU(H): registers 8s + e <-> hidden
    // 32 q + 16 s + 8 hh + e
    u32x4 g[2];
    const long hrow = row0 + tl;
    const bool hok = hrow < M;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      float bv[8];
      ds_f32x8_untracked(b1_lane + 4u * (uint32_t)(SCH * q + 16 * s), bv);
      float u[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) u[e] = round16<T>(h[8 * s + e] + bv[e]);
      if constexpr (H_OUT) {
        const u32x4 hv = {pack2<T>(u[0], u[1]), pack2<T>(u[2], u[3]), pack2<T>(u[4], u[5]), pack2<T>(u[6], u[7])};
        if (hok) *reinterpret_cast<u32x4*>(A.hout + hrow * SH + SCH * q + 16 * s + 8 * hh) = hv;
      }
      g[s] = u32x4{pack2<T>(gelu_fast(u[0]), gelu_fast(u[1])), pack2<T>(gelu_fast(u[2]), gelu_fast(u[3])),
                   pack2<T>(gelu_fast(u[4]), gelu_fast(u[5])), pack2<T>(gelu_fast(u[6]), gelu_fast(u[7]))};
    }
    if (H_OUT && full) issued += 2;
    // ---- fc2: y^T[c][t] += W2[c][chunk] . GELU(H)^T, six 32-channel tiles, two 16-deep k steps
    const uint32_t a2 = ring0 + (uint32_t)(slot * SLOT * 2) + a2_lane;
    auto addr2 = [&](int ct, int s) { return a2 + 2048u * (uint32_t)ct + 16u * (uint32_t)((2 * s + hh) ^ w2sw); };
    bf16x8 af[2];
    af[0] = ds_b128_untracked<0>(addr2(0, 0));
    unroll_for<12>([&](auto I) {
      constexpr int i = decltype(I)::value, s = i / 6, ct = i % 6;
      if constexpr (i + 1 < 12) {
        af[(i + 1) & 1] = ds_b128_untracked<0>(addr2((i + 1) % 6, (i + 1) / 6));
        lds_wait_tie<1>(af[i & 1]);
      } else {
        lds_wait_tie<0>(af[i & 1]);
      }
      yacc[ct] = Fmt16<T>::mma32(af[i & 1], __builtin_bit_cast(bf16x8, g[s]), yacc[ct]);
    });
    const bool tile_end = q == NCH - 1;
    q = tile_end ? 0 : q + 1;
    slot = slot + 1 == SNS ? 0 : slot + 1;
    if (!tile_end) continue;
    // ---- tile epilogue: y = y^T + b2; lane (token tl) holds channels 32 ct + 8 r4 + 4 hh + i in
    // register 4 r4 + i; a permlane32 swap pairs the halves into 8 consecutive channels per lane
    const long row = row0 + tl;
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
    if (full) issued += 12;
    tile += G;
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
