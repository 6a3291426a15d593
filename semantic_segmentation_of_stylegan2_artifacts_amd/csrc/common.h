// Shared device helpers for the MS-UNet gfx950 kernels.
// Activations are f32 (parity mode), bf16 (training mode) or f16 (the reference's
// torch.amp.autocast(float16), trainer.py:308); every reduction and every normalisation
// statistic is computed in f32.  The two 16-bit formats share every kernel: the storage is
// moved as raw 16-bit words (bf16x8 below is only a 16-byte operand container) and only the
// conversions and the MFMA opcode depend on the format (Fmt16<T>).
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <stdint.h>

#include <mutex>

#define MSU_DEV __device__ __forceinline__

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));  // register-resident 16-B chunk
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));  // a register pair (v_pk_*_f32 operands)
typedef uint16_t bf16_t;  // storage type of a bf16 activation
typedef _Float16 f16_t;   // storage type of an f16 activation
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

enum MsuDtype { MSU_F32 = 0, MSU_BF16 = 1, MSU_F16 = 2 };

// ------------------------------------------------------------------ scalar conversion
MSU_DEV float to_f32(float v) { return v; }
MSU_DEV float to_f32(bf16_t v) { return __uint_as_float(((uint32_t)v) << 16); }
template <typename T> MSU_DEV T from_f32(float v);
template <> MSU_DEV float from_f32<float>(float v) { return v; }
template <> MSU_DEV bf16_t from_f32<bf16_t>(float v) {
  __hip_bfloat16 h = __float2bfloat16(v);  // v_cvt_pk_bf16_f32 (RNE, NaN-preserving)
  return *reinterpret_cast<bf16_t*>(&h);
}

MSU_DEV float to_f32(f16_t v) { return (float)v; }
template <> MSU_DEV f16_t from_f32<f16_t>(float v) { return (f16_t)v; }  // v_cvt_f16_f32 (RNE)

// ------------------------------------------------------------------ 16-bit formats
// Raw-word view of a 16-bit activation format: encode / decode through a uint32 word pair and
// the matching MFMA opcodes on 8-element operands held in a bf16x8 container.
template <typename T> struct Fmt16;
template <> struct Fmt16<bf16_t> {
  static MSU_DEV uint32_t bits(float v) { return (uint32_t)from_f32<bf16_t>(v); }
  static MSU_DEV float lo(uint32_t w) { return __uint_as_float(w << 16); }
  static MSU_DEV float hi(uint32_t w) { return __uint_as_float(w & 0xffff0000u); }
  static MSU_DEV f32x16 mma32(bf16x8 a, bf16x8 b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
  }
  static MSU_DEV f32x4 mma16(bf16x8 a, bf16x8 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
  }
};
template <> struct Fmt16<f16_t> {
  static MSU_DEV uint32_t bits(float v) { return (uint32_t)__builtin_bit_cast(uint16_t, (f16_t)v); }
  static MSU_DEV float lo(uint32_t w) { return (float)__builtin_bit_cast(f16_t, (uint16_t)(w & 0xffffu)); }
  static MSU_DEV float hi(uint32_t w) { return (float)__builtin_bit_cast(f16_t, (uint16_t)(w >> 16)); }
  static MSU_DEV f32x16 mma32(bf16x8 a, bf16x8 b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c,
                                                  0, 0, 0);
  }
  static MSU_DEV f32x4 mma16(bf16x8 a, bf16x8 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c,
                                                  0, 0, 0);
  }
};
// two values -> one packed 32-bit word (lo in bits 0-15)
template <typename T> MSU_DEV uint32_t pack2(float lo, float hi) {
  return Fmt16<T>::bits(lo) | (Fmt16<T>::bits(hi) << 16);
}
// the 16-bit word of a stored value (for hi/lo splits: bits of from_f32<T>(v))
template <typename T> MSU_DEV float round16(float v) { return to_f32(from_f32<T>(v)); }
// a bf16x8 container of eight constants
template <typename T> MSU_DEV bf16x8 splat8(float a0, float a1, float rest) {
  u32x4 w = {pack2<T>(a0, a1), pack2<T>(rest, rest), pack2<T>(rest, rest), pack2<T>(rest, rest)};
  return __builtin_bit_cast(bf16x8, w);
}

// ------------------------------------------------------------------ 4-wide vector I/O
// f32: one 16-B load; bf16: one 8-B load.
template <typename T> struct Vec4;
template <> struct Vec4<float> {
  static MSU_DEV void load(const float* p, float (&v)[4]) {
    float4 q = *reinterpret_cast<const float4*>(p);
    v[0] = q.x; v[1] = q.y; v[2] = q.z; v[3] = q.w;
  }
  static MSU_DEV void store(float* p, const float (&v)[4]) {
    *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
  }
};
template <> struct Vec4<bf16_t> {
  static MSU_DEV void load(const bf16_t* p, float (&v)[4]) {
    uint2 q = *reinterpret_cast<const uint2*>(p);
    v[0] = __uint_as_float(q.x << 16); v[1] = __uint_as_float(q.x & 0xffff0000u);
    v[2] = __uint_as_float(q.y << 16); v[3] = __uint_as_float(q.y & 0xffff0000u);
  }
  static MSU_DEV void store(bf16_t* p, const float (&v)[4]) {
    uint2 q;
    q.x = (uint32_t)from_f32<bf16_t>(v[0]) | ((uint32_t)from_f32<bf16_t>(v[1]) << 16);
    q.y = (uint32_t)from_f32<bf16_t>(v[2]) | ((uint32_t)from_f32<bf16_t>(v[3]) << 16);
    *reinterpret_cast<uint2*>(p) = q;
  }
};

template <> struct Vec4<f16_t> {
  static MSU_DEV void load(const f16_t* p, float (&v)[4]) {
    uint2 q = *reinterpret_cast<const uint2*>(p);
    v[0] = Fmt16<f16_t>::lo(q.x); v[1] = Fmt16<f16_t>::hi(q.x);
    v[2] = Fmt16<f16_t>::lo(q.y); v[3] = Fmt16<f16_t>::hi(q.y);
  }
  static MSU_DEV void store(f16_t* p, const float (&v)[4]) {
    uint2 q;
    q.x = pack2<f16_t>(v[0], v[1]);
    q.y = pack2<f16_t>(v[2], v[3]);
    *reinterpret_cast<uint2*>(p) = q;
  }
};

// ------------------------------------------------------------------ reductions
template <int W> MSU_DEV float group_sum(float v) {
#pragma unroll
  for (int o = W / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
template <int W> MSU_DEV float group_max(float v) {
#pragma unroll
  for (int o = W / 2; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// ------------------------------------------------------------------ activations
MSU_DEV float gelu_f(float x) { return 0.5f * x * (1.0f + erff(x * 0.70710678118654752f)); }
MSU_DEV float gelu_grad_f(float x) {
  const float cdf = 0.5f * (1.0f + erff(x * 0.70710678118654752f));
  const float pdf = 0.39894228040143268f * __expf(-0.5f * x * x);
  return cdf + x * pdf;
}

// bf16-path GELU: erf by Abramowitz & Stegun 7.1.26 (|error| <= 1.5e-7, far below the bf16
// rounding of every consumer), one v_rcp + one v_exp; gelu' reuses the same exponential.
MSU_DEV float erf_fast(float x, float& e_neg_x2) {
  const float ax = fabsf(x);
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, ax, 1.0f));
  const float p = fmaf(fmaf(fmaf(fmaf(1.061405429f, t, -1.453152027f), t, 1.421413741f), t, -0.284496736f), t,
                       0.254829592f) * t;
  e_neg_x2 = __expf(-ax * ax);
  return copysignf(fmaf(-p, e_neg_x2, 1.0f), x);
}
MSU_DEV float gelu_fast(float x) {
  float e;
  return 0.5f * x * (1.0f + erf_fast(x * 0.70710678118654752f, e));
}
MSU_DEV float gelu_grad_fast(float x) {
  float e;  // e = exp(-x^2 / 2)
  const float cdf = 0.5f * (1.0f + erf_fast(x * 0.70710678118654752f, e));
  return fmaf(x * 0.39894228040143268f, e, cdf);
}

// The same on a register pair: every multiply / fma / add of erf_fast as one v_pk_*_f32 (the same
// IEEE operations in the same order: bitwise equal to two scalar calls); the v_rcp / v_exp and the
// sign copies stay per element.  For the VALU-bound fused MLPs (the epilogues of the GEMMs and
// convs are store-bound: packed there measured neutral, r05ai).
MSU_DEV f32x2 pk_fma(f32x2 a, f32x2 b, f32x2 c) { return __builtin_elementwise_fma(a, b, c); }
MSU_DEV f32x2 splat2(float v) { return f32x2{v, v}; }
MSU_DEV f32x2 erf_fast2(f32x2 x, f32x2& e_neg_x2) {
  const f32x2 ax = {fabsf(x.x), fabsf(x.y)};
  const f32x2 d = pk_fma(splat2(0.3275911f), ax, splat2(1.0f));
  const f32x2 t = {__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y)};
  f32x2 p = pk_fma(splat2(1.061405429f), t, splat2(-1.453152027f));
  p = pk_fma(p, t, splat2(1.421413741f));
  p = pk_fma(p, t, splat2(-0.284496736f));
  p = pk_fma(p, t, splat2(0.254829592f)) * t;
  const f32x2 q = -ax * ax;
  e_neg_x2 = f32x2{__expf(q.x), __expf(q.y)};
  const f32x2 r = pk_fma(-p, e_neg_x2, splat2(1.0f));
  return f32x2{copysignf(r.x, x.x), copysignf(r.y, x.y)};
}
MSU_DEV f32x2 gelu_fast2(f32x2 x) {
  f32x2 e;
  return splat2(0.5f) * x * (splat2(1.0f) + erf_fast2(x * splat2(0.70710678118654752f), e));
}

// ------------------------------------------------------------------ counter-based RNG
// Philox-free 32-bit hash (splitmix-style) of (seed, index): uniform in [0, 1).
MSU_DEV float hash_uniform(uint64_t seed, uint64_t idx) {
  uint64_t z = seed + 0x9E3779B97F4A7C15ull * (idx + 1);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  return (float)(uint32_t)(z >> 40) * (1.0f / 16777216.0f);
}

// Dropout seed of a launch: the host seed, mixed with a device-resident per-step counter when
// one is given (seed_dev: a HIP-graph replay draws fresh masks without a host round trip).
MSU_DEV uint64_t launch_seed(uint64_t seed, const unsigned long long* seed_dev) {
  if (seed_dev == nullptr) return seed;
  uint64_t z = seed ^ ((uint64_t)seed_dev[0] * 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 31)) * 0xBF58476D1CE4E5B9ull;
  return z ^ (z >> 29);
}

// Dropout masks of window attention.  The 64 x 64 keep decisions of an item (window, head) come
// from 2 x 64 short streams, one per (query row i, key half hh): a murmur3 fmix32 hash of
// (seed, item, i, hh) seeds a xorshift32 + Weyl generator (xorwow-style, the generator cuRAND
// long used for dropout) whose 16 words hold the key pairs of that half -- word n covers keys
// j0, j0 + 1 with j0 = 32 (n >> 3) + crow(2 (n & 7), hh) (crow: the 32x32 MFMA accumulator row
// order, so a lane's bits line up with its score registers).  Each 16-bit half is compared with
// ceil(p 2^16): keep probability 1 - ceil(p 2^16) / 2^16, within 2^-16 of 1 - p.  One hash and
// 16 multiply-free steps per stream instead of a 3-multiply hash per key pair.
MSU_DEV uint32_t fmix32_hash(uint32_t seed, uint32_t idx) {
  uint32_t x = idx * 0x9E3779B9u + seed;
  x ^= x >> 16; x *= 0x85EBCA6Bu;
  x ^= x >> 13; x *= 0xC2B2AE35u;
  return x ^ (x >> 16);
}
MSU_DEV uint32_t drop_thresh16(float p) { return (uint32_t)ceilf(p * 65536.0f); }
MSU_DEV uint32_t drop_seed32(uint64_t seed) { return (uint32_t)seed ^ (uint32_t)(seed >> 32); }
// stream state of (item = window * nh + head, query i, key half hh); x != 0
struct DropStream {
  uint32_t x, d;
};
MSU_DEV DropStream drop_stream(uint32_t seed, uint32_t item, int i, int hh) {
  const uint32_t h = fmix32_hash(seed, (item * 64u + (uint32_t)i) * 2u + (uint32_t)hh);
  return DropStream{h | 1u, h};
}
// next word's keep bits: bit 0 <-> key j0, bit 1 <-> key j0 + 1
MSU_DEV uint32_t drop_next2(DropStream& s, uint32_t thr) {
  s.x ^= s.x << 13;
  s.x ^= s.x >> 17;
  s.x ^= s.x << 5;
  s.d += 362437u;
  const uint32_t w = s.x + s.d;
  return (uint32_t)((w & 0xFFFFu) >= thr) | ((uint32_t)((w >> 16) >= thr) << 1);
}
// keep decision of one (query i, key j) pair of an item (the f32 kernels: one element at a time)
MSU_DEV bool drop_keep_bit(uint32_t seed, uint32_t item, int i, int j, uint32_t thr) {
  const int jt = j >> 5, jj = j & 31;
  const int hh = (jj >> 2) & 1, r = (jj & 3) + 4 * (jj >> 3);  // j = 32 jt + crow(r, hh)
  const int n = jt * 8 + (r >> 1);
  DropStream s = drop_stream(seed, item, i, hh);
  uint32_t b = 0;
  for (int k = 0; k <= n; ++k) b = drop_next2(s, thr);
  return (b >> (r & 1)) & 1u;
}

// XCD-aware bijective block remap: blocks b and b+8 share an XCD under round-robin
// dispatch; give each XCD group a contiguous range of work items (speed only).
MSU_DEV int xcd_remap(int b, int nb) {
  const int x = b & 7, local = b >> 3;
  const int q = nb >> 3, r = nb & 7;
  const int start = x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q;
  return start + local;
}

// opaque copy of a value: stops the compiler from hoisting per-chunk index math out of a
// persistent tile loop (it would keep ~5 registers per chunk live across the whole loop)
MSU_DEV int opaque(int v) {
  asm volatile("" : "+v"(v));
  return v;
}

// ------------------------------------------------------------------ LDS-DMA helpers
// global_load_lds_dwordx4: each lane's 16 B land at lds_base + 16 * lane (lds_base is
// wave-uniform); counted by vmcnt like any global load.
typedef __attribute__((address_space(3))) void msu_lds_void;
typedef __attribute__((address_space(1))) void msu_glb_void;
// (Issuing it as inline asm, invisible to hipcc's lgkmcnt tracking, measured neutral at two
// waves per SIMD: r04l, not kept.)
MSU_DEV void glds16(const void* src, void* lds_base) {
  __builtin_amdgcn_global_load_lds((msu_glb_void*)src, (msu_lds_void*)lds_base, 16, 0, 0);
}
// s_waitcnt vmcnt(N) only (gfx9 encoding: vmcnt[3:0], expcnt[6:4], lgkmcnt[11:8], vmcnt_hi[15:14])
template <int N> MSU_DEV void wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | 0x70 | 0xF00);
}
// Zero source for DMA slots that must read zeros (rows / pixels outside the tensor): 4 KB,
// addressed by slot so the requests spread over L2 channels instead of hammering one line.
// Pure pad slots should re-read a real address of the same row instead.
namespace {
__device__ __attribute__((aligned(16))) uint32_t g_zero_region[1024];
}
MSU_DEV const void* zero_src(int slot) { return g_zero_region + 4 * (slot & 255); }

#define MSU_CHECK_LAUNCH() (hipGetLastError() == hipSuccess ? 0 : -1)

// ------------------------------------------------------------------ tile queues
// Persistent kernels beside the side stream: a workgroup takes its first
// tile statically and claims the others from a device counter, so workgroups that get a CU late
// (the side stream's weight-gradient kernels hold whole CUs) take fewer tiles instead of running
// a fixed share past the others' end.  A slot = 8 claim counters (one per XCD, for kernels
// that keep each XCD on its own tile range; others use counter 0) and a finished-workgroup
// count, each on its own 128-B line; the launch's last workgroup resets the slot (no memset
// launch; graph-replay safe).  One slot per stream and translation unit.
namespace {
constexpr int TQ_SLOTS = 16, TQ_LINE = 32, TQ_DONE = 8 * TQ_LINE, TQ_INTS = 9 * TQ_LINE;
__device__ int g_tile_queue[TQ_SLOTS * TQ_INTS];

// claim k = 0, 1, ... of counter `line` (atomicInc: the add form goes through the atomic
// optimizer, whose lane arithmetic on the result makes the wave wait for it at once)
MSU_DEV int tq_claim(int* tq, int line) { return (int)atomicInc((unsigned*)tq + TQ_LINE * line, 0xffffffffu); }

// thread 0 of every workgroup once at its end: the last one out resets the slot
MSU_DEV void tq_finish(int* tq) {
  if (tq != nullptr && threadIdx.x == 0 && atomicInc((unsigned*)tq + TQ_DONE, 0xffffffffu) == gridDim.x - 1) {
#pragma unroll
    for (int i = 0; i <= 8; ++i) atomicExch(tq + TQ_LINE * i, 0);
  }
}

// the queue slot of stream `st`, or nullptr (the static schedule: more streams than slots)
inline int* tile_queue(hipStream_t st) {
  static std::mutex mu;
  static int* base = nullptr;
  static hipStream_t owner[TQ_SLOTS];
  static int used = 0;
  std::lock_guard<std::mutex> lock(mu);
  if (base == nullptr && hipGetSymbolAddress((void**)&base, HIP_SYMBOL(g_tile_queue)) != hipSuccess) {
    base = nullptr;
    return nullptr;
  }
  for (int i = 0; i < used; ++i)
    if (owner[i] == st) return base + TQ_INTS * i;
  if (used == TQ_SLOTS) return nullptr;
  owner[used] = st;
  return base + TQ_INTS * used++;
}
}  // namespace

// Run a statement with T bound to the storage type of `dtype` (f32 / bf16 / f16).
#define MSU_DISPATCH(dtype, T, ...)          \
  switch (dtype) {                           \
    case MSU_BF16: {                         \
      typedef bf16_t T;                      \
      __VA_ARGS__;                           \
    } break;                                 \
    case MSU_F16: {                          \
      typedef f16_t T;                       \
      __VA_ARGS__;                           \
    } break;                                 \
    default: {                               \
      typedef float T;                       \
      __VA_ARGS__;                           \
    }                                        \
  }
// the 16-bit formats only (f32 handled by the caller)
#define MSU_DISPATCH16(dtype, T, ...)        \
  switch (dtype) {                           \
    case MSU_F16: {                          \
      typedef f16_t T;                       \
      __VA_ARGS__;                           \
    } break;                                 \
    default: {                               \
      typedef bf16_t T;                      \
      __VA_ARGS__;                           \
    }                                        \
  }
inline bool msu_is16(int dtype) { return dtype == MSU_BF16 || dtype == MSU_F16; }

// Order stream `pst` after the work queued so far on `st` (an event; one per host thread,
// reused: each record captures the state at that moment).  pst == st or null: nothing.
// Lets an entry point put its parameter-gradient tail on the caller's side stream.
inline int attn_param_stream(hipStream_t st, hipStream_t& pst) {
  if (pst == nullptr || pst == st) {
    pst = st;
    return 0;
  }
  static thread_local hipEvent_t ev = nullptr;
  if (ev == nullptr && hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) return -1;
  if (hipEventRecord(ev, st) != hipSuccess) return -1;
  if (hipStreamWaitEvent(pst, ev, 0) != hipSuccess) return -1;
  return 0;
}
