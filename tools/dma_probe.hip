// Ingest-rate probe: LDS-DMA (global_load_lds_dwordx4) vs register staging (global_load_dwordx4 +
// ds_write_b128) into LDS, every CU at once, from an L2-resident region or a streamed HBM buffer.
// Tells whether the LDS-DMA path caps a CU's operand rate below what the GEMM kernels need.
//   hipcc --offload-arch=gfx950 -O3 -shared -fPIC tools/dma_probe.hip -o tools/exp/libdma_probe.so
//   python tools/dma_probe.py
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(1))) void glb_void;

// each block: `iters` rounds of PER 16-B pieces per thread (PER * 256 * 16 B = 32 KB per round
// at PER = 8) into a 64 KB LDS ring; `mask` wraps the source offset (region size - 1)
template <int PER, bool DMA>
__global__ void __launch_bounds__(256) probe(const unsigned char* __restrict__ src, unsigned long long mask, int iters,
                                             unsigned* sink) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  const int tid = threadIdx.x;
  unsigned long long off = ((unsigned long long)blockIdx.x * 32768ull) & mask;
  u32x4 acc = {0, 0, 0, 0};
  for (int it = 0; it < iters; ++it) {
    const int ring = (it & 1) * 32768;
    if constexpr (DMA) {
#pragma unroll
      for (int p = 0; p < PER; ++p) {
        const unsigned long long o = (off + (unsigned long long)(p * 256 + tid) * 16ull) & mask;
        __builtin_amdgcn_global_load_lds((glb_void*)(src + o), (lds_void*)(lds + ring + p * 4096 + (tid & ~63) * 16),
                                         16, 0, 0);
      }
      __builtin_amdgcn_s_waitcnt(0);  // vmcnt(0) expcnt(0) lgkmcnt(0)
    } else {
      u32x4 v[PER];
#pragma unroll
      for (int p = 0; p < PER; ++p) {
        const unsigned long long o = (off + (unsigned long long)(p * 256 + tid) * 16ull) & mask;
        v[p] = *reinterpret_cast<const u32x4*>(src + o);
      }
#pragma unroll
      for (int p = 0; p < PER; ++p) *reinterpret_cast<u32x4*>(lds + ring + (p * 256 + tid) * 16) = v[p];
    }
    __builtin_amdgcn_s_barrier();
    acc += *reinterpret_cast<const u32x4*>(lds + ring + ((tid * 16 + it * 64) & 32767));
    off = (off + 32768ull * gridDim.x) & mask;
  }
  if (acc[0] == 0x12345678u && acc[1] == 0x9abcdef0u) sink[blockIdx.x] = acc[2];
}

extern "C" int dma_probe(int dma, const void* src, unsigned long long mask, int iters, int blocks, void* sink,
                         void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (dma)
    hipLaunchKernelGGL((probe<8, true>), dim3(blocks), dim3(256), 65536, st, (const unsigned char*)src, mask, iters,
                       (unsigned*)sink);
  else
    hipLaunchKernelGGL((probe<8, false>), dim3(blocks), dim3(256), 65536, st, (const unsigned char*)src, mask, iters,
                       (unsigned*)sink);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
