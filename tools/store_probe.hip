// Global-store shape probe: HBM write rate of 16-B-per-lane stores by the row footprint of one
// wave instruction (the GEMM / conv epilogues write 16 rows x 64 B per instruction), over a
// row-major [rows][row_bytes] buffer.  Build: hipcc --offload-arch=gfx950 -O3 tools/store_probe.hip
// -o /tmp/store_probe; run: /tmp/store_probe [row_bytes]
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// SEGS: rows touched per wave instruction (64 lanes x 16 B = 1 KB split into SEGS runs of 1024 / SEGS B)
template <int SEGS>
__global__ void __launch_bounds__(256) store_kernel(char* out, long rows, int row_bytes, long insts_per_wave) {
  constexpr int LPS = 64 / SEGS;  // lanes per run
  const int lane = threadIdx.x & 63;
  const long wave = ((long)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const long nwaves = ((long)gridDim.x * blockDim.x) >> 6;
  const int seg = lane / LPS, pos = lane % LPS;
  const int runs_per_row = row_bytes / (16 * LPS);
  const u32x4 v = {(unsigned)lane, 1u, 2u, 3u};
  for (long i = 0; i < insts_per_wave; ++i) {
    const long inst = i * nwaves + wave;  // instruction index: SEGS rows x one run
    if (runs_per_row == 0) {  // runs longer than a row: the buffer as one contiguous range
      const long off = inst * 1024 + lane * 16;
      if (off < rows * row_bytes) *reinterpret_cast<u32x4*>(out + off) = v;
      continue;
    }
    const long rg = inst / runs_per_row, run = inst % runs_per_row;
    const long row = rg * SEGS + seg;
    if (row < rows) *reinterpret_cast<u32x4*>(out + row * row_bytes + run * 16 * LPS + pos * 16) = v;
  }
}

template <int SEGS>
float run(char* buf, long bytes, int row_bytes) {
  const long rows = bytes / row_bytes;
  const long insts = bytes / 1024;
  const int blocks = 256 * 8, threads = 256;
  const long nwaves = (long)blocks * threads / 64;
  const long ipw = (insts + nwaves - 1) / nwaves;
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  store_kernel<SEGS><<<blocks, threads>>>(buf, rows, row_bytes, ipw);
  hipEventRecord(a);
  for (int r = 0; r < 5; ++r) store_kernel<SEGS><<<blocks, threads>>>(buf, rows, row_bytes, ipw);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0;
  hipEventElapsedTime(&ms, a, b);
  return (float)(5.0 * bytes / (ms * 1e-3) / 1e9);
}

int main(int argc, char** argv) {
  const int row_bytes = argc > 1 ? atoi(argv[1]) : 768;
  const long bytes = 805306368L;  // the stage-0 fc1 dual output (2 x 524288 x 384 bf16)
  char* buf;
  if (hipMalloc(&buf, bytes) != hipSuccess) return 1;
  printf("row %d B: GB/s by rows per wave instruction (16 B per lane)\n", row_bytes);
  printf("  1 row  (1 KB run)   %.0f\n", run<1>(buf, bytes, row_bytes));
  printf("  2 rows (512 B runs) %.0f\n", run<2>(buf, bytes, row_bytes));
  printf("  4 rows (256 B runs) %.0f\n", run<4>(buf, bytes, row_bytes));
  printf("  8 rows (128 B runs) %.0f\n", run<8>(buf, bytes, row_bytes));
  printf(" 16 rows (64 B runs)  %.0f\n", run<16>(buf, bytes, row_bytes));
  printf(" 32 rows (32 B runs)  %.0f\n", run<32>(buf, bytes, row_bytes));
  hipFree(buf);
  return 0;
}
