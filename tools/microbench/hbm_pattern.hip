// HBM read-pattern microbenchmark (MI355X): does the per-row contiguous span of a weight-streaming
// GEMV matter? Streams a bf16 matrix [R x K] once, three ways, and reports TB/s:
//   A: a wave covers 16 rows x 128 B per step (the decode GEMM's MFMA fragment pattern)
//   B: a wave covers  2 rows x 512 B per step (64 lanes x 16 B, 32 lanes per row)
//   C: a wave covers  1 row  x 1 KiB per step (64 lanes x 16 B contiguous)
// Each lane keeps `DEPTH` 16-B loads in flight; results are xor-reduced so nothing is elided.
// Build: hipcc --offload-arch=gfx950 -O3 -o /tmp/hbm_pattern tools/microbench/hbm_pattern.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef __attribute__((ext_vector_type(4))) unsigned u32x4;
constexpr int DEPTH = 8;

template <int MODE>
__global__ __launch_bounds__(256) void stream_kernel(const char* __restrict__ w, long R, long K2, int rows_per_block,
                                                      unsigned* __restrict__ out) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const long r0 = (long)blockIdx.x * rows_per_block;
  unsigned acc = 0;
  // per-wave row group and in-row offset of this lane for one step
  int rows_per_step, lane_row, lane_off, step_bytes;
  if (MODE == 0) { rows_per_step = 16; lane_row = lane & 15; lane_off = (lane >> 4) * 16; step_bytes = 64; }
  else if (MODE == 1) { rows_per_step = 2; lane_row = lane >> 5; lane_off = (lane & 31) * 16; step_bytes = 512; }
  else { rows_per_step = 1; lane_row = 0; lane_off = lane * 16; step_bytes = 1024; }
  // MODE 0 covers 128 B per row per step with two loads (lane_off, lane_off + 64)
  const int loads_per_step = MODE == 0 ? 2 : 1;
  const int waves_rows = rows_per_block / 4;  // rows owned by this wave
  const long wrow0 = r0 + wid * waves_rows;
  for (int rg = 0; rg < waves_rows; rg += rows_per_step) {
    const char* rowp = w + (wrow0 + rg + lane_row) * K2;
    const int span = MODE == 0 ? 128 : step_bytes;
    const int nsteps = (int)(K2 / span);
    for (int s = 0; s < nsteps; s += DEPTH) {
      u32x4 v[DEPTH][2];
#pragma unroll
      for (int d = 0; d < DEPTH; ++d) {
        const char* p = rowp + (long)(s + d) * span + lane_off;
        v[d][0] = __builtin_nontemporal_load((const u32x4*)p);
        if (loads_per_step == 2) v[d][1] = __builtin_nontemporal_load((const u32x4*)(p + 64));
      }
#pragma unroll
      for (int d = 0; d < DEPTH; ++d) {
        acc ^= v[d][0].x ^ v[d][0].w;
        if (loads_per_step == 2) acc ^= v[d][1].y;
      }
    }
  }
  if (acc == 0x12345678u) out[0] = acc;
}

int main() {
  const long R = 131072, K = 4096, K2 = K * 2;  // 1 GiB of bf16
  char* w;
  unsigned* out;
  hipMalloc(&w, R * K2);
  hipMalloc(&out, 4);
  hipMemset(w, 1, R * K2);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int rpb : {64, 128, 256}) {
    for (int mode = 0; mode < 3; ++mode) {
      const int blocks = (int)(R / rpb);
      auto launch = [&]() {
        if (mode == 0) hipLaunchKernelGGL(stream_kernel<0>, dim3(blocks), dim3(256), 0, 0, w, R, K2, rpb, out);
        if (mode == 1) hipLaunchKernelGGL(stream_kernel<1>, dim3(blocks), dim3(256), 0, 0, w, R, K2, rpb, out);
        if (mode == 2) hipLaunchKernelGGL(stream_kernel<2>, dim3(blocks), dim3(256), 0, 0, w, R, K2, rpb, out);
      };
      launch();
      hipDeviceSynchronize();
      hipEventRecord(a);
      for (int i = 0; i < 5; ++i) launch();
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      printf("{\"mode\": \"%c\", \"rows_per_block\": %d, \"blocks\": %d, \"tbs\": %.2f}\n", 'A' + mode, rpb, blocks,
             R * K2 * 5 / (ms * 1e-3) / 1e12);
    }
  }
  hipFree(w);
  return 0;
}
