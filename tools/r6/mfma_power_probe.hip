// MFMA-only throughput under register-resident random operands: v_mfma_f32_16x16x32_bf16 vs
// v_mfma_f32_32x32x16_bf16 at equal MACs, 8 waves per CU (2 per SIMD, the gemm_big shape). The
// GEMMs of the PPO step run at 1.9-2.0 GHz with random data (power-throttled, profiles/r5/
// gemm_clock_pmc.txt): this asks whether the 32x32 form sustains more FLOP/s at that power.
// Build: hipcc --offload-arch=gfx950 -O3 tools/r6/mfma_power_probe.hip -o /tmp/mfma_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(16))) float f32x16;

template <int SHAPE>
__global__ __launch_bounds__(512, 2) void probe(const unsigned* __restrict__ seed, int iters, float* out) {
  const int lane = threadIdx.x;
  bf16x8 a[4], b[4];
  unsigned s = seed[blockIdx.x * 512 + lane];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    unsigned short v[8];
    for (int e = 0; e < 8; ++e) {
      s = s * 1664525u + 1013904223u;
      // random bf16 in about [-2, 2): sign, exponent 126..128, random mantissa
      v[e] = (unsigned short)(((s >> 31) << 15) | ((126u + ((s >> 20) % 3u)) << 7) | ((s >> 8) & 0x7Fu));
    }
    a[i] = __builtin_bit_cast(bf16x8, *(const __attribute__((ext_vector_type(4))) unsigned*)v);
    s = s * 1664525u + 1013904223u;
    for (int e = 0; e < 8; ++e) {
      s = s * 1664525u + 1013904223u;
      v[e] = (unsigned short)(((s >> 31) << 15) | ((126u + ((s >> 20) % 3u)) << 7) | ((s >> 8) & 0x7Fu));
    }
    b[i] = __builtin_bit_cast(bf16x8, *(const __attribute__((ext_vector_type(4))) unsigned*)v);
  }
  if constexpr (SHAPE == 16) {
    f32x4 acc[8][4];
    for (int i = 0; i < 8; ++i)
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0, 0, 0, 0};
    // operand indices are compile-time (an it-dependent register-array index spills to scratch)
    for (int it = 0; it < iters; it += 4) {
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[(i + r) & 3], b[(j + r) & 3], acc[i][j], 0, 0, 0);
    }
    float t = 0;
    for (int i = 0; i < 8; ++i)
      for (int j = 0; j < 4; ++j) t += acc[i][j][0] + acc[i][j][3];
    out[blockIdx.x * 512 + lane] = t;
  } else {
    // same MACs per iteration: 32 x 16x16x32 = 262144 MACs = 16 x 32x32x16
    f32x16 acc[4][2];
    for (int i = 0; i < 4; ++i)
      for (int j = 0; j < 2; ++j)
        for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;
    for (int it = 0; it < iters; it += 4) {
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int kk = 0; kk < 2; ++kk)
#pragma unroll
          for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j)
              acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[(i + r + kk) & 3], b[(j + r + kk) & 3], acc[i][j], 0, 0, 0);
    }
    float t = 0;
    for (int i = 0; i < 4; ++i)
      for (int j = 0; j < 2; ++j) t += acc[i][j][0] + acc[i][j][15];
    out[blockIdx.x * 512 + lane] = t;
  }
}

int main() {
  const int nwg = 256 * 2, iters = 40000;
  unsigned* seed;
  float* out;
  hipMalloc(&seed, nwg * 512 * 4);
  hipMalloc(&out, nwg * 512 * 4);
  std::vector<unsigned> h(nwg * 512);
  for (size_t i = 0; i < h.size(); ++i) h[i] = 2654435761u * (unsigned)(i + 1);
  hipMemcpy(seed, h.data(), h.size() * 4, hipMemcpyHostToDevice);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const double flops = 2.0 * 262144.0 * 64.0 * iters * 8.0 * nwg;  // per-wave MACs x lanes-agnostic: see note
  for (int rep = 0; rep < 3; ++rep) {
    for (int shape : {16, 32}) {
      hipEventRecord(e0);
      if (shape == 16) hipLaunchKernelGGL(probe<16>, dim3(nwg), dim3(512), 0, 0, seed, iters, out);
      else hipLaunchKernelGGL(probe<32>, dim3(nwg), dim3(512), 0, 0, seed, iters, out);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      // MACs per wave per iteration = 262144 (32 MFMA 16x16x32 = 32 x 8192); waves = 8 x nwg
      const double f = 2.0 * 262144.0 * (double)iters * 8.0 * nwg;
      printf("shape %dx%d: %.2f ms  %.1f TFLOP/s\n", shape, shape, ms, f / (ms * 1e-3) / 1e12);
    }
  }
  (void)flops;
  return 0;
}
