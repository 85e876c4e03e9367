// fp8 (OCP e4m3fn, gfx950) quantisation: per-row absmax scaling, one wave per row.
//   scale[r] = max(|x[r,:]|) / 448 (448 = e4m3fn max finite), q[r,c] = x[r,c] / scale[r]
// Used for frozen weights (per output channel, once per adapter update) and for activations
// (per token, before every W8A8 GEMM) on the config-5 fp8 path.
#include "rt_common.h"

namespace rt {

__global__ __launch_bounds__(256) void quant_fp8_rows_kernel(const bf16_t* __restrict__ x, long ldx,
                                                             unsigned char* __restrict__ q, long ldq,
                                                             float* __restrict__ scale, long R, int C) {
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= R) return;
  const bf16_t* xr = x + row * ldx;
  float amax = 0.f;
  for (int c = lane * 8; c < C; c += 512) {
    float v[8];
    unpack8(*(const uint4*)(xr + c), v);
#pragma unroll
    for (int k = 0; k < 8; ++k) amax = fmaxf(amax, fabsf(v[k]));
  }
  amax = wave_max(amax);
  const float s = amax > 0.f ? amax / 448.f : 1.f;
  const float inv = 1.f / s;
  unsigned char* qr = q + row * ldq;
  for (int c = lane * 8; c < C; c += 512) {
    float v[8];
    unpack8(*(const uint4*)(xr + c), v);
    unsigned lo = 0, hi = 0;
    lo = __builtin_amdgcn_cvt_pk_fp8_f32(v[0] * inv, v[1] * inv, lo, false);
    lo = __builtin_amdgcn_cvt_pk_fp8_f32(v[2] * inv, v[3] * inv, lo, true);
    hi = __builtin_amdgcn_cvt_pk_fp8_f32(v[4] * inv, v[5] * inv, hi, false);
    hi = __builtin_amdgcn_cvt_pk_fp8_f32(v[6] * inv, v[7] * inv, hi, true);
    *(uint2*)(qr + c) = make_uint2(lo, hi);
  }
  if (lane == 0) scale[row] = s;
}

}  // namespace rt

using namespace rt;

extern "C" int rt_quant_fp8_rows(const void* x, long ldx, void* q, long ldq, float* scale, long R, int C,
                                 hipStream_t stream) {
  if (R <= 0) return 0;
  if (C % 8) return -1;
  hipLaunchKernelGGL(quant_fp8_rows_kernel, dim3((R + 3) / 4), dim3(256), 0, stream, (const bf16_t*)x, ldx,
                     (unsigned char*)q, ldq, scale, R, C);
  RT_LAUNCH_CHECK();
  return 0;
}
