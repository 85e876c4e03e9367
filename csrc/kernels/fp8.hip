// fp8 (OCP e4m3fn, gfx950) quantisation: per-row absmax scaling.
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

// One 256-thread workgroup per row with the whole row in registers (up to 8 16-B chunks per
// thread, C <= 16384): every load of a row is issued before the absmax (one memory round trip
// instead of 2 x C / 512 dependent ones), and M rows fill M CUs — the per-row quantisation of the
// W8A8 decode inputs (M = 256, C = 5120 / 13824). Same arithmetic as quant_fp8_rows_kernel.
__global__ __launch_bounds__(256) void quant_fp8_rows_reg_kernel(const bf16_t* __restrict__ x, long ldx,
                                                                 unsigned char* __restrict__ q, long ldq,
                                                                 float* __restrict__ scale, int C) {
  constexpr int MAXK = 8;
  __shared__ float red[4];
  const long row = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int nch = C / 8;
  const bf16_t* xr = x + row * ldx;
  uint4 v[MAXK];
#pragma unroll
  for (int k = 0; k < MAXK; ++k) {
    const int c = tid + k * 256;
    v[k] = c < nch ? *(const uint4*)(xr + c * 8) : make_uint4(0, 0, 0, 0);
  }
  float amax = 0.f;
#pragma unroll
  for (int k = 0; k < MAXK; ++k) {
    float f[8];
    unpack8(v[k], f);
#pragma unroll
    for (int e = 0; e < 8; ++e) amax = fmaxf(amax, fabsf(f[e]));
  }
  amax = wave_max(amax);
  if (lane == 0) red[wid] = amax;
  __syncthreads();
  amax = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  const float s = amax > 0.f ? amax / 448.f : 1.f;
  const float inv = 1.f / s;
  unsigned char* qr = q + row * ldq;
#pragma unroll
  for (int k = 0; k < MAXK; ++k) {
    const int c = tid + k * 256;
    if (c < nch) {
      float f[8];
      unpack8(v[k], f);
      unsigned lo = 0, hi = 0;
      lo = __builtin_amdgcn_cvt_pk_fp8_f32(f[0] * inv, f[1] * inv, lo, false);
      lo = __builtin_amdgcn_cvt_pk_fp8_f32(f[2] * inv, f[3] * inv, lo, true);
      hi = __builtin_amdgcn_cvt_pk_fp8_f32(f[4] * inv, f[5] * inv, hi, false);
      hi = __builtin_amdgcn_cvt_pk_fp8_f32(f[6] * inv, f[7] * inv, hi, true);
      *(uint2*)(qr + c * 8) = make_uint2(lo, hi);
    }
  }
  if (tid == 0) scale[row] = s;
}

}  // namespace rt

using namespace rt;

extern "C" int rt_quant_fp8_rows(const void* x, long ldx, void* q, long ldq, float* scale, long R, int C,
                                 hipStream_t stream) {
  if (R <= 0) return 0;
  if (C % 8) return -1;
  // one workgroup per row with the row in registers (decode inputs: 5.1 vs 18.5 us at 256 x 5120;
  // training forwards: 9632 rows); rows wider than 16384: one wave per row
  if (C <= 16384 && (ldx % 8) == 0 && (ldq % 8) == 0)
    hipLaunchKernelGGL(quant_fp8_rows_reg_kernel, dim3((unsigned)R), dim3(256), 0, stream, (const bf16_t*)x, ldx,
                       (unsigned char*)q, ldq, scale, C);
  else
    hipLaunchKernelGGL(quant_fp8_rows_kernel, dim3((R + 3) / 4), dim3(256), 0, stream, (const bf16_t*)x, ldx,
                       (unsigned char*)q, ldq, scale, R, C);
  RT_LAUNCH_CHECK();
  return 0;
}
