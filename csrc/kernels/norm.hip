// Normalisation kernels: fused residual-add + RMSNorm (decoder) and fused
// residual-add + LayerNorm (encoders / OPT), forward and backward.
//
// Forward contract (both norms):
//   h = x (+ res)            -> written to h_out when res is given (the new residual stream)
//   y = norm(h) * w (+ b)    -> bf16
//   rstd (and mean for LN)   -> fp32 per row (saved for backward)
// One workgroup per row; the row lives in registers (16-B vectors, <= 8 per thread), so a row is
// read once and written once: the op runs at the HBM roofline. Reductions are wave64 shuffles
// followed by one LDS exchange.
#include "rt_common.h"

namespace rt {

constexpr int NORM_MAXV = 8;  // max 16-B vectors per thread -> H <= 256*8*8 = 16384

template <bool LAYERNORM, int NV, int MAXT = 512>
__global__ __launch_bounds__(MAXT) void norm_fwd_kernel(const bf16_t* __restrict__ x, const bf16_t* __restrict__ res,
                                                       const bf16_t* __restrict__ w, const bf16_t* __restrict__ b,
                                                       bf16_t* __restrict__ y, bf16_t* __restrict__ h_out,
                                                       float* __restrict__ rstd_out, float* __restrict__ mean_out,
                                                       int H, float eps, const float* __restrict__ xs, int nsplit,
                                                       long sstride) {
  // xs != null: x is the bf16-rounded sum of nsplit fp32 split-K slabs (stride sstride floats):
  // the split-K reduce of the producing GEMM fused into this pass (decode at batch 65..512)
  __shared__ float sbuf[16];  // <= 16 waves
  const long row = blockIdx.x;
  const int nv = H / 8;
  const bf16_t* xr = x + row * H;
  float v[NV][8];
  float s = 0.f;
  // weight (and bias) loads are issued with the row loads: one memory round trip before the
  // reduction instead of a second dependent one after it (decode rows are latency-bound)
  uint4 wraw[NV], braw[NV];
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = threadIdx.x + i * blockDim.x;
    if (c < nv) {
      wraw[i] = *(const uint4*)(w + c * 8);
      if (LAYERNORM && b) braw[i] = *(const uint4*)(b + c * 8);
    }
  }
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = threadIdx.x + i * blockDim.x;
    if (c < nv) {
      if (xs) {
        float t8[8];
        sum_slabs8(xs + row * H + c * 8, sstride, nsplit, t8);
#pragma unroll
        for (int k = 0; k < 8; ++k) v[i][k] = bf2f(f2bf(t8[k]));  // = the reduce kernel's bf16 output
      } else {
        unpack8(*(const uint4*)(xr + c * 8), v[i]);
      }
      if (res) {
        float r[8];
        unpack8(*(const uint4*)(res + row * H + c * 8), r);
#pragma unroll
        for (int k = 0; k < 8; ++k) v[i][k] += r[k];
        // the residual stream is kept in bf16: round before normalising so fwd == what bwd sees
#pragma unroll
        for (int k = 0; k < 8; ++k) v[i][k] = bf2f(f2bf(v[i][k]));
        *(uint4*)(h_out + row * H + c * 8) = pack8(v[i]);
      }
#pragma unroll
      for (int k = 0; k < 8; ++k) s += LAYERNORM ? v[i][k] : v[i][k] * v[i][k];
    }
  }
  float mean = 0.f, rstd;
  if (LAYERNORM) {
    mean = block_sum(s, sbuf) / H;
    float s2 = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int c = threadIdx.x + i * blockDim.x;
      if (c < nv)
#pragma unroll
        for (int k = 0; k < 8; ++k) { const float d = v[i][k] - mean; s2 += d * d; }
    }
    rstd = rsqrtf(block_sum(s2, sbuf) / H + eps);
  } else {
    rstd = rsqrtf(block_sum(s, sbuf) / H + eps);
  }
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = threadIdx.x + i * blockDim.x;
    if (c < nv) {
      float wv[8], bv[8], o[8];
      unpack8(wraw[i], wv);
      if (LAYERNORM && b) unpack8(braw[i], bv);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        o[k] = (v[i][k] - mean) * rstd * wv[k];
        if (LAYERNORM && b) o[k] += bv[k];
      }
      *(uint4*)(y + row * H + c * 8) = pack8(o);
    }
  }
  if (threadIdx.x == 0) {
    if (rstd_out) rstd_out[row] = rstd;
    if (LAYERNORM && mean_out) mean_out[row] = mean;
  }
}

// Backward. Each workgroup walks `rows_per_block` rows, accumulating dw (and db) in registers,
// then stores its partial as row blockIdx.x of the fp32 dw / db slabs [gridDim.x, H] (the caller
// sums the rows in a fixed order: no arrival-order atomics).
//   xhat = (h - mean) * rstd ; y = xhat*w (+b)
//   g = dy*w ; dh = rstd * (g - mean(g) [LN only] - xhat * mean(g*xhat))  (+ dh_res)
template <bool LAYERNORM, int NV>
__global__ __launch_bounds__(256) void norm_bwd_kernel(const bf16_t* __restrict__ dy, const bf16_t* __restrict__ h,
                                                       const bf16_t* __restrict__ w, const float* __restrict__ rstd_in,
                                                       const float* __restrict__ mean_in,
                                                       const bf16_t* __restrict__ dh_res, bf16_t* __restrict__ dh,
                                                       float* __restrict__ dw, float* __restrict__ db, int T, int H,
                                                       int rows_per_block) {
  __shared__ float sbuf[8];
  const int nv = H / 8;
  float dwacc[NV][8], dbacc[NV][8];
  float wv[NV][8];
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = threadIdx.x + i * blockDim.x;
#pragma unroll
    for (int k = 0; k < 8; ++k) { dwacc[i][k] = 0.f; dbacc[i][k] = 0.f; }
    if (c < nv) unpack8(*(const uint4*)(w + c * 8), wv[i]);
  }
  const long r0 = (long)blockIdx.x * rows_per_block;
  for (long row = r0; row < min((long)T, r0 + rows_per_block); ++row) {
    const float rstd = rstd_in[row];
    const float mean = LAYERNORM ? mean_in[row] : 0.f;
    float xh[NV][8], gg[NV][8];
    float s_g = 0.f, s_gx = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int c = threadIdx.x + i * blockDim.x;
      if (c < nv) {
        float hv[8], dv[8];
        unpack8(*(const uint4*)(h + row * H + c * 8), hv);
        unpack8(*(const uint4*)(dy + row * H + c * 8), dv);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          xh[i][k] = (hv[k] - mean) * rstd;
          gg[i][k] = dv[k] * wv[i][k];
          s_g += gg[i][k];
          s_gx += gg[i][k] * xh[i][k];
          dwacc[i][k] += dv[k] * xh[i][k];
          dbacc[i][k] += dv[k];
        }
      }
    }
    const float mg = LAYERNORM ? block_sum(s_g, sbuf) / H : 0.f;
    const float mgx = block_sum(s_gx, sbuf) / H;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int c = threadIdx.x + i * blockDim.x;
      if (c < nv) {
        float o[8], rr[8];
        if (dh_res) unpack8(*(const uint4*)(dh_res + row * H + c * 8), rr);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          o[k] = rstd * (gg[i][k] - mg - xh[i][k] * mgx);
          if (dh_res) o[k] += rr[k];
        }
        *(uint4*)(dh + row * H + c * 8) = pack8(o);
      }
    }
  }
  if (dw || db) {
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int c = threadIdx.x + i * blockDim.x;
      if (c < nv)
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          if (dw) dw[(long)blockIdx.x * H + c * 8 + k] = dwacc[i][k];
          if (LAYERNORM && db) db[(long)blockIdx.x * H + c * 8 + k] = dbacc[i][k];
        }
    }
  }
}

static void norm_geom(int H, int& threads, int& nvpt) {
  const int nv = H / 8;
  threads = nv >= 256 ? 256 : ((nv + 63) / 64) * 64;
  const int need = (nv + threads - 1) / threads;
  nvpt = need <= 1 ? 1 : need <= 2 ? 2 : need <= 4 ? 4 : 8;
}

}  // namespace rt

using namespace rt;

#define NORM_DISPATCH(LN, KER, ...)                                                              \
  switch (nvpt) {                                                                                \
    case 1: hipLaunchKernelGGL((KER<LN, 1>), __VA_ARGS__); break;                                 \
    case 2: hipLaunchKernelGGL((KER<LN, 2>), __VA_ARGS__); break;                                 \
    case 4: hipLaunchKernelGGL((KER<LN, 4>), __VA_ARGS__); break;                                 \
    default: hipLaunchKernelGGL((KER<LN, 8>), __VA_ARGS__); break;                                \
  }

extern "C" int rt_norm_fwd(int layernorm, const void* x, const void* res, const void* w, const void* b, void* y,
                           void* h_out, float* rstd, float* mean, int T, int H, float eps, const float* xs,
                           int nsplit, hipStream_t stream) {
  if (H % 8 != 0 || H > 256 * 8 * NORM_MAXV) return -1;
  if (T == 0) return 0;
  int threads, nvpt;
  norm_geom(H, threads, nvpt);
  // split-K slab reduce (decode at batch 65..512: one row per block, rows <= CUs): twice the waves
  // per row (one 8-element chunk per thread) keep twice the slab loads in flight per CU
  const int sl = tuning().norm_slab_threads;
  if (xs && sl >= 512 && H / 8 >= 512 && H / 8 <= 512) {
    threads = 512;
    nvpt = 1;
  }
  // H = 5120 (Llama-2-13B, config 5): one chunk per thread over 640 threads — the 256-thread form
  // sums three chunks' slabs one memory round trip after another (19.6 us per norm at batch 256)
  if (xs && sl >= 512 && H / 8 > 512 && H / 8 <= 1024) {
    const int t = (H / 8 + 63) / 64 * 64;
    if (layernorm)
      hipLaunchKernelGGL((norm_fwd_kernel<true, 1, 1024>), dim3(T), dim3(t), 0, stream, (const bf16_t*)x,
                         (const bf16_t*)res, (const bf16_t*)w, (const bf16_t*)b, (bf16_t*)y, (bf16_t*)h_out, rstd, mean,
                         H, eps, xs, nsplit, (long)T * H);
    else
      hipLaunchKernelGGL((norm_fwd_kernel<false, 1, 1024>), dim3(T), dim3(t), 0, stream, (const bf16_t*)x,
                         (const bf16_t*)res, (const bf16_t*)w, (const bf16_t*)b, (bf16_t*)y, (bf16_t*)h_out, rstd, mean,
                         H, eps, xs, nsplit, (long)T * H);
    RT_LAUNCH_CHECK();
    return 0;
  }
  if (layernorm) {
    NORM_DISPATCH(true, norm_fwd_kernel, dim3(T), dim3(threads), 0, stream, (const bf16_t*)x, (const bf16_t*)res,
                  (const bf16_t*)w, (const bf16_t*)b, (bf16_t*)y, (bf16_t*)h_out, rstd, mean, H, eps, xs, nsplit,
                  (long)T * H)
  } else {
    NORM_DISPATCH(false, norm_fwd_kernel, dim3(T), dim3(threads), 0, stream, (const bf16_t*)x, (const bf16_t*)res,
                  (const bf16_t*)w, (const bf16_t*)b, (bf16_t*)y, (bf16_t*)h_out, rstd, mean, H, eps, xs, nsplit,
                  (long)T * H)
  }
  RT_LAUNCH_CHECK();
  return 0;
}

// workgroups of rt_norm_bwd for T rows (= the rows of its dw / db partial slabs)
extern "C" int rt_norm_bwd_blocks(int T) {
  if (T <= 0) return 0;
  const int nblk = T < 1024 ? T : 1024;
  const int rpb = (T + nblk - 1) / nblk;
  return (T + rpb - 1) / rpb;
}

// dw / db (optional): fp32 [rt_norm_bwd_blocks(T), H] partial slabs, every row written
extern "C" int rt_norm_bwd(int layernorm, const void* dy, const void* h, const void* w, const float* rstd,
                           const float* mean, const void* dh_res, void* dh, float* dw, float* db, int T, int H,
                           hipStream_t stream) {
  if (H % 8 != 0 || H > 256 * 8 * NORM_MAXV) return -1;
  if (T == 0) return 0;
  int threads, nvpt;
  norm_geom(H, threads, nvpt);
  const int nblk = T < 1024 ? T : 1024;
  const int rpb = (T + nblk - 1) / nblk;
  const int grid = rt_norm_bwd_blocks(T);
  if (layernorm) {
    NORM_DISPATCH(true, norm_bwd_kernel, dim3(grid), dim3(threads), 0, stream, (const bf16_t*)dy, (const bf16_t*)h,
                  (const bf16_t*)w, rstd, mean, (const bf16_t*)dh_res, (bf16_t*)dh, dw, db, T, H, rpb)
  } else {
    NORM_DISPATCH(false, norm_bwd_kernel, dim3(grid), dim3(threads), 0, stream, (const bf16_t*)dy, (const bf16_t*)h,
                  (const bf16_t*)w, rstd, mean, (const bf16_t*)dh_res, (bf16_t*)dh, dw, db, T, H, rpb)
  }
  RT_LAUNCH_CHECK();
  return 0;
}
