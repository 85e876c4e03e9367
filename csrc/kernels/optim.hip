// Fused AdamW with on-device global grad-norm clipping and non-finite skip.
//
// The trainer keeps every trainable parameter in ONE flat fp32 buffer (params are views into it;
// likewise grads / exp_avg / exp_avg_sq), so "multi-tensor" is a single grid-stride launch, the
// DP all-reduce is a few large contiguous buckets, and nothing is synchronised with the host:
//   1. rt_grad_sumsq : per-workgroup partial sum of g^2 -> partials[nblk]
//   2. rt_adamw      : every workgroup reduces the partials itself (<= 1024 floats), derives
//                      norm, clip coefficient (torch clip_grad_norm_: max_norm / (norm + 1e-6),
//                      capped at 1) and a skip flag when the norm is non-finite, then applies
//                      torch.optim.AdamW semantics (decoupled weight decay, bias correction) and
//                      optionally refreshes a bf16 shadow copy used by the MFMA kernels.
// Replaces clip_grad_norm_ + AdamW.step of reinforcement_learning_optimization_after_rag.py:230-232.
#include "rt_common.h"

namespace rt {

constexpr int OPT_NBLK = 1024;

__global__ __launch_bounds__(256) void grad_sumsq_kernel(const float* __restrict__ g, long n, float* __restrict__ partials) {
  __shared__ float sb[4];
  float s = 0.f;
  const long n4 = n / 4;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n4; i += (long)gridDim.x * 256) {
    const float4 v = ((const float4*)g)[i];
    s += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
  }
  for (long i = n4 * 4 + (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) s += g[i] * g[i];
  s = block_sum(s, sb);
  if (threadIdx.x == 0) partials[blockIdx.x] = s;
}

struct AdamArgs {
  float* p; const float* g; float* m; float* v; bf16_t* pbf; long n;
  float lr, b1, b2, eps, wd, bc1, bc2, max_norm;
  const float* partials; int nparts;
  float* norm_out; int* skipped;
};

__global__ __launch_bounds__(256) void adamw_kernel(AdamArgs a) {
  __shared__ float sb[4];
  float s = 0.f;
  for (int i = threadIdx.x; i < a.nparts; i += 256) s += a.partials[i];
  const float tot = block_sum(s, sb);
  const float norm = sqrtf(tot);
  if (!isfinite(norm)) {
    if (blockIdx.x == 0 && threadIdx.x == 0) {
      if (a.skipped) atomicAdd(a.skipped, 1);
      if (a.norm_out) *a.norm_out = norm;
    }
    return;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0 && a.norm_out) *a.norm_out = norm;
  const float clip = a.max_norm > 0.f ? fminf(1.f, a.max_norm / (norm + 1e-6f)) : 1.f;
  const float decay = 1.f - a.lr * a.wd;
  const float step_scale = a.lr / a.bc1;
  const float inv_bc2_sqrt = rsqrtf(a.bc2);
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < a.n; i += (long)gridDim.x * 256) {
    const float gr = a.g[i] * clip;
    float mm = a.m[i], vv = a.v[i], pp = a.p[i];
    mm = a.b1 * mm + (1.f - a.b1) * gr;
    vv = a.b2 * vv + (1.f - a.b2) * gr * gr;
    pp = pp * decay;
    pp -= step_scale * mm / (sqrtf(vv) * inv_bc2_sqrt + a.eps);
    a.m[i] = mm;
    a.v[i] = vv;
    a.p[i] = pp;
    if (a.pbf) a.pbf[i] = f2bf(pp);
  }
}

}  // namespace rt

using namespace rt;

extern "C" int rt_grad_sumsq(const float* g, long n, float* partials, int nparts, hipStream_t stream) {
  if (nparts > OPT_NBLK || nparts <= 0) return -1;
  hipLaunchKernelGGL(grad_sumsq_kernel, dim3(nparts), dim3(256), 0, stream, g, n, partials);
  RT_LAUNCH_CHECK();
  return 0;
}

extern "C" int rt_adamw(float* p, const float* g, float* m, float* v, void* pbf, long n, float lr, float b1, float b2,
                        float eps, float wd, float bc1, float bc2, float max_norm, const float* partials, int nparts,
                        float* norm_out, int* skipped, hipStream_t stream) {
  AdamArgs a{p, g, m, v, (bf16_t*)pbf, n, lr, b1, b2, eps, wd, bc1, bc2, max_norm, partials, nparts, norm_out, skipped};
  long blocks = (n + 255) / 256;
  if (blocks > 2048) blocks = 2048;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(adamw_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, a);
  RT_LAUNCH_CHECK();
  return 0;
}
