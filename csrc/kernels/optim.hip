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
// Mixed form (rt_grad_sumsq_mixed / rt_adamw_mixed, full-parameter training of a bf16 model,
// ops.MixedFlatParams): elements [0, n16) read bf16 gradients and rewrite the bf16 compute copy
// in the same pass; elements [n16, n) (fp32 parameters: the value head) read fp32 gradients.
// 4 elements per lane (16-B master / moment accesses); every segment boundary is a multiple of 16
// elements, so a group of 4 never straddles the bf16 / fp32 seam.
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
  float lr, b1, b2, eps, wd;
  int step;  // optimizer calls so far (this one included); bias correction uses step - *skipped
  float max_norm;
  const float* partials; int nparts;
  float* norm_out; int* skipped;
  // mixed form: g16 = bf16 gradients of elements [0, n16), g = fp32 gradients of [n16, n) indexed
  // from n16; pbf (if given) covers [0, npbf). Plain form: g16 = nullptr, n16 = 0, npbf = n.
  const bf16_t* g16; long n16; long npbf;
};

__global__ __launch_bounds__(256) void grad_sumsq_mixed_kernel(const bf16_t* __restrict__ g16, long n16,
                                                               const float* __restrict__ g32, long n32,
                                                               float* __restrict__ partials) {
  __shared__ float sb[4];
  float s = 0.f;
  const long stride = (long)gridDim.x * 256, t = (long)blockIdx.x * 256 + threadIdx.x;
  for (long i = t; i < n16 / 8; i += stride) {  // n16 % 8 == 0 (checked by the binding)
    float f[8];
    unpack8(((const uint4*)g16)[i], f);
#pragma unroll
    for (int k = 0; k < 8; ++k) s += f[k] * f[k];
  }
  for (long i = t; i < n32; i += stride) s += g32[i] * g32[i];
  s = block_sum(s, sb);
  if (threadIdx.x == 0) partials[blockIdx.x] = s;
}

__device__ __forceinline__ void adam_elem(const AdamArgs& a, float gr, float& pp, float& mm, float& vv, float decay,
                                          float step_scale, float inv_bc2_sqrt) {
  mm = a.b1 * mm + (1.f - a.b1) * gr;
  vv = a.b2 * vv + (1.f - a.b2) * gr * gr;
  pp = pp * decay;
  pp -= step_scale * mm / (sqrtf(vv) * inv_bc2_sqrt + a.eps);
}

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
  // applied steps = calls - skipped (non-finite) calls, read on the device so a skip decided by an
  // earlier launch never desynchronises the bias correction from the host's call counter
  const float tstep = (float)(a.step - (a.skipped ? *a.skipped : 0));
  const float bc1 = 1.f - powf(a.b1, tstep), bc2 = 1.f - powf(a.b2, tstep);
  const float step_scale = a.lr / bc1;
  const float inv_bc2_sqrt = rsqrtf(bc2);
  const long stride = (long)gridDim.x * 256, t = (long)blockIdx.x * 256 + threadIdx.x;
  const long n4 = a.n / 4;
  for (long q = t; q < n4; q += stride) {
    const long i = q * 4;
    float g[4];
    if (i < a.n16) {
      const uint2 w = ((const uint2*)a.g16)[q];
      g[0] = __uint_as_float(w.x << 16); g[1] = __uint_as_float(w.x & 0xffff0000u);
      g[2] = __uint_as_float(w.y << 16); g[3] = __uint_as_float(w.y & 0xffff0000u);
    } else {
      const float4 w = *(const float4*)(a.g + (i - a.n16));
      g[0] = w.x; g[1] = w.y; g[2] = w.z; g[3] = w.w;
    }
    const float4 p4 = ((const float4*)a.p)[q], m4 = ((const float4*)a.m)[q], v4 = ((const float4*)a.v)[q];
    float P[4] = {p4.x, p4.y, p4.z, p4.w}, M[4] = {m4.x, m4.y, m4.z, m4.w}, V[4] = {v4.x, v4.y, v4.z, v4.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) adam_elem(a, g[k] * clip, P[k], M[k], V[k], decay, step_scale, inv_bc2_sqrt);
    ((float4*)a.p)[q] = make_float4(P[0], P[1], P[2], P[3]);
    ((float4*)a.m)[q] = make_float4(M[0], M[1], M[2], M[3]);
    ((float4*)a.v)[q] = make_float4(V[0], V[1], V[2], V[3]);
    if (i < a.npbf) ((uint2*)a.pbf)[q] = make_uint2(pack2bf(P[0], P[1]), pack2bf(P[2], P[3]));
  }
  for (long i = n4 * 4 + t; i < a.n; i += stride) {  // tail (n % 4 != 0)
    const float gr = (i < a.n16 ? bf2f(a.g16[i]) : a.g[i - a.n16]) * clip;
    float pp = a.p[i], mm = a.m[i], vv = a.v[i];
    adam_elem(a, gr, pp, mm, vv, decay, step_scale, inv_bc2_sqrt);
    a.p[i] = pp;
    a.m[i] = mm;
    a.v[i] = vv;
    if (i < a.npbf) a.pbf[i] = f2bf(pp);
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
                        float eps, float wd, int step, float max_norm, const float* partials, int nparts,
                        float* norm_out, int* skipped, hipStream_t stream) {
  AdamArgs a{p, g, m, v, (bf16_t*)pbf, n, lr, b1, b2, eps, wd, step, max_norm, partials, nparts, norm_out, skipped,
             nullptr, 0, pbf ? n : 0};
  long blocks = (n + 255) / 256;
  if (blocks > 2048) blocks = 2048;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(adamw_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, a);
  RT_LAUNCH_CHECK();
  return 0;
}

extern "C" int rt_grad_sumsq_mixed(const void* g16, long n16, const float* g32, long n32, float* partials, int nparts,
                                   hipStream_t stream) {
  if (nparts > OPT_NBLK || nparts <= 0 || n16 % 8) return -1;
  hipLaunchKernelGGL(grad_sumsq_mixed_kernel, dim3(nparts), dim3(256), 0, stream, (const bf16_t*)g16, n16, g32, n32,
                     partials);
  RT_LAUNCH_CHECK();
  return 0;
}

extern "C" int rt_adamw_mixed(float* p, const void* g16, long n16, const float* g32, float* m, float* v, void* p16,
                              long n, float lr, float b1, float b2, float eps, float wd, int step,
                              float max_norm, const float* partials, int nparts, float* norm_out, int* skipped,
                              hipStream_t stream) {
  if (n16 % 4 || n16 > n) return -1;
  AdamArgs a{p, g32, m, v, (bf16_t*)p16, n, lr, b1, b2, eps, wd, (int)step, max_norm, partials, nparts, norm_out, skipped,
             (const bf16_t*)g16, n16, n16};
  long blocks = (n / 4 + 255) / 256;
  if (blocks > 2048) blocks = 2048;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(adamw_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, a);
  RT_LAUNCH_CHECK();
  return 0;
}

// ---------------------------------------------------------------------------------------------
// Batched scaled scatter fp32 -> bf16 (LoRA compute images after an optimizer step): entry e of
// the int64 table [n, 7] = {src, src_ld, dst, dst_ld, rows, cols, bit pattern of the fp32 scale}
// writes dst[r * dst_ld + c] = bf16(src[r * src_ld + c] * scale). One launch rebuilds every
// adapter's A_pad (scaled A rows) and UB (B blocks at their column / rank offsets) of a model,
// instead of two torch copies (plus a scale) per adapter. blockIdx.y = entry.
namespace rt {
__global__ __launch_bounds__(256) void scatter_scaled_kernel(const long* __restrict__ tab) {
  const long* t = tab + (long)blockIdx.y * 7;
  const float* src = (const float*)t[0];
  bf16_t* dst = (bf16_t*)t[2];
  const long sld = t[1], dld = t[3], rows = t[4], cols = t[5];
  const float scale = __int_as_float((int)t[6]);
  const long n = rows * cols;
  for (long e = (long)blockIdx.x * 256 + threadIdx.x; e < n; e += (long)gridDim.x * 256) {
    const long r = e / cols, c = e - r * cols;
    dst[r * dld + c] = f2bf(src[r * sld + c] * scale);
  }
}

// LoRA backward epilogue: per descriptor (9 int64: src, src row stride, dst, dst row stride, rows,
// cols, fp32 scale bits, slabs, slab stride) dst[r][c] += scale * sum_s src[s][r][c], the split-K
// slabs of dA_all / dB_all summed in a fixed order (bitwise-reproducible gradients) straight into
// the parameters' .grad buffers. One blockIdx.y per descriptor.
__global__ __launch_bounds__(256) void lora_grad_accum_kernel(const long* __restrict__ tab) {
  const long* t = tab + (long)blockIdx.y * 9;
  const float* src = (const float*)t[0];
  float* dst = (float*)t[2];
  const long sld = t[1], dld = t[3], rows = t[4], cols = t[5];
  const float scale = __int_as_float((int)t[6]);
  const int ns = (int)t[7];
  const long sst = t[8];
  const long n = rows * cols;
  for (long e = (long)blockIdx.x * 256 + threadIdx.x; e < n; e += (long)gridDim.x * 256) {
    const long r = e / cols, c = e - r * cols;
    const float* sp = src + r * sld + c;
    float v = 0.f;
    for (int k = 0; k < ns; ++k) v += sp[(long)k * sst];
    dst[r * dld + c] += scale * v;
  }
}
}  // namespace rt

extern "C" int rt_lora_grad_accum(const long* tab, int n, long max_elems, hipStream_t stream) {
  if (n <= 0) return 0;
  if (n > 65535) return -1;
  long bx = (max_elems + 255) / 256;
  if (bx > 256) bx = 256;
  if (bx < 1) bx = 1;
  hipLaunchKernelGGL(lora_grad_accum_kernel, dim3((unsigned)bx, (unsigned)n), dim3(256), 0, stream, tab);
  RT_LAUNCH_CHECK();
  return 0;
}

extern "C" int rt_scatter_scaled(const long* tab, int n, long max_elems, hipStream_t stream) {
  if (n <= 0) return 0;
  if (n > 65535) return -1;
  long bx = (max_elems + 255) / 256;
  if (bx > 64) bx = 64;
  if (bx < 1) bx = 1;
  hipLaunchKernelGGL(scatter_scaled_kernel, dim3((unsigned)bx, (unsigned)n), dim3(256), 0, stream, tab);
  RT_LAUNCH_CHECK();
  return 0;
}
