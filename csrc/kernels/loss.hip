// Fused log-softmax -> token log-prob / entropy, forward and backward.
//
// PPO needs, per response token, log pi(a_t|s_t) (policy and frozen reference) and the policy
// entropy; SFT needs the cross-entropy of the target. All are one pass over a logits row with an
// online (max, sum e^x, sum e^x * x) triple, so the fp32 softmax is never materialised
// (the reference computes a scalar CE through HF's full fp32 logits + log_softmax,
// reinforcement_learning_optimization_after_rag.py:200-204).
// Temperature: x' = x * inv_temp (PPO scores the same tempered distribution it sampled from).
#include "rt_common.h"

namespace rt {

template <typename T> __device__ __forceinline__ void load8(const T* p, float* f);
template <> __device__ __forceinline__ void load8<bf16_t>(const bf16_t* p, float* f) { unpack8(*(const uint4*)p, f); }
template <> __device__ __forceinline__ void load8<float>(const float* p, float* f) {
  const float4 a = *(const float4*)p, b = *(const float4*)(p + 4);
  f[0] = a.x; f[1] = a.y; f[2] = a.z; f[3] = a.w; f[4] = b.x; f[5] = b.y; f[6] = b.z; f[7] = b.w;
}
template <typename T> __device__ __forceinline__ float load1(const T* p);
template <> __device__ __forceinline__ float load1<bf16_t>(const bf16_t* p) { return bf2f(*p); }
template <> __device__ __forceinline__ float load1<float>(const float* p) { return *p; }

struct MST { float m, s, t; };

__device__ __forceinline__ MST mst_merge(MST a, MST b) {
  const float m = fmaxf(a.m, b.m);
  if (m == -INFINITY) return a;
  const float ea = __expf(a.m - m), eb = __expf(b.m - m);
  return MST{m, a.s * ea + b.s * eb, a.t * ea + b.t * eb};
}

template <typename T>
__global__ __launch_bounds__(256) void logprob_fwd_kernel(const T* __restrict__ logits, long ld,
                                                          const long* __restrict__ tgt, float inv_temp, int V,
                                                          float* __restrict__ logp, float* __restrict__ ent,
                                                          float* __restrict__ lse_out, float* __restrict__ ex_out) {
  __shared__ float sm[4][3];
  const long row = blockIdx.x;
  const T* x = logits + row * ld;
  MST a{-INFINITY, 0.f, 0.f};
  const int nv = V / 8;
  for (int c = threadIdx.x; c < nv; c += 256) {
    float f[8];
    load8<T>(x + c * 8, f);
    float mx = -INFINITY;
#pragma unroll
    for (int k = 0; k < 8; ++k) { f[k] *= inv_temp; mx = fmaxf(mx, f[k]); }
    const float m = fmaxf(a.m, mx);
    const float sc = __expf(a.m - m);
    float s = a.s * sc, t = a.t * sc;
#pragma unroll
    for (int k = 0; k < 8; ++k) { const float e = __expf(f[k] - m); s += e; t += e * f[k]; }
    a = MST{m, s, t};
  }
  for (int c = nv * 8 + threadIdx.x; c < V; c += 256) {  // tail
    const float f = load1<T>(x + c) * inv_temp;
    a = mst_merge(a, MST{f, 1.f, f});
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    MST o{__shfl_xor(a.m, off, 64), __shfl_xor(a.s, off, 64), __shfl_xor(a.t, off, 64)};
    a = mst_merge(a, o);
  }
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) { sm[wid][0] = a.m; sm[wid][1] = a.s; sm[wid][2] = a.t; }
  __syncthreads();
  if (threadIdx.x == 0) {
    MST r{sm[0][0], sm[0][1], sm[0][2]};
    for (int w = 1; w < 4; ++w) r = mst_merge(r, MST{sm[w][0], sm[w][1], sm[w][2]});
    const float lse = r.m + __logf(r.s);
    const float ex = r.t / r.s;  // E_p[x']
    const long tg = tgt ? tgt[row] : -1;
    if (logp) logp[row] = tg >= 0 ? load1<T>(x + tg) * inv_temp - lse : 0.f;
    if (ent) ent[row] = lse - ex;
    if (lse_out) lse_out[row] = lse;
    if (ex_out) ex_out[row] = ex;
  }
}

// dlogits = inv_temp * [ g_lp (onehot - p) - g_ent p (x' - E[x']) ]
template <typename T>
__global__ __launch_bounds__(256) void logprob_bwd_kernel(const T* __restrict__ logits, long ld,
                                                          const long* __restrict__ tgt, float inv_temp, int V,
                                                          const float* __restrict__ lse, const float* __restrict__ ex,
                                                          const float* __restrict__ g_lp, const float* __restrict__ g_ent,
                                                          bf16_t* __restrict__ dlogits, long ldd) {
  const long row = blockIdx.x;
  const T* x = logits + row * ld;
  bf16_t* dx = dlogits + row * ldd;
  const float L = lse[row], E = ex[row];
  const long tg = tgt ? tgt[row] : -1;
  const float gl = (g_lp && tg >= 0) ? g_lp[row] : 0.f;
  const float ge = g_ent ? g_ent[row] : 0.f;
  const int nv = V / 8;
  for (int c = threadIdx.x; c < nv; c += 256) {
    float f[8], o[8];
    load8<T>(x + c * 8, f);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const float xs = f[k] * inv_temp;
      const float p = __expf(xs - L);
      const float oh = (c * 8 + k) == tg ? 1.f : 0.f;
      o[k] = inv_temp * (gl * (oh - p) - ge * p * (xs - E));
    }
    *(uint4*)(dx + c * 8) = pack8(o);
  }
  for (int c = nv * 8 + threadIdx.x; c < V; c += 256) {
    const float xs = load1<T>(x + c) * inv_temp;
    const float p = __expf(xs - L);
    const float oh = c == tg ? 1.f : 0.f;
    dx[c] = f2bf(inv_temp * (gl * (oh - p) - ge * p * (xs - E)));
  }
}

// Value head V(s) = w . h + b per row (rl.py:150 nn.Linear(H, 1)): one wave per row, a
// fixed per-lane order over 16-B chunks and a fixed butterfly, so a row's value does not depend on
// how many rows the launch holds (torch's last-dim reduction picks its block split from the row
// count: the PPO scoring forward must give bitwise the same value at minibatch 32 and 128).
__global__ __launch_bounds__(256) void rowdot_kernel(const bf16_t* __restrict__ h, long ldh, const float* __restrict__ w,
                                                     const float* __restrict__ bias, int H, long T,
                                                     float* __restrict__ out) {
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= T) return;
  const bf16_t* x = h + row * ldh;
  float acc = 0.f;
  const int nv = H / 8;
  for (int c = lane; c < nv; c += 64) {
    float f[8];
    unpack8(*(const uint4*)(x + c * 8), f);
    const float4 a = *(const float4*)(w + c * 8), b = *(const float4*)(w + c * 8 + 4);
    acc = fmaf(f[0], a.x, acc); acc = fmaf(f[1], a.y, acc); acc = fmaf(f[2], a.z, acc); acc = fmaf(f[3], a.w, acc);
    acc = fmaf(f[4], b.x, acc); acc = fmaf(f[5], b.y, acc); acc = fmaf(f[6], b.z, acc); acc = fmaf(f[7], b.w, acc);
  }
  for (int c = nv * 8 + lane; c < H; c += 64) acc = fmaf(bf2f(x[c]), w[c], acc);
  acc = wave_sum(acc);
  if (lane == 0) out[row] = acc + (bias ? bias[0] : 0.f);
}

}  // namespace rt

using namespace rt;

extern "C" int rt_logprob_fwd(const void* logits, int is_f32, long ld, const long* tgt, float inv_temp, long T, int V,
                              float* logp, float* ent, float* lse, float* ex, hipStream_t stream) {
  if (T == 0) return 0;
  if (is_f32)
    hipLaunchKernelGGL(logprob_fwd_kernel<float>, dim3(T), dim3(256), 0, stream, (const float*)logits, ld, tgt,
                       inv_temp, V, logp, ent, lse, ex);
  else
    hipLaunchKernelGGL(logprob_fwd_kernel<bf16_t>, dim3(T), dim3(256), 0, stream, (const bf16_t*)logits, ld, tgt,
                       inv_temp, V, logp, ent, lse, ex);
  RT_LAUNCH_CHECK();
  return 0;
}

extern "C" int rt_logprob_bwd(const void* logits, int is_f32, long ld, const long* tgt, float inv_temp, long T, int V,
                              const float* lse, const float* ex, const float* g_lp, const float* g_ent, void* dlogits,
                              long ldd, hipStream_t stream) {
  if (T == 0) return 0;
  if (is_f32)
    hipLaunchKernelGGL(logprob_bwd_kernel<float>, dim3(T), dim3(256), 0, stream, (const float*)logits, ld, tgt,
                       inv_temp, V, lse, ex, g_lp, g_ent, (bf16_t*)dlogits, ldd);
  else
    hipLaunchKernelGGL(logprob_bwd_kernel<bf16_t>, dim3(T), dim3(256), 0, stream, (const bf16_t*)logits, ld, tgt,
                       inv_temp, V, lse, ex, g_lp, g_ent, (bf16_t*)dlogits, ldd);
  RT_LAUNCH_CHECK();
  return 0;
}

extern "C" int rt_rowdot(const void* h, long ldh, const float* w, const float* bias, int H, long T, float* out,
                         hipStream_t stream) {
  if (T == 0) return 0;
  if (ldh % 8) return -1;
  hipLaunchKernelGGL(rowdot_kernel, dim3((unsigned)((T + 3) / 4)), dim3(256), 0, stream, (const bf16_t*)h, ldh, w, bias,
                     H, T, out);
  RT_LAUNCH_CHECK();
  return 0;
}
