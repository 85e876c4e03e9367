// RL kernels: token-level GAE reverse scan, and the decode-step bookkeeping kernel
// that keeps a hipGraph-captured generation loop free of host round trips.
//
// GAE follows reinforcement_learning_optimization_after_rag.py:176-191 (delta = r + g*V' - V,
// A = delta + g*lam*A') but over the tokens of each response instead of across batch samples, with
// lam a parameter (reference hard-codes 0.95) and padding tokens masked out.
#include "rt_common.h"

namespace rt {

__global__ void gae_kernel(const float* __restrict__ rewards, const float* __restrict__ values,
                           const float* __restrict__ mask, int B, int T, float gamma, float lam,
                           float* __restrict__ adv, float* __restrict__ ret) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  float nextv = 0.f, last = 0.f;
  for (int t = T - 1; t >= 0; --t) {
    const long i = (long)b * T + t;
    if (mask[i] == 0.f) {
      adv[i] = 0.f;
      ret[i] = 0.f;
      continue;
    }
    const float v = values[i];
    const float delta = rewards[i] + gamma * nextv - v;
    last = delta + gamma * lam * last;
    adv[i] = last;
    ret[i] = last + v;
    nextv = v;
  }
}

// After sampling token `tok[b]` at decode step `step`: record it, update finished flags (eos or
// length budget), advance per-row cache length/position, bump the RNG offset and step counter.
// Rows that are finished keep emitting pad and stop advancing.
__global__ void decode_update_kernel(const long* __restrict__ tok, long* __restrict__ out_tokens, int max_new,
                                     float* __restrict__ out_logp, const float* __restrict__ logp,
                                     float* __restrict__ out_values, const float* __restrict__ values,
                                     uint8_t* __restrict__ active, int* __restrict__ kv_len, int* __restrict__ pos,
                                     long* __restrict__ next_input, int* __restrict__ gen_len,
                                     int64_t* __restrict__ step, int64_t* __restrict__ rng_offset, int B,
                                     const long* __restrict__ eos_ids, int n_eos, long pad_id) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t s = *step;
  if (b < B) {
    const bool act = active[b] != 0;
    long t = tok[b];
    if (act && s < max_new) {
      out_tokens[(long)b * max_new + s] = t;
      if (out_logp) out_logp[(long)b * max_new + s] = logp[b];
      if (out_values && values) out_values[(long)b * max_new + s] = values[b];
      gen_len[b] = (int)s + 1;
      bool fin = (s + 1 >= max_new);
      for (int e = 0; e < n_eos; ++e) fin = fin || (t == eos_ids[e]);
      if (fin) active[b] = 0;
      kv_len[b] += 1;
      pos[b] += 1;
      next_input[b] = t;
    } else {
      next_input[b] = pad_id;
    }
  }
  __syncthreads();
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    *step = s + 1;
    *rng_offset = *rng_offset + 1;
  }
}

}  // namespace rt

using namespace rt;

extern "C" int rt_gae(const float* rewards, const float* values, const float* mask, int B, int T, float gamma, float lam,
                      float* adv, float* ret, hipStream_t stream) {
  if (B == 0) return 0;
  hipLaunchKernelGGL(gae_kernel, dim3((B + 63) / 64), dim3(64), 0, stream, rewards, values, mask, B, T, gamma, lam, adv,
                     ret);
  RT_LAUNCH_CHECK();
  return 0;
}

extern "C" int rt_decode_update(const long* tok, long* out_tokens, int max_new, float* out_logp, const float* logp,
                                float* out_values, const float* values, uint8_t* active, int* kv_len, int* pos,
                                long* next_input, int* gen_len, int64_t* step, int64_t* rng_offset, int B,
                                const long* eos_ids, int n_eos, long pad_id, hipStream_t stream) {
  if (B > 1024) return -1;
  hipLaunchKernelGGL(decode_update_kernel, dim3(1), dim3(((B + 63) / 64) * 64), 0, stream, tok, out_tokens, max_new,
                     out_logp, logp, out_values, values, active, kv_len, pos, next_input, gen_len, step, rng_offset, B,
                     eos_ids, n_eos, pad_id);
  RT_LAUNCH_CHECK();
  return 0;
}
